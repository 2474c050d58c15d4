// Compile-time model descriptions for model-specific physics kernels.
//
// The cooperative physics (dcoop.h) is written against a model "traits"
// object m: m.nv, m.body_parentid[i], m.body_pos[3*i], ...  The generic
// instantiation uses DevModel (runtime sizes, pointers into the LDS-staged
// image).  For the bundled models, tools/gen_static_models.py emits structs
// (static_models.h) whose sizes and integer tables are compile-time constants
// and whose float arrays are LDS pointers at compile-time offsets.  The same
// source then compiles to straight-line code: constant loop bounds (unrolled
// tree walks), constant LDS addresses the scheduler can disambiguate, no
// integer index arithmetic and no SGPR spills for model pointers.
//
// Integer tables are packed into 64-bit words so that a per-lane (divergent)
// index is a shift and a mask, not a memory access, and a uniform index folds
// to an immediate.  Only integer data is baked in: float data (masses,
// geometry, ...) stays runtime, so one specialisation serves every model with
// the same structure.  The host selects a specialisation by comparing the
// model's specialisation key (ilqg_model_static_key) with the generated one.
#pragma once

namespace ilqg {
namespace stat {

// N small integers in [-1, 2^BITS - 2], stored +1 in BITS-bit fields
template <int N, int BITS = 8>
struct PackedI {
  static constexpr int PER = 64 / BITS;
  static constexpr int NW = N > 0 ? (N + PER - 1) / PER : 1;
  unsigned long long w[NW];
  __host__ __device__ constexpr int operator[](int i) const {
    unsigned long long x = w[0];
    for (int k = 1; k < NW; k++)
      if ((i / PER) == k) x = w[k];
    return (int)((x >> ((i % PER) * BITS)) & ((1ull << BITS) - 1)) - 1;
  }
  __host__ __device__ constexpr explicit operator bool() const { return true; }
};

// N bits
template <int N>
struct PackedBits {
  static constexpr int NW = N > 0 ? (N + 63) / 64 : 1;
  unsigned long long w[NW];
  __host__ __device__ constexpr int operator[](int e) const {
    unsigned long long x = w[0];
    for (int k = 1; k < NW; k++)
      if ((e / 64) == k) x = w[k];
    return (int)((x >> (e % 64)) & 1ull);
  }
};

}  // namespace stat
}  // namespace ilqg
