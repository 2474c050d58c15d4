// In-launch hand-offs between workgroups (gfx950: 8 XCDs with private L2s,
// per-CU L1s never refreshed by other CUs' stores).
//
// Protocol (MI355X_MICROARCH.md "inter-workgroup visibility", Valid forms,
// first row): the producer stores every handed-off word write-through (sc1,
// an 8-byte relaxed agent-scope atomic store), drains them with
// s_waitcnt vmcnt(0), then ONE lane signals with an agent-scope atomic (a
// counter add or a flag store).  The consumer polls that word relaxed (sc1
// load, bounded, with s_sleep) and reads every handed-off word with sc1 loads
// (L1 bypassed).  Handed-off records are padded to whole 128-byte lines that
// nothing reads before they are published in the launch, so no stale copy of
// them can sit in any cache.  Every polled word is zeroed before each launch.
#pragma once
#include <hip/hip_runtime.h>

namespace ilqg {

typedef __attribute__((address_space(1))) unsigned gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;

// ~2^22 polls of >= 256 cycles: seconds, far beyond any legitimate wait; a
// timed-out wait gives up, so a broken producer can never hang the GPU.  The
// fault block is two words: fault[0] is the report (read and cleared by
// ilqg_synchronize), fault[1] the launch's own word (zeroed before every
// launch): a timed-out wait sets both, and every later wait of the same launch
// sees fault[1] and gives up at once, while the next launch waits normally.
__device__ __forceinline__ void raise_fault(unsigned* fault) {
  __hip_atomic_fetch_or((gu32*)(fault), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_fetch_or((gu32*)(fault + 1), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool launch_faulted(const unsigned* fault) {
  return __builtin_amdgcn_readfirstlane(
             __hip_atomic_load((gu32*)(fault + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) != 0u;
}
constexpr unsigned HANDOFF_SPIN_LIMIT = 1u << 22;

#ifdef ILQG_STAMPS
// diagnostic build: fused-sweep timeline (s_memtime ticks) -- [0] backward role 0
// cycles, [1] of which waiting for records, [2] waits that polled more than
// once, [3] role-0 start, [4] latest FD team end, [5] role-0 end, [8 + s] role s cycles
__device__ unsigned long long g_fused_diag[24];
// per-step completion time (s_memrealtime) of the backward roles of seeds
// 0..7 inside the fused sweep: [s * 512 + n] for step n < 512
__device__ unsigned long long g_bstep[8 * 512];
#define BSTEP_LOG(s, n)                                                                   \
  do {                                                                                     \
    if (done && tid == 0 && (s) < 8 && (n) < 512) g_bstep[(s) * 512 + (n)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define BSTEP_LOG(s, n) \
  do {                  \
  } while (0)
#endif

__device__ __forceinline__ double ld_sc1(const double* p) {
  return __longlong_as_double(
      (long long)__hip_atomic_load((gu64*)(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void st_sc1(double* p, double v) {
  __hip_atomic_store((gu64*)(p), (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int ld_sc1_i(const int* p) {
  return (int)__hip_atomic_load((gu32*)(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1_i(int* p, int v) {
  __hip_atomic_store((gu32*)(p), (unsigned)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// every storing wave, after its sc1 payload stores and before the signal
__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// wave-uniform: every lane polls the same word until it reaches `target`
__device__ inline bool bw_wait_geq(const unsigned* w, unsigned target, unsigned* fault) {
  for (unsigned spins = 0;; spins++) {
    // after one timed-out wait every later one gives up at once
    if ((spins & 255) == 255 && fault && launch_faulted(fault)) return false;
    const unsigned v = __builtin_amdgcn_readfirstlane(
        __hip_atomic_load((gu32*)(w), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    if (v >= target) break;
    if (spins > HANDOFF_SPIN_LIMIT) {
      if (fault && (threadIdx.x & 63) == 0) raise_fault(fault);
      return false;
    }
    __builtin_amdgcn_s_sleep(4);
  }
  // keep the payload's loads below the poll
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return true;
}

// wave-uniform: the first record of a window is awaited, and the window's
// later records are checked in the same poll (lane l reads flag p + l), so a
// consumer running behind its producer polls once per run of published records
// instead of once per record (an agent-scope load takes microseconds while a
// sweep loads the memory system).  Returns the last index q >= p with flags
// p..q all >= target (p on a timed-out wait, after setting *fault).
__device__ inline int bw_wait_window(const unsigned* flags, int p, int n, unsigned target, unsigned* fault) {
  const int lane = threadIdx.x & 63;
  for (unsigned spins = 0;; spins++) {
    if ((spins & 255) == 255 && fault && launch_faulted(fault)) return p;
    const int q = p + lane;
    const bool ok = q < n && __hip_atomic_load((gu32*)(flags + q), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target;
    const unsigned long long mask = __ballot(ok);
    if (mask & 1ull) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      return ~mask ? p + (int)__builtin_ctzll(~mask) - 1 : p + 63;
    }
    if (spins > HANDOFF_SPIN_LIMIT) {
      if (fault && lane == 0) raise_fault(fault);
      return p;
    }
    __builtin_amdgcn_s_sleep(4);
  }
}

// one lane signals for the (single-wave) team after drain_stores()
__device__ __forceinline__ void signal_add(unsigned* w) {
  __hip_atomic_fetch_add((gu32*)(w), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void signal_set(unsigned* w, unsigned v) {
  __hip_atomic_store((gu32*)(w), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace ilqg
