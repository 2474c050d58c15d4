// Latency of the primitives on the physics' serial chains (one wave, gfx950):
// cycles per dependent step for
//   add     x = x + c                           (v_add_f64)
//   rl      x = x + readlane(x, 5)              (v_readlane x2 -> SGPR -> v_add_f64)
//   div     x = x / b, b = 1 + x*0 (IEEE, compiler sequence)
//   cnd     x = (x < c) ? x + c : x - c         (v_cmp -> v_cndmask x2 + add)
//   lds     x = lds[f(x)] + c                   (ds_write, ds_read round trip)
//   shfl    x = x + __shfl(x, 5)                (ds_bpermute)
//   dpp     x = x + row_shr:1(x)                (DPP mov)
// hipcc --offload-arch=gfx950 -O3 -ffp-contract=off lat3.hip -o lat3
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ double rlane(double x, int l) {
  long long b = __double_as_longlong(x);
  int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), l);
  int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

constexpr int N = 128;

__global__ void k(double* out, unsigned long long* t, double seed) {
  __shared__ double sh[64];
  const int lane = threadIdx.x;
  double x = seed + lane * 1e-9, c = 0.5 + 1e-9 * lane;
  unsigned long long t0, t1;
#define TIME(slot, body)                          \
  x = seed + lane * 1e-9;                         \
  asm volatile("" : "+v"(x), "+v"(c));            \
  t0 = __builtin_amdgcn_s_memtime();              \
  asm volatile("" : "+v"(x));                     \
  _Pragma("unroll") for (int i = 0; i < N; i++) { body; } \
  asm volatile("" : "+v"(x));                     \
  t1 = __builtin_amdgcn_s_memtime();              \
  if (lane == 0) t[slot] = t1 - t0;               \
  out[slot * 64 + lane] = x;
  TIME(0, x = x + c)
  TIME(1, x = x + rlane(x, 5))
  TIME(2, x = x / (1.0 + x * 1e-300))
  TIME(3, x = (x < c) ? x + c : x - c)
  TIME(4, sh[lane] = x; __builtin_amdgcn_wave_barrier(); x = sh[(lane + 1) & 63] + c; __builtin_amdgcn_wave_barrier())
  TIME(5, x = x + __shfl(x, 5))
  TIME(6, x = x + __longlong_as_double(((long long)__builtin_amdgcn_update_dpp(0, (int)(__double_as_longlong(x) >> 32), 0x111, 0xf, 0xf, false) << 32) | (unsigned)__builtin_amdgcn_update_dpp(0, (int)__double_as_longlong(x), 0x111, 0xf, 0xf, false)))
  TIME(7, x = x * c)
  TIME(8, x = __builtin_fma(x, c, c))
}

int main() {
  double* o;
  unsigned long long* t;
  (void)hipMalloc(&o, 16 * 64 * 8);
  (void)hipMalloc(&t, 16 * 8);
  const char* names[] = {"add", "readlane+add", "div (IEEE)", "cmp+cndmask+add", "lds store/load", "shfl (bpermute)+add",
                         "dpp+add", "mul", "fma"};
  for (int waves = 1; waves <= 2; waves++) {
    for (int rep = 0; rep < 3; rep++) {
      // waves = 2: a second wave on every SIMD of the CU (4 SIMDs x 2 = 8 blocks on one CU is not
      // guaranteed; launch 2 blocks per CU's worth over the chip) -- one block per CU first
      hipLaunchKernelGGL(k, dim3(256 * 4 * waves), dim3(64), 0, 0, o, t, 1.0);
      (void)hipDeviceSynchronize();
    }
    unsigned long long h[16];
    (void)hipMemcpy(h, t, sizeof(h), hipMemcpyDeviceToHost);
    printf("-- %d wave(s) per SIMD (approx.)\n", waves);
    for (int i = 0; i < 9; i++) printf("%-22s %6.2f cycles per dependent step\n", names[i], h[i] / (double)N);
  }
  return 0;
}
