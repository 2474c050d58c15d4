// fp64 dependent vs independent chains on one wave (lane 0 active), unrolled.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(double* out, unsigned long long* t, double seed) {
  double a = seed, b = seed + 1, c = seed + 2, d = seed + 3;
  unsigned long long t0, t1;
  if (threadIdx.x == 0) {
    asm volatile("" : "+v"(a));
    t0 = __builtin_amdgcn_s_memtime();
    asm volatile("" : "+v"(a));
#pragma unroll
    for (int i = 0; i < 256; i++) a = a * 1.0000001 + 0.5;
    asm volatile("" : "+v"(a));
    t1 = __builtin_amdgcn_s_memtime(); t[0] = t1 - t0; out[0] = a;
    a = seed;
    asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    t0 = __builtin_amdgcn_s_memtime();
    asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
#pragma unroll
    for (int i = 0; i < 256; i++) { a = a * 1.0000001 + 0.5; b = b * 1.0000001 + 0.5; c = c * 1.0000001 + 0.5; d = d * 1.0000001 + 0.5; }
    asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    t1 = __builtin_amdgcn_s_memtime(); t[1] = t1 - t0; out[1] = a + b + c + d;
    a = seed;
    asm volatile("" : "+v"(a));
    t0 = __builtin_amdgcn_s_memtime();
    asm volatile("" : "+v"(a));
#pragma unroll
    for (int i = 0; i < 256; i++) a = a + 1.0000001;
    asm volatile("" : "+v"(a));
    t1 = __builtin_amdgcn_s_memtime(); t[2] = t1 - t0; out[2] = a;
  }
}
int main() {
  double* o; unsigned long long* t;
  (void)hipMalloc(&o, 64 * 8); (void)hipMalloc(&t, 64 * 8);
  for (int rep = 0; rep < 3; rep++) { hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, o, t, 1.0); (void)hipDeviceSynchronize(); }
  unsigned long long h[8]; (void)hipMemcpy(h, t, 64, hipMemcpyDeviceToHost);
  printf("dependent mul+add (fp-contract off): %.2f cycles per op\n", h[0] / 512.0);
  printf("4 independent mul+add chains:        %.2f cycles per op\n", h[1] / 2048.0);
  printf("dependent add:                       %.2f cycles per op\n", h[2] / 256.0);
  return 0;
}
