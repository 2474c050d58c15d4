// Latency microbenchmarks on one wavefront (lane 0 active where noted):
// dependent fp64 add / mul / div / sqrt chains, LDS store->load round trip.
#include <hip/hip_runtime.h>
#include <cstdio>
#define N 256
__global__ void k(double* out, unsigned long long* t, double seed) {
  __shared__ double sh[256];
  sh[threadIdx.x] = seed + threadIdx.x;
  __syncthreads();
  double x = seed;
  unsigned long long t0, t1;
  if (threadIdx.x == 0) {
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; i++) x = x + 1.0000001;
    t1 = __builtin_amdgcn_s_memtime(); t[0] = t1 - t0; out[0] = x;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; i++) x = x * 1.0000001;
    t1 = __builtin_amdgcn_s_memtime(); t[1] = t1 - t0; out[1] = x;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; i++) x = 1.5 / x;
    t1 = __builtin_amdgcn_s_memtime(); t[2] = t1 - t0; out[2] = x;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; i++) x = sqrt(x + 1.0);
    t1 = __builtin_amdgcn_s_memtime(); t[3] = t1 - t0; out[3] = x;
    // LDS dependent chain: load -> add -> store to next slot
    volatile double* vs = sh;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; i++) vs[(i + 1) & 255] = vs[i & 255] + 1.0;
    t1 = __builtin_amdgcn_s_memtime(); t[4] = t1 - t0; out[4] = vs[7];
    // LDS pointer chase (int)
    int* si = (int*)sh;
    for (int i = 0; i < 256; i++) si[i] = (i * 7 + 3) & 255;
    volatile int* vi = si;
    int p = 0;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; i++) p = vi[p];
    t1 = __builtin_amdgcn_s_memtime(); t[5] = t1 - t0; out[5] = p;
    // s_memrealtime vs memtime calibration: spin 
    unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < 20000; i++) x = x + 1.0000001;
    t1 = __builtin_amdgcn_s_memtime();
    unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    t[6] = t1 - t0; t[7] = r1 - r0; out[6] = x;
  }
}
int main() {
  double* o; unsigned long long* t;
  hipMalloc(&o, 64 * 8); hipMalloc(&t, 64 * 8);
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, o, t, 1.0);
    hipDeviceSynchronize();
  }
  unsigned long long h[8]; hipMemcpy(h, t, 64, hipMemcpyDeviceToHost);
  const char* nm[] = {"f64 add", "f64 mul", "f64 div", "f64 sqrt+add", "lds st->ld chain", "lds int chase"};
  for (int i = 0; i < 6; i++) printf("%-18s %8.1f memtime-cycles/op\n", nm[i], h[i] / (double)N);
  printf("memtime per realtime tick (100MHz): %.2f  => memtime clock %.0f MHz\n", h[6] / (double)h[7], 100.0 * h[6] / h[7]);
  return 0;
}
