// Which SIMD does each wave of a three-wave workgroup land on?  The rollout
// runs one 192-lane workgroup (waves A, B, C) per (seed, candidate) with
// ~24 KB of LDS, 64 workgroups on 256 CUs; if two of its waves share a SIMD
// they split that SIMD's issue slots.  Each wave records HW_ID (gfx9 layout:
// wave slot [3:0], SIMD [5:4], CU [11:8], SH [12], SE [15:13]) and XCC_ID.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench/simd_place.hip -o tools/ubench/simd_place
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>

__global__ __launch_bounds__(192) void k_place(unsigned* out, int spin) {
  extern __shared__ double lds[];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    const unsigned hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));
    const unsigned xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11));
    out[2 * (blockIdx.x * 3 + w)] = hw;
    out[2 * (blockIdx.x * 3 + w) + 1] = xcc;
  }
  // keep the workgroup resident for a while (LDS in use, as the rollout's)
  double acc = threadIdx.x;
  for (int i = 0; i < spin; i++) acc = acc * 0.999 + 1.0;
  lds[threadIdx.x] = acc;
  __syncthreads();
  if (lds[(threadIdx.x + 1) % 192] == -1.0) out[0] = 0;  // keeps the loop
}

int main(int argc, char** argv) {
  const int nwg = 64;
  const int lds_kb = argc > 1 ? atoi(argv[1]) : 24;
  unsigned* d;
  hipMalloc(&d, nwg * 3 * 2 * 4);
  hipMemset(d, 0, nwg * 3 * 2 * 4);
  if (lds_kb > 64)
    hipFuncSetAttribute(reinterpret_cast<const void*>(k_place), hipFuncAttributeMaxDynamicSharedMemorySize, lds_kb * 1024);
  k_place<<<nwg, 192, lds_kb * 1024>>>(d, 1 << 16);
  if (hipDeviceSynchronize() != hipSuccess) {
    printf("kernel failed\n");
    return 1;
  }
  std::vector<unsigned> h(nwg * 3 * 2);
  hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
  int shared = 0, distinct_cu = 0;
  std::map<unsigned long long, int> cus;
  for (int b = 0; b < nwg; b++) {
    unsigned simd[3], cu[3];
    for (int w = 0; w < 3; w++) {
      const unsigned hw = h[2 * (b * 3 + w)], xcc = h[2 * (b * 3 + w) + 1];
      simd[w] = (hw >> 4) & 3;
      cu[w] = ((xcc & 15) << 16) | (hw >> 8);
    }
    cus[cu[0]]++;
    const bool sh = simd[0] == simd[1] || simd[0] == simd[2] || simd[1] == simd[2];
    shared += sh;
    if (b < 8)
      printf("wg %2d: waves on SIMD %u %u %u (same CU: %s)\n", b, simd[0], simd[1], simd[2],
             (cu[0] == cu[1] && cu[1] == cu[2]) ? "yes" : "no");
  }
  distinct_cu = (int)cus.size();
  printf("LDS %d KB per workgroup: %d of %d workgroups have two waves on one SIMD; %d distinct CUs\n", lds_kb, shared,
         nwg, distinct_cu);
  return 0;
}
