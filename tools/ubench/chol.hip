// Micro-benchmark of the Newton solver's dense pieces at the humanoid's size
// (nv = 27, one wavefront): the Cholesky factor of H (LDS column form as in
// coop::hessian_factor, and cholesky_rows32) and the search-direction
// substitution (chol_solve_wave, chol_solve_rows32).  Prints cycles per call
// and checks that the register forms give the LDS forms' bits.
//   hipcc -std=c++20 -O3 -ffp-contract=off --offload-arch=gfx950
//         -I ilqg-mujoco_amd/csrc/device -I ilqg-mujoco_amd/csrc tools/ubench/chol.hip -o tools/ubench/chol
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "dsmall.h"

using namespace ilqg::coop;

constexpr int NV = 27, REPS = 64;

// the LDS column Cholesky of hessian_factor (nv <= 64, lane i owns row i)
__device__ void chol_lds(int nv, int tid, double* H) {
  const int i = tid;
  const bool own = i < nv;
  for (int j = 0; j < nv; j++) {
    const bool part = own && i >= j;
    double s = 0;
    if (part) {
      int k = 0;
      for (; k + 8 <= j; k += 8) {
        double x[8], y[8];
#pragma unroll
        for (int q = 0; q < 8; q++) {
          x[q] = H[i * nv + k + q];
          y[q] = H[j * nv + k + q];
        }
#pragma unroll
        for (int q = 0; q < 8; q++) s += x[q] * y[q];
      }
      for (; k < j; k++) s += H[i * nv + k] * H[j * nv + k];
    }
    double t = 0;
    if (i == j) {
      t = H[j * nv + j];
      if (j) t -= s;
      if (t < MINVAL) t = MINVAL;
      t = sqrt(t);
    }
    const double d = bcast(t, j);
    const double tinv = 1 / d;
    if (i == j) H[j * nv + j] = d;
    if (part && i > j) H[i * nv + j] = (H[i * nv + j] - s) * tinv;
    team_sync();
  }
}

__global__ __launch_bounds__(64) void k_bench(const double* H0, const double* g0, double* out, unsigned long long* cyc) {
  __shared__ double Ha[NV * NV], Hb[NV * NV], g[NV], s1[NV], s2[NV], s3[NV];
  const int tid = threadIdx.x;
  unsigned long long c[5] = {0, 0, 0, 0, 0}, c0[5] = {0, 0, 0, 0, 0};
  for (int r = 0; r < REPS; r++) {
    for (int e = tid; e < NV * NV; e += 64) Ha[e] = Hb[e] = H0[e];
    for (int e = tid; e < NV; e += 64) g[e] = g0[e];
    team_sync();
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    chol_lds(NV, tid, Ha);
    team_sync();
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    cholesky_rows32(NV, tid, Hb);
    unsigned long long t2 = __builtin_amdgcn_s_memtime();
    chol_solve_wave(NV, tid, Ha, g, s1);
    unsigned long long t3 = __builtin_amdgcn_s_memtime();
    chol_solve_rows32(NV, tid, Ha, g, s2);
    unsigned long long t4 = __builtin_amdgcn_s_memtime();
    chol_solve_u2(NV, tid, Ha, g, s3);
    unsigned long long t5 = __builtin_amdgcn_s_memtime();
    c[0] += t1 - t0; c[1] += t2 - t1; c[2] += t3 - t2; c[3] += t4 - t3; c[4] += t5 - t4;
    if (r == 0) {  // cold instruction cache
      c0[0] = t1 - t0; c0[1] = t2 - t1; c0[2] = t3 - t2; c0[3] = t4 - t3; c0[4] = t5 - t4;
    }
  }
  for (int e = tid; e < NV * NV; e += 64) {
    out[e] = Ha[e];
    out[NV * NV + e] = Hb[e];
  }
  for (int e = tid; e < NV; e += 64) {
    out[2 * NV * NV + e] = s1[e];
    out[2 * NV * NV + NV + e] = s2[e];
    out[2 * NV * NV + 2 * NV + e] = s3[e];
  }
  if (tid == 0)
    for (int q = 0; q < 5; q++) {
      cyc[q] = c[q];
      cyc[5 + q] = c0[q];
    }
}

int main() {
  // an SPD matrix like M + J'DJ: A A' + diag
  std::vector<double> H(NV * NV), A(NV * NV), gg(NV);
  unsigned s = 12345;
  auto rnd = [&] { s = s * 1103515245u + 12345u; return ((s >> 8) & 0xffff) / 65536.0 - 0.5; };
  for (auto& a : A) a = rnd();
  for (int i = 0; i < NV; i++)
    for (int j = 0; j < NV; j++) {
      double t = 0;
      for (int k = 0; k < NV; k++) t += A[i * NV + k] * A[j * NV + k];
      H[i * NV + j] = t + (i == j ? 1.0 : 0.0);
    }
  for (auto& x : gg) x = rnd();
  double *dH, *dg, *dout;
  unsigned long long* dc;
  hipMalloc(&dH, H.size() * 8);
  hipMalloc(&dg, NV * 8);
  hipMalloc(&dout, (2 * NV * NV + 3 * NV) * 8);
  hipMalloc(&dc, 10 * 8);
  hipMemcpy(dH, H.data(), H.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(dg, gg.data(), NV * 8, hipMemcpyHostToDevice);
  k_bench<<<1, 64>>>(dH, dg, dout, dc);
  if (hipDeviceSynchronize() != hipSuccess) {
    printf("kernel failed\n");
    return 1;
  }
  std::vector<double> out(2 * NV * NV + 3 * NV);
  unsigned long long c[10];
  hipMemcpy(out.data(), dout, out.size() * 8, hipMemcpyDeviceToHost);
  hipMemcpy(c, dc, 80, hipMemcpyDeviceToHost);
  int badf = 0, bads = 0;
  for (int i = 0; i < NV; i++)
    for (int j = 0; j <= i; j++)
      if (memcmp(&out[i * NV + j], &out[NV * NV + i * NV + j], 8)) badf++;
  for (int i = 0; i < NV; i++)
    if (memcmp(&out[2 * NV * NV + i], &out[2 * NV * NV + NV + i], 8) ||
        memcmp(&out[2 * NV * NV + i], &out[2 * NV * NV + 2 * NV + i], 8)) bads++;
  printf("nv=%d cycles per call (s_memtime): factor LDS %.0f, factor rows32 %.0f, solve wave %.0f, solve rows32 %.0f, "
         "solve u2 %.0f\n", NV, c[0] / (double)REPS, c[1] / (double)REPS, c[2] / (double)REPS, c[3] / (double)REPS,
         c[4] / (double)REPS);
  printf("first call (cold instruction cache): factor LDS %llu, factor rows32 %llu, solve wave %llu, solve rows32 %llu, "
         "solve u2 %llu\n", c[5], c[6], c[7], c[8], c[9]);
  printf("bit mismatches: factor %d of %d, solve %d of %d\n", badf, NV * (NV + 1) / 2, bads, NV);
  return (badf || bads) ? 2 : 0;
}
