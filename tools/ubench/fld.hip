// Micro-benchmark of the rollout's phase-4 factorizations at the hopper's size
// (nv = 6, a dof chain): the L'DL factors of M and of M + h D by
// factor_ld_rows2 (two half-wave register rows, broadcasts from both halves)
// and by factor_ld_lanes (each factor serially in one lane's registers).
// Prints cycles per call and checks that both give the same bits.
//   hipcc -std=c++20 -O3 -ffp-contract=off --offload-arch=gfx950
//         -I ilqg-mujoco_amd/csrc/device -I ilqg-mujoco_amd/csrc tools/ubench/fld.hip -o tools/ubench/fld
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

#include "dsmall.h"

using namespace ilqg::coop;

constexpr int NV = 6, REPS = 64, NCASE = 64;
struct ChainX {  // the hopper's ancestor masks: dof k's proper ancestors are 0..k-1
  static constexpr unsigned long long pmask[NV] = {0x0, 0x1, 0x3, 0x7, 0xf, 0x1f};
};

__global__ __launch_bounds__(64) void k_bench(const double* M0, const double* hd0, double* out, unsigned long long* cyc) {
  __shared__ double M[NV * NV], H[NV * NV], LA[NV * NV], DA[NV], LB[NV * NV], DB[NV], LC[NV * NV], DC[NV],
      LE[NV * NV], DE[NV];
  const int tid = threadIdx.x;
  const int cs = blockIdx.x;
  unsigned long long c[2] = {0, 0};
  double hd[NV];
  for (int i = 0; i < NV; i++) hd[i] = hd0[cs * NV + i];
  for (int r = 0; r < REPS; r++) {
    for (int e = tid; e < NV * NV; e += 64) {
      const int i = e / NV, j = e % NV;
      M[e] = M0[cs * NV * NV + e];
      H[e] = M[e] + (i == j ? hd[i] : 0.0);
    }
    team_sync();
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    factor_ld_rows2(NV, ChainX::pmask, tid, M, LA, DA, H, LB, DB);
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    factor_ld_lanes<ChainX, NV>(tid, M, hd, true, LC, DC, (int)(LE - LC), (int)(DE - DC));
    unsigned long long t2 = __builtin_amdgcn_s_memtime();
    c[0] += t1 - t0;
    c[1] += t2 - t1;
  }
  double* o = out + (size_t)cs * 4 * (NV * NV + NV);
  for (int e = tid; e < NV * NV; e += 64) {
    o[e] = LA[e];
    o[NV * NV + e] = LB[e];
    o[2 * NV * NV + e] = LC[e];
    o[3 * NV * NV + e] = LE[e];
  }
  for (int e = tid; e < NV; e += 64) {
    o[4 * NV * NV + e] = DA[e];
    o[4 * NV * NV + NV + e] = DB[e];
    o[4 * NV * NV + 2 * NV + e] = DC[e];
    o[4 * NV * NV + 3 * NV + e] = DE[e];
  }
  if (tid == 0 && cs == 0) {
    cyc[0] = c[0];
    cyc[1] = c[1];
  }
}

int main() {
  // SPD matrices like a mass matrix (A A' + diag), some with a tiny pivot so
  // the MINVAL clamp is exercised; damping h*D with zeros
  std::vector<double> M(NCASE * NV * NV), hd(NCASE * NV);
  unsigned s = 12345;
  auto rnd = [&] { s = s * 1103515245u + 12345u; return ((s >> 8) & 0xffff) / 65536.0 - 0.5; };
  for (int c = 0; c < NCASE; c++) {
    double A[NV * NV];
    for (auto& a : A) a = rnd();
    for (int i = 0; i < NV; i++)
      for (int j = 0; j < NV; j++) {
        double t = 0;
        for (int k = 0; k < NV; k++) t += A[i * NV + k] * A[j * NV + k];
        M[c * NV * NV + i * NV + j] = t + (i == j ? (c % 7 == 3 ? 1e-17 : 0.1) : 0.0);
      }
    if (c % 5 == 1) M[c * NV * NV + 0] = -1.0;  // a negative pivot: clamped
    for (int i = 0; i < NV; i++) hd[c * NV + i] = (i % 3 == 0) ? 0.0 : 0.002 * (1 + i) * (1 + c % 3);
  }
  double *dM, *dh, *dout;
  unsigned long long* dc;
  const size_t per = 4 * (NV * NV + NV);
  hipMalloc(&dM, M.size() * 8);
  hipMalloc(&dh, hd.size() * 8);
  hipMalloc(&dout, NCASE * per * 8);
  hipMalloc(&dc, 2 * 8);
  hipMemcpy(dM, M.data(), M.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(dh, hd.data(), hd.size() * 8, hipMemcpyHostToDevice);
  k_bench<<<NCASE, 64>>>(dM, dh, dout, dc);
  if (hipDeviceSynchronize() != hipSuccess) {
    printf("kernel failed\n");
    return 1;
  }
  std::vector<double> out(NCASE * per);
  unsigned long long c[2];
  hipMemcpy(out.data(), dout, out.size() * 8, hipMemcpyDeviceToHost);
  hipMemcpy(c, dc, 16, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int cs = 0; cs < NCASE; cs++) {
    const double* o = &out[cs * per];
    for (int e = 0; e < NV * NV; e++) {
      if (memcmp(&o[e], &o[2 * NV * NV + e], 8)) bad++;
      if (memcmp(&o[NV * NV + e], &o[3 * NV * NV + e], 8)) bad++;
    }
    for (int e = 0; e < NV; e++) {
      if (memcmp(&o[4 * NV * NV + e], &o[4 * NV * NV + 2 * NV + e], 8)) bad++;
      if (memcmp(&o[4 * NV * NV + NV + e], &o[4 * NV * NV + 3 * NV + e], 8)) bad++;
    }
  }
  printf("nv=%d cycles per call (s_memtime, case 0): factor_ld_rows2 %.0f, factor_ld_lanes %.0f\n", NV,
         c[0] / (double)REPS, c[1] / (double)REPS);
  printf("bit mismatches over %d cases: %d of %d\n", NCASE, bad, NCASE * 2 * (NV * NV + NV));
  return bad ? 2 : 0;
}
