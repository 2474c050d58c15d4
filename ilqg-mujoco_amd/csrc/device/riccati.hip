// initV + Riccati backward pass (inc/ilqr.h:100-107,133-176), one 64-lane
// wavefront per seed, every matrix LDS-resident.
//
// Same loops, same summation order as oracle/ilqr_ora.c ora_riccati_step, so
// K, k, V, v are bit-identical to the oracle.  The kernel is a template on
// (NV, NU): the bundled models' sizes (pendulum 2/1, hopper 6/3) get
// compile-time loop bounds and index arithmetic (no integer divisions by a
// runtime nx); <0,0> is the generic instance.  Square matrices use a padded
// leading dimension nx+1 so the strided column walks of the products spread
// over the LDS banks.
#include <hip/hip_runtime.h>

#include "dphys.h"
#include "kernels.h"

namespace ilqg {
namespace {

#ifdef ILQG_STAMPS
__device__ unsigned long long g_bstamp_acc[16];
__device__ unsigned long long g_bstamp_cnt[16];
#define BSTAMP(id)                                            \
  do {                                                        \
    if (tid == 0 && blockIdx.x == 0) {                        \
      unsigned long long t_ = __builtin_amdgcn_s_memtime();   \
      if ((id) >= 0) {                                        \
        g_bstamp_acc[(id) < 0 ? 0 : (id)] += t_ - bst_prev;   \
        g_bstamp_cnt[(id) < 0 ? 0 : (id)]++;                  \
      }                                                       \
      bst_prev = t_;                                          \
    }                                                         \
  } while (0)
#else
#define BSTAMP(id) \
  do {             \
  } while (0)
#endif

}  // namespace
}  // namespace ilqg

#include "riccati.h"
#include "riccati_mfma.h"
#include "dsmall.h"

namespace ilqg {
namespace {

template <int NV_, int NU_>
__global__ __launch_bounds__(rmfma::THREADS) void k_backward_mfma(DevModel m, int nq, int nv, int nu, int P, double dt,
                                                                  double mu, const double* deriv, int Ds, TrajDev tr,
                                                                  double* Kg, double* kg, double* Vg, double* vg,
                                                                  RicFlags fl) {
  extern __shared__ double sh[];
  rmfma::backward_seed_mfma<NV_, NU_>(m, nq, nv, nu, P, dt, mu, deriv, Ds, tr, Kg, kg, Vg, vg, blockIdx.x, sh, fl);
}

template <int NV_, int NU_>
__global__ __launch_bounds__(BW_THREADS) void k_backward(DevModel m, int nq, int nv_rt, int nu_rt, int P, double dt,
                                                         double mu, const double* deriv, int Ds, TrajDev tr,
                                                         double* Kg, double* kg, double* Vg, double* vg,
                                                         RicFlags fl) {
  extern __shared__ double sh[];
  backward_seed<NV_, NU_>(m, nq, nv_rt, nu_rt, P, dt, mu, deriv, Ds, tr, Kg, kg, Vg, vg, blockIdx.x, threadIdx.x, sh,
                          nullptr, 0u, nullptr, fl);
}

template <int NV, int NU>
void launch_t(const DevModel& m, int S, int P, double mu, const double* deriv, int Ds, TrajDev tr, double* K,
              double* k, double* V, double* v, RicFlags fl, size_t lds, hipStream_t st) {
  hipLaunchKernelGGL((k_backward<NV, NU>), dim3(S), dim3(BW_THREADS), lds, st, m, m.nq, m.nv, m.nu, P,
                     m.opt_timestep, mu, deriv, Ds, tr, K, k, V, v, fl);
}

}  // namespace

size_t backward_lds_bytes(int nv, int nu) {
  const size_t nx = 2 * (size_t)nv, LX = nx <= 32 ? nx + 1 : nx;
  const size_t D = (size_t)nv * (2 * nv + nu) + 2 * nv + nu;
  const size_t pre = D <= (size_t)BW_PF * BW_THREADS ? D : 0;
  size_t nd = 4 * nx * LX + 2 * nu * LX + 3 * (size_t)nu * nx + (size_t)nu * nu + 7 * nx + 4 * (size_t)nu + pre;
  return nd * sizeof(double) + 2 * (size_t)nu * sizeof(int) + 16;  // + transp, perm
}

// dynamic + static LDS of k_backward_mfma (the limit check counts both)
size_t backward_mfma_lds_bytes(int nv, int nu) {
  return rmfma::lds_doubles(nv, nu) * sizeof(double) + rmfma::STATIC_LDS_BYTES;
}
bool backward_mfma_supported(int nv, int nu) {
  const int D = nv * (2 * nv + nu) + 2 * nv + nu;
  // stage 5 solves one right-hand side per thread of its waves
  return nu <= rmfma::NU_MAX && D <= rmfma::MPF * rmfma::THREADS && 2 * nv + 1 <= 64 * rmfma::SOLVE_WAVES &&
         backward_mfma_lds_bytes(nv, nu) <= 160 * 1024;
}

hipError_t launch_backward_mfma(const DevModel& m, int S, int P, double mu, const double* deriv, int Ds, TrajDev tr,
                                double* K, double* k, double* V, double* v, RicFlags fl, hipStream_t st) {
  if (!backward_mfma_supported(m.nv, m.nu)) return hipErrorInvalidValue;
  const size_t lds = rmfma::lds_doubles(m.nv, m.nu) * sizeof(double);  // dynamic part
  // nv = 27, nu = 21 (the bundled humanoid): the compile-time instance (ILQG_MFMA_T=0: the generic one, A/B)
  static const int ct = [] {
    const char* e = getenv("ILQG_MFMA_T");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  // ILQG_LDLT_REG=0: the compile-time instance's LDLT on LDS (ldlt_factor_wave_t)
  // instead of in registers (ldlt_factor_reg_t), the same factor; =2: the
  // register path with its pivot replay forced (A/B and tests; read per launch
  // so a test can compare them in one process)
  {
    const char* e = getenv("ILQG_LDLT_REG");
    fl.ldlt_lds = (e && e[0] == '0') ? 1 : (e && e[0] == '2') ? 2 : 0;
  }
#ifndef ILQG_MFMA_NV
#define ILQG_MFMA_NV 0  // 27: nv a compile-time constant too (A/B: 6.78 against 6.34 ms, its VGPRs spill)
#endif
  const bool hum = ct && (ILQG_MFMA_NV == 0 || m.nv == ILQG_MFMA_NV) && m.nu == 21;
  const void* kf = hum ? reinterpret_cast<const void*>(k_backward_mfma<ILQG_MFMA_NV, 21>)
                       : reinterpret_cast<const void*>(k_backward_mfma<0, 0>);
  hipError_t e = hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  if (hum)
    hipLaunchKernelGGL((k_backward_mfma<ILQG_MFMA_NV, 21>), dim3(S), dim3(rmfma::THREADS), lds, st, m, m.nq, m.nv, m.nu, P,
                       m.opt_timestep, mu, deriv, Ds, tr, K, k, V, v, fl);
  else
    hipLaunchKernelGGL((k_backward_mfma<0, 0>), dim3(S), dim3(rmfma::THREADS), lds, st, m, m.nq, m.nv, m.nu, P,
                       m.opt_timestep, mu, deriv, Ds, tr, K, k, V, v, fl);
  return hipGetLastError();
}

hipError_t launch_backward(const DevModel& m, int S, int P, double mu, const double* deriv, int Ds, TrajDev tr,
                           double* K, double* k, double* V, double* v, RicFlags fl, hipStream_t st) {
  if (m.nu > 32) return hipErrorInvalidValue;  // LDLT scratch bound
  const size_t lds = backward_lds_bytes(m.nv, m.nu);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  if (lds > 65536) {
    const void* kf = m.nv == 6 && m.nu == 3   ? reinterpret_cast<const void*>(k_backward<6, 3>)
                     : m.nv == 2 && m.nu == 1 ? reinterpret_cast<const void*>(k_backward<2, 1>)
                                              : reinterpret_cast<const void*>(k_backward<0, 0>);
    hipError_t e = hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  if (m.nv == 6 && m.nu == 3) launch_t<6, 3>(m, S, P, mu, deriv, Ds, tr, K, k, V, v, fl, lds, st);
  else if (m.nv == 2 && m.nu == 1) launch_t<2, 1>(m, S, P, mu, deriv, Ds, tr, K, k, V, v, fl, lds, st);
  else launch_t<0, 0>(m, S, P, mu, deriv, Ds, tr, K, k, V, v, fl, lds, st);
  return hipGetLastError();
}

// ilqg_selftest_div: the split division (dsmall.h) against nothing but the
// host's IEEE quotient -- every-lane form into q, one-lane form into q2
__global__ void k_selftest_div(const double* a, const double* b, double* q, double* q2, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const double x = i < n ? a[i] : 1.0, y = i < n ? b[i] : 1.0;
  const double r = coop::rcp_ref(y);
  const double v = coop::div_ref(x, y, r);
  double w = 0;
  coop::sfor<0, 64>(SLAM(kk) {
    const double t = coop::div_ref_lane<SK(kk)>(x, y, r);
    if (lane == SK(kk)) w = t;
  });
  if (i < n) {
    q[i] = v;
    if (q2) q2[i] = w;
  }
}
hipError_t launch_selftest_div(const double* a, const double* b, double* q, double* q2, int n, hipStream_t st) {
  hipLaunchKernelGGL(k_selftest_div, dim3((n + 255) / 256), dim3(256), 0, st, a, b, q, q2, n);
  return hipGetLastError();
}

}  // namespace ilqg

#ifdef ILQG_STAMPS
// diagnostic build only: per-stage cycles of the Riccati kernel (block 0)
extern "C" int ilqg_debug_bstamps(unsigned long long* acc, unsigned long long* cnt, int reset) {
  if (hipMemcpyFromSymbol(acc, HIP_SYMBOL(ilqg::g_bstamp_acc), sizeof(unsigned long long) * 16) != hipSuccess)
    return 3;
  if (hipMemcpyFromSymbol(cnt, HIP_SYMBOL(ilqg::g_bstamp_cnt), sizeof(unsigned long long) * 16) != hipSuccess)
    return 3;
  if (reset) {
    unsigned long long z[16] = {0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(ilqg::g_bstamp_acc), z, sizeof(z));
    (void)hipMemcpyToSymbol(HIP_SYMBOL(ilqg::g_bstamp_cnt), z, sizeof(z));
  }
  return 0;
}
#endif
