// libilqg_mujoco.so: the legacy C++ boundary over the C ABI.
//
// Implements the MuJoCo 2.0 API subset of include/legacy/mujoco/mujoco.h, the
// reference's free functions calcMJDerivatives / cpMjData / forwardStep /
// forwardFrame (inc/mjderivative.h:7, inc/util.h:6, inc/update.h:6-8) and the
// non-template core of ILQR<nv,nu,N>.  All physics goes to the GPU through
// include/ilqg_amd.h; this file only moves state and calls the user's host
// cost callback for the cost-gradient samples.
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "ilqg_amd.h"
#include "ilqg_legacy.h"
#include "ilqg_model_blob.h"
#include "ilqg_model_fields.h"
#include "mjderivative.h"
#include "mujoco/mujoco.h"
#include "update.h"
#include "util.h"

namespace {

constexpr mjtNum kEps = 1e-6;  // src/mjderivative.cpp:39

void check(int rc, const char* what) {
  if (rc != ILQG_OK) {
    char buf[512];
    snprintf(buf, sizeof buf, "%s failed (%d): %s", what, rc, ilqg_last_error());
    mju_error(buf);
  }
}

ilqg_model* handle(const mjModel* m) { return static_cast<ilqg_model*>(m->ilqg_model); }

// model arrays live in one arena owned by the mjModel
struct ModelArena {
  std::vector<unsigned char> blob;
};

// cost descriptors registered for host cost callbacks
struct CostDesc {
  std::vector<double> a[9];
  ilqg_cost c{};
};
std::mutex g_cost_mu;
std::map<stepCostFn_t, CostDesc>& cost_registry() {
  static std::map<stepCostFn_t, CostDesc> r;
  return r;
}
const ilqg_cost* lookup_cost(stepCostFn_t fn) {
  std::lock_guard<std::mutex> lk(g_cost_mu);
  auto it = cost_registry().find(fn);
  return it == cost_registry().end() ? nullptr : &it->second.c;
}

int fd_dim(const mjModel* m) { return m->nv * (2 * m->nv + m->nu) + 2 * m->nv + m->nu; }

}  // namespace

// ------------------------------------------------------------------ MuJoCo API
extern "C" {

int mj_activate(const char*) { return 1; }
void mj_deactivate(void) {}

mjModel* mj_loadXML(const char* filename, const void* vfs, char* error, int error_sz) {
  if (error && error_sz > 0) error[0] = 0;
  if (vfs) {
    if (error && error_sz > 0) snprintf(error, error_sz, "VFS is not supported");
    return nullptr;
  }
  ilqg_model* h = nullptr;
  if (ilqg_model_load_xml(filename, &h) != ILQG_OK) {
    if (error && error_sz > 0) snprintf(error, error_sz, "%s", ilqg_last_error());
    return nullptr;
  }
  size_t need = 0;
  ilqg_model_blob(h, nullptr, 0, &need);
  auto* arena = new ModelArena;
  arena->blob.resize(need);
  if (ilqg_model_blob(h, arena->blob.data(), need, &need) != ILQG_OK) {
    if (error && error_sz > 0) snprintf(error, error_sz, "%s", ilqg_last_error());
    delete arena;
    ilqg_model_free(h);
    return nullptr;
  }
  auto* m = static_cast<mjModel*>(calloc(1, sizeof(mjModel)));
  m->ilqg_model = h;
  m->ilqg_arena = arena;
  // walk the compiled-model record (include/ilqg_model_blob.h) and bind fields by name
  unsigned char* p = arena->blob.data() + 16;
  const unsigned char* end = arena->blob.data() + arena->blob.size();
  std::map<std::string, std::pair<int, void*>> fields;
  while (p + sizeof(ilqg_blob_field_hdr) <= end) {
    ilqg_blob_field_hdr hd;
    memcpy(&hd, p, sizeof hd);
    p += sizeof hd;
    size_t bytes = (size_t)hd.count * (hd.dtype == ILQG_BLOB_F64 ? 8 : 4);
    fields[std::string(hd.name, strnlen(hd.name, ILQG_BLOB_NAMELEN))] = {hd.dtype, p};
    p += (bytes + 7) & ~(size_t)7;
  }
  auto i32 = [&](const char* n) { auto it = fields.find(n); return it == fields.end() ? 0 : *(int*)it->second.second; };
  auto f64 = [&](const char* n) {
    auto it = fields.find(n);
    return it == fields.end() ? 0.0 : *(double*)it->second.second;
  };
  m->nq = i32("nq"); m->nv = i32("nv"); m->nu = i32("nu"); m->nbody = i32("nbody");
  m->njnt = i32("njnt"); m->ngeom = i32("ngeom"); m->nconmax = i32("nconmax"); m->njmax = i32("njmax");
  m->nstack = i32("nstack");
  m->opt.timestep = f64("opt_timestep"); m->opt.impratio = f64("opt_impratio");
  m->opt.tolerance = f64("opt_tolerance");
  m->opt.gravity[0] = f64("opt_gravity0"); m->opt.gravity[1] = f64("opt_gravity1");
  m->opt.gravity[2] = f64("opt_gravity2");
  m->opt.integrator = i32("opt_integrator"); m->opt.cone = i32("opt_cone"); m->opt.solver = i32("opt_solver");
  m->opt.iterations = i32("opt_iterations"); m->opt.disableflags = i32("opt_disableflags");
  m->opt.enableflags = i32("opt_enableflags");
  m->stat.meaninertia = f64("stat_meaninertia");
#define ILQG_BIND(nm, cnt) \
  { auto it = fields.find(#nm); m->nm = it == fields.end() ? nullptr : (decltype(m->nm))it->second.second; }
  ILQG_MODEL_F64_ARRAYS(ILQG_BIND)
  ILQG_MODEL_I32_ARRAYS(ILQG_BIND)
#undef ILQG_BIND
  return m;
}

void mj_deleteModel(mjModel* m) {
  if (!m) return;
  ilqg_model_free(handle(m));
  delete static_cast<ModelArena*>(m->ilqg_arena);
  free(m);
}

mjData* mj_makeData(const mjModel* m) {
  auto* d = static_cast<mjData*>(calloc(1, sizeof(mjData)));
  const size_t n = (size_t)m->nq + 5 * (size_t)m->nv + m->nu + 6 * (size_t)m->nbody;
  auto* buf = static_cast<mjtNum*>(calloc(n, sizeof(mjtNum)));
  d->ilqg_arena = buf;
  d->qpos = buf;
  d->qvel = d->qpos + m->nq;  // contiguous with qpos (inc/ilqr.h:90)
  d->qacc_warmstart = d->qvel + m->nv;
  d->qacc = d->qacc_warmstart + m->nv;
  d->qfrc_applied = d->qacc + m->nv;
  d->ctrl = d->qfrc_applied + m->nv;
  d->xfrc_applied = d->ctrl + m->nu;
  d->nstack = m->nstack > 0 ? m->nstack : 1;
  d->stack = static_cast<mjtNum*>(calloc((size_t)d->nstack, sizeof(mjtNum)));
  mj_resetData(m, d);
  return d;
}

void mj_deleteData(mjData* d) {
  if (!d) return;
  free(d->ilqg_arena);
  free(d->stack);
  free(d);
}

void mj_resetData(const mjModel* m, mjData* d) {
  d->time = 0;
  mju_copy(d->qpos, m->qpos0, m->nq);
  mju_zero(d->qvel, m->nv);
  mju_zero(d->qacc_warmstart, m->nv);
  mju_zero(d->qacc, m->nv);
  mju_zero(d->qfrc_applied, m->nv);
  mju_zero(d->ctrl, m->nu);
  mju_zero(d->xfrc_applied, 6 * m->nbody);
  d->pstack = 0;
  d->maxuse_stack = 0;
}

mjtNum* mj_stackAlloc(mjData* d, int size) {
  if (size <= 0) return d->stack + d->pstack;
  if (d->pstack + size > d->nstack) mju_error("mj_stackAlloc: insufficient memory");
  mjtNum* r = d->stack + d->pstack;
  d->pstack += size;
  if (d->pstack > d->maxuse_stack) d->maxuse_stack = d->pstack;
  return r;
}

void mj_step(const mjModel* m, mjData* d) {
  check(ilqg_step_batch(handle(m), 1, 1, &d->time, d->qpos, d->qvel, d->qacc_warmstart, d->ctrl, d->qfrc_applied,
                        d->xfrc_applied),
        "mj_step");
}

void mj_forward(const mjModel* m, mjData* d) {
  check(ilqg_forward_batch(handle(m), 1, d->qpos, d->qvel, d->qacc_warmstart, d->ctrl, d->qfrc_applied,
                           d->xfrc_applied, d->qacc),
        "mj_forward");
}

void mj_forwardSkip(const mjModel* m, mjData* d, int, int) { mj_forward(m, d); }

void mju_copy(mjtNum* res, const mjtNum* data, int n) {
  if (n > 0) memmove(res, data, sizeof(mjtNum) * (size_t)n);
}
void mju_zero(mjtNum* res, int n) {
  if (n > 0) memset(res, 0, sizeof(mjtNum) * (size_t)n);
}
void* mju_malloc(size_t size) {
  void* p = nullptr;
  if (posix_memalign(&p, 8, size ? size : 8)) mju_error("mju_malloc: out of memory");
  return p;
}
void mju_free(void* ptr) { free(ptr); }
void mju_error(const char* msg) {
  fprintf(stderr, "ERROR: %s\n", msg);
  exit(1);
}
void mju_error_s(const char* msg, const char* text) {
  char buf[1024];
  snprintf(buf, sizeof buf, msg, text);
  mju_error(buf);
}

// MuJoCo 2.0 mju_quatIntegrate: rotate quat by vel*scale (axis-angle), host libm
void mju_quatIntegrate(mjtNum* quat, const mjtNum* vel, mjtNum scale) {
  mjtNum ax[3] = {vel[0], vel[1], vel[2]};
  mjtNum nrm = std::sqrt(ax[0] * ax[0] + ax[1] * ax[1] + ax[2] * ax[2]);
  if (nrm < mjMINVAL) {
    ax[0] = 1; ax[1] = 0; ax[2] = 0;
  } else {
    ax[0] /= nrm; ax[1] /= nrm; ax[2] /= nrm;
  }
  const mjtNum ang = scale * nrm;
  const mjtNum s = std::sin(ang * 0.5);
  mjtNum qr[4] = {std::cos(ang * 0.5), ax[0] * s, ax[1] * s, ax[2] * s};
  mjtNum qn = std::sqrt(quat[0] * quat[0] + quat[1] * quat[1] + quat[2] * quat[2] + quat[3] * quat[3]);
  if (qn < mjMINVAL) {
    quat[0] = 1; quat[1] = quat[2] = quat[3] = 0;
  } else {
    for (int i = 0; i < 4; i++) quat[i] /= qn;
  }
  mjtNum q[4] = {quat[0] * qr[0] - quat[1] * qr[1] - quat[2] * qr[2] - quat[3] * qr[3],
                 quat[0] * qr[1] + quat[1] * qr[0] + quat[2] * qr[3] - quat[3] * qr[2],
                 quat[0] * qr[2] - quat[1] * qr[3] + quat[2] * qr[0] + quat[3] * qr[1],
                 quat[0] * qr[3] + quat[1] * qr[2] - quat[2] * qr[1] + quat[3] * qr[0]};
  for (int i = 0; i < 4; i++) quat[i] = q[i];
}

}  // extern "C"

// ------------------------------------------------- reference free functions
void cpMjData(const mjModel* m, mjData* dst, const mjData* src) {
  dst->time = src->time;
  mju_copy(dst->qpos, src->qpos, m->nq);
  mju_copy(dst->qvel, src->qvel, m->nv);
  mju_copy(dst->qacc, src->qacc, m->nv);
  mju_copy(dst->qacc_warmstart, src->qacc_warmstart, m->nv);
  mju_copy(dst->qfrc_applied, src->qfrc_applied, m->nv);
  mju_copy(dst->xfrc_applied, src->xfrc_applied, 6 * m->nbody);
  mju_copy(dst->ctrl, src->ctrl, m->nu);
}

void forwardStep(mjModel* model, mjData* data) { mj_step(model, data); }

void forwardFrame(mjModel* model, mjData* data) {
  const mjtNum start = data->time;
  while (data->time - start < 1.0 / 60.0f) forwardStep(model, data);
}

void calcMJDerivatives(mjModel* m, mjData* dmain, mjtNum* deriv, stepCostFn_t stepCostFn) {
  const ilqg_cost* dc = lookup_cost(stepCostFn);
  check(ilqg_fd_batch(handle(m), 1, dmain->qpos, dmain->qvel, dmain->qacc_warmstart, dmain->ctrl,
                      dmain->qfrc_applied, dmain->xfrc_applied, dc, deriv),
        "calcMJDerivatives");
  if (!dc && stepCostFn) ilqg_legacy::host_cost_columns(m, dmain, stepCostFn, deriv);
}

namespace ilqg_legacy {

void register_cost(stepCostFn_t fn, const ilqg_cost* desc, int nq, int nv, int nu) {
  std::lock_guard<std::mutex> lk(g_cost_mu);
  CostDesc& cd = cost_registry()[fn];
  const double* src[9] = {desc->wq, desc->tq, desc->lq, desc->wv, desc->tv, desc->lv, desc->wu, desc->tu, desc->lu};
  const int len[9] = {nq, nq, nq, nv, nv, nv, nu, nu, nu};
  const double** dst[9] = {&cd.c.wq, &cd.c.tq, &cd.c.lq, &cd.c.wv, &cd.c.tv, &cd.c.lv, &cd.c.wu, &cd.c.tu, &cd.c.lu};
  for (int i = 0; i < 9; i++) {
    cd.a[i].assign(len[i], 0.0);
    if (src[i]) cd.a[i].assign(src[i], src[i] + len[i]);
    *dst[i] = cd.a[i].data();
  }
}

void host_cost_columns(const mjModel* m, const mjData* dmain, stepCostFn_t fn, mjtNum* deriv) {
  const int nv = m->nv, nu = m->nu;
  mjData* d = mj_makeData(m);
  cpMjData(m, d, dmain);
  mjtNum* g = deriv + nv * (2 * nv + nu);
  const mjtNum center = fn(dmain);  // src/mjderivative.cpp:72
  for (int i = 0; i < nu && i < nv; i++) {  // ctrl columns, :78-90
    d->ctrl[i] = dmain->ctrl[i] + kEps;
    g[2 * nv + i] = (fn(d) - center) / kEps;
    d->ctrl[i] = dmain->ctrl[i];
  }
  for (int i = 0; i < nv; i++) {  // qvel columns, :114-120
    d->qvel[i] = dmain->qvel[i] + kEps;
    g[nv + i] = (fn(d) - center) / kEps;
    d->qvel[i] = dmain->qvel[i];
  }
  for (int i = 0; i < nv; i++) {  // qpos columns, :145-174
    const int j = m->dof_jntid[i];
    const int type = m->jnt_type[j];
    if (type == mjJNT_BALL || (type == mjJNT_FREE && i >= m->jnt_dofadr[j] + 3)) {
      const int qa = m->jnt_qposadr[j] + (type == mjJNT_FREE ? 3 : 0);
      const int dp = i - m->jnt_dofadr[j] - (type == mjJNT_FREE ? 3 : 0);
      mjtNum av[3] = {0, 0, 0};
      av[dp] = kEps;
      mju_quatIntegrate(d->qpos + qa, av, 1);
    } else {
      d->qpos[m->jnt_qposadr[j] + i - m->jnt_dofadr[j]] += kEps;
    }
    g[i] = (fn(d) - center) / kEps;
    mju_copy(d->qpos, dmain->qpos, m->nq);
  }
  mj_deleteData(d);
}

// ------------------------------------------------------------ ILQR core
struct SolverCore::Impl {
  mjModel* m = nullptr;
  ilqg_solver* s = nullptr;
  int N = 0, P = 0, nq = 0, nv = 0, nu = 0, D = 0;
  stepCostFn_t fn = nullptr;
  bool device_cost = false;
  std::vector<double> time, qpos, qvel, warm, ctrl, deriv;
  bool swept = false;  // deriv holds the records of the trajectory in time..ctrl
};

SolverCore::SolverCore(mjModel* m, int N, stepCostFn_t fn) : p_(new Impl) {
  Impl& I = *p_;
  I.m = m;
  I.N = N;
  I.P = N + 1;
  I.nq = m->nq;
  I.nv = m->nv;
  I.nu = m->nu;
  I.D = fd_dim(m);
  I.fn = fn;
  const ilqg_cost* dc = lookup_cost(fn);
  I.device_cost = dc != nullptr;
  ilqg_cost zero{};
  const double one = 1.0;
  ilqg_solver_opts o{};
  o.horizon = N;
  o.nseed = 1;
  o.nalpha = 1;
  o.alphas = &one;
  o.select_mode = 0;
  o.mu = 1000.0;  // inc/ilqr.h:65
  o.device = 0;
  check(ilqg_solver_create(handle(m), &o, dc ? dc : &zero, &I.s), "ILQR");
  I.time.resize(I.P);
  I.qpos.resize((size_t)I.P * I.nq);
  I.qvel.resize((size_t)I.P * I.nv);
  I.warm.resize((size_t)I.P * I.nv);
  I.ctrl.resize((size_t)I.P * I.nu);
  I.deriv.resize((size_t)I.P * I.D);
}

SolverCore::~SolverCore() {
  if (p_->s) ilqg_solver_free(p_->s);
  delete p_;
}

void SolverCore::pull_traj(mjData* const* dArray) {
  Impl& I = *p_;
  check(ilqg_solver_get_traj(I.s, I.time.data(), I.qpos.data(), I.qvel.data(), I.warm.data(), I.ctrl.data()),
        "ILQR trajectory");
  for (int n = 0; n < I.P; n++) {
    mjData* d = dArray[n];
    d->time = I.time[n];
    mju_copy(d->qpos, &I.qpos[(size_t)n * I.nq], I.nq);
    mju_copy(d->qvel, &I.qvel[(size_t)n * I.nv], I.nv);
    mju_copy(d->qacc_warmstart, &I.warm[(size_t)n * I.nv], I.nv);
    mju_copy(d->ctrl, &I.ctrl[(size_t)n * I.nu], I.nu);
  }
}

void SolverCore::push_traj(mjData* const* dArray) {
  Impl& I = *p_;
  for (int n = 0; n < I.P; n++) {
    const mjData* d = dArray[n];
    I.time[n] = d->time;
    mju_copy(&I.qpos[(size_t)n * I.nq], d->qpos, I.nq);
    mju_copy(&I.qvel[(size_t)n * I.nv], d->qvel, I.nv);
    mju_copy(&I.warm[(size_t)n * I.nv], d->qacc_warmstart, I.nv);
    mju_copy(&I.ctrl[(size_t)n * I.nu], d->ctrl, I.nu);
  }
  check(ilqg_solver_set_traj(I.s, I.time.data(), I.qpos.data(), I.qvel.data(), I.warm.data(), I.ctrl.data()),
        "ILQR trajectory");
}

void SolverCore::init(const mjData* dmain, mjData* const* dArray) {
  Impl& I = *p_;
  check(ilqg_solver_init(I.s, &dmain->time, dmain->qpos, dmain->qvel, dmain->qacc_warmstart, dmain->ctrl,
                         dmain->qfrc_applied, dmain->xfrc_applied),
        "ILQR init");
  pull_traj(dArray);
  // the applied forces ride along in every cpMjData record (src/util.cpp:11-12)
  for (int n = 0; n < I.P; n++) {
    mju_copy(dArray[n]->qfrc_applied, dmain->qfrc_applied, I.nv);
    mju_copy(dArray[n]->xfrc_applied, dmain->xfrc_applied, 6 * I.m->nbody);
  }
}

void SolverCore::set_dinit(const mjData* d) {
  check(ilqg_solver_set_dinit(p_->s, &d->time, d->qpos, d->qvel, d->qacc_warmstart, d->ctrl), "setDInit");
}

void SolverCore::forward(mjData* const* dArray, const mjtNum* K, const mjtNum* k) {
  push_traj(dArray);
  check(ilqg_solver_set_gains(p_->s, K, k), "ILQR gains");
  check(ilqg_forward(p_->s), "forwardPass");
  pull_traj(dArray);
  p_->swept = false;
}

void SolverCore::sweep(mjData* const* dArray) {
  Impl& I = *p_;
  push_traj(dArray);
  check(ilqg_fd_sweep(I.s), "calcMJDerivatives sweep");
  if (!I.device_cost && I.fn) {
    // cost-gradient entries by host evaluation of the user's callback
    check(ilqg_solver_get_deriv(I.s, I.deriv.data()), "ILQR deriv");
    for (int n = 0; n < I.P; n++) host_cost_columns(I.m, dArray[n], I.fn, &I.deriv[(size_t)n * I.D]);
    check(ilqg_solver_set_deriv(I.s, I.deriv.data()), "ILQR deriv");
  } else {
    // only the records the host reads: initV's (n = 0) and the differentiator's (n = N)
    check(ilqg_solver_get_deriv_point(I.s, 0, 0, &I.deriv[0]), "ILQR deriv");
    check(ilqg_solver_get_deriv_point(I.s, 0, I.N, &I.deriv[(size_t)I.N * I.D]), "ILQR deriv");
  }
  I.swept = true;
}

bool SolverCore::deriv_current(int n, const mjData* d) const {
  const Impl& I = *p_;
  if (!I.swept || n < 0 || n >= I.P) return false;
  return d->time == I.time[n] && !memcmp(d->qpos, &I.qpos[(size_t)n * I.nq], sizeof(mjtNum) * I.nq) &&
         !memcmp(d->qvel, &I.qvel[(size_t)n * I.nv], sizeof(mjtNum) * I.nv) &&
         !memcmp(d->qacc_warmstart, &I.warm[(size_t)n * I.nv], sizeof(mjtNum) * I.nv) &&
         !memcmp(d->ctrl, &I.ctrl[(size_t)n * I.nu], sizeof(mjtNum) * I.nu);
}

bool SolverCore::traj_current(mjData* const* dArray) const {
  for (int n = 0; n < p_->P; n++)
    if (!deriv_current(n, dArray[n])) return false;
  return true;
}

void SolverCore::riccati(mjtNum mu, mjtNum* K, mjtNum* k, mjtNum* V, mjtNum* v) {
  Impl& I = *p_;
  check(ilqg_solver_set_mu(I.s, mu), "ILQR mu");
  // V0 / v0 from initV (virtual, inc/ilqr.h:100-107,142)
  check(ilqg_solver_set_value(I.s, V, v), "ILQR initV");
  check(ilqg_backward(I.s), "backwardPass");
  check(ilqg_solver_get_gains(I.s, K, k), "ILQR gains");
  check(ilqg_solver_get_value(I.s, V, v), "ILQR value");
}

const mjtNum* SolverCore::deriv(int n) const { return &p_->deriv[(size_t)n * p_->D]; }

}  // namespace ilqg_legacy
