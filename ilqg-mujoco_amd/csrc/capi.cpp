// C ABI (include/ilqg_amd.h): model lifecycle, solver context, host<->device
// state exchange and the asynchronous hot-path launches.  No CPU physics:
// every mj_forward / mj_step / FD evaluation runs in the HIP kernels; when no
// GPU is present the device entry points fail with ILQG_ERR_NODEVICE.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "device/dmodel.h"
#include "device/kernels.h"
#include "device/static_models.h"
#include "ilqg_amd.h"
#include "model/model.h"

using namespace ilqg;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
int hip_fail(hipError_t e, const char* what) {
  return fail(e == hipErrorNoDevice ? ILQG_ERR_NODEVICE : ILQG_ERR_HIP,
              std::string(what) + ": " + hipGetErrorName(e) + " (" + hipGetErrorString(e) + ")");
}
#define HIPCHK(expr)                                  \
  do {                                                \
    hipError_t e_ = (expr);                           \
    if (e_ != hipSuccess) return hip_fail(e_, #expr); \
  } while (0)

struct DevBuf {
  void* p = nullptr;
  size_t n = 0;
  ~DevBuf() { release(); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
  hipError_t alloc(size_t bytes) {
    release();
    n = bytes;
    if (!bytes) return hipSuccess;
    hipError_t e = hipMalloc(&p, bytes);
    if (e != hipSuccess) { p = nullptr; return e; }
    return hipMemset(p, 0, bytes);
  }
  template <typename T>
  T* as() const { return static_cast<T*>(p); }
};

// model-specific kernels for the bundled models (ILQG_STATIC=0 disables, for A/B)
bool use_static() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("ILQG_STATIC");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v == 1;
}

constexpr size_t kMaxLds = 160 * 1024;

static int getenv_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e && *e ? atoi(e) : dflt;
}

int check_device_support(const HostModel& m, bool solver, std::string& why) {
  for (int j = 0; j < m.njnt; j++)
    if ((m.jnt_type[j] == 0 || m.jnt_type[j] == 1) && m.jnt_stiffness[j] != 0) {
      why = "stiffness on ball/free joints is not supported";
      return ILQG_ERR_UNSUPPORTED;
    }
  auto power_ok = [](double p) { return p == (double)(int)p && p >= 1 && p <= 8; };
  for (int j = 0; j < m.njnt; j++)
    if (!power_ok(m.jnt_solimp[5 * j + 4])) { why = "solimp power must be an integer in [1,8]"; return ILQG_ERR_UNSUPPORTED; }
  for (int g = 0; g < m.ngeom; g++)
    if (!power_ok(m.geom_solimp[5 * g + 4])) { why = "solimp power must be an integer in [1,8]"; return ILQG_ERR_UNSUPPORTED; }
  if (m.opt_disableflags != 0) { why = "disableflags are not supported"; return ILQG_ERR_UNSUPPORTED; }
  if (solver) {
    // nq != nv (ball/free joints): the state difference runs in the tangent
    // space (oracle ora_state_diff), an extension of inc/ilqr.h:90 (quirk Q21)
    if (m.nu > 32 || m.nu < 1) { why = "nu must be in [1, 32]"; return ILQG_ERR_UNSUPPORTED; }
    if (backward_lds_bytes(m.nv, m.nu) > 160 * 1024) {
      why = "the Riccati workspace exceeds one CU's 160 KB of LDS";
      return ILQG_ERR_UNSUPPORTED;
    }
  }
  return ILQG_OK;
}

}  // namespace

struct ilqg_model {
  HostModel host;
  std::vector<unsigned char> blob;
  // host-side device image: every model array 8-byte aligned in one block, so a
  // workgroup stages the whole read-only model into LDS with one coalesced copy
  std::vector<unsigned char> img;
  std::vector<std::pair<size_t, const void**>> fix;  // (image offset, DevModel pointer field)
  size_t isanc_at = 0, pair_at = 0, pmask_at = 0;
  int npair = 0;
  std::vector<int> key;  // specialization key (ilqg_model_static_key)
  int static_id = 0;     // compiled model-specific kernels, 0 = generic
  // device copy (per device ordinal)
  int dev = -1;
  DevBuf buf;
  DevModel dm{};
  WsLayout Lc{};  // cooperative layout (union scratch)
  coop::CoopAux X{};
  coop::CoopLayout C{};
  hipStream_t stream = nullptr;

  // host preparation: static collision pairs, dof ancestry, image layout, key
  void prepare() {
    const HostModel& h = host;
    // dof ancestor matrix and the statically admissible geom pairs in the
    // oracle's (g1 < g2) enumeration order
    std::vector<int> isanc(h.nv * h.nv, 0), pairs;
    for (int i = 0; i < h.nv; i++)
      for (int j = i; j >= 0; j = h.dof_parentid[j]) isanc[i * h.nv + j] = 1;
    // proper-ancestor bitmask per dof (nv <= 64): the serial tree recursions
    // visit set bits from the highest down, i.e. MuJoCo's parent-chase order
    std::vector<unsigned long long> pmask(h.nv, 0);
    if (h.nv <= 64)
      for (int i = 0; i < h.nv; i++)
        for (int j = h.dof_parentid[i]; j >= 0; j = h.dof_parentid[j]) pmask[i] |= 1ull << j;
    for (int g1 = 0; g1 < h.ngeom; g1++)
      for (int g2 = g1 + 1; g2 < h.ngeom; g2++) {
        int b1 = h.geom_bodyid[g1], b2 = h.geom_bodyid[g2];
        int w1 = h.body_weldid[b1], w2 = h.body_weldid[b2];
        int wp1 = h.body_weldid[h.body_parentid[w1]], wp2 = h.body_weldid[h.body_parentid[w2]];
        if (w1 == w2) continue;
        if (w1 != 0 && w2 != 0 && (w1 == wp2 || w2 == wp1)) continue;
        if (!((h.geom_contype[g1] & h.geom_conaffinity[g2]) || (h.geom_contype[g2] & h.geom_conaffinity[g1])))
          continue;
        pairs.push_back(g1);
        pairs.push_back(g2);
      }
    npair = (int)pairs.size() / 2;
    img.clear();
    fix.clear();
    std::vector<int> offs;
    auto put = [&](const void* src, size_t bytes, const void** dst) {
      size_t at = img.size();
      img.resize(at + ((bytes + 7) & ~(size_t)7), 0);
      if (bytes) memcpy(img.data() + at, src, bytes);
      if (dst) fix.emplace_back(at, dst);
      offs.push_back((int)at);
      return at;
    };
#define ILQG_CP_F(nm, cnt) put(host.nm.data(), host.nm.size() * 8, (const void**)&dm.nm);
#define ILQG_CP_I(nm, cnt)                                          \
  {                                                                 \
    std::vector<int> v_(host.nm.begin(), host.nm.end());            \
    put(v_.data(), v_.size() * 4, (const void**)&dm.nm);            \
  }
    ILQG_MODEL_F64_ARRAYS(ILQG_CP_F)
    ILQG_MODEL_I32_ARRAYS(ILQG_CP_I)
#undef ILQG_CP_F
#undef ILQG_CP_I
    isanc_at = put(isanc.data(), isanc.size() * 4, nullptr);
    pair_at = put(pairs.data(), pairs.size() * 4, nullptr);
    pmask_at = put(pmask.data(), pmask.size() * 8, nullptr);
    img.resize(img.size() + 8, 0);
    // key: everything the model-specific kernels take as compile-time constants
    key.clear();
#define ILQG_K_S(nm) key.push_back(h.nm);
    ILQG_MODEL_I32_SCALARS(ILQG_K_S)
#undef ILQG_K_S
    key.push_back(h.maxcon);
    key.push_back(h.maxefc);
    key.push_back(npair);
    key.push_back((int)img.size());
    key.push_back((int)offs.size());
    key.insert(key.end(), offs.begin(), offs.end());
#define ILQG_K_A(nm, cnt) key.insert(key.end(), h.nm.begin(), h.nm.end());
    ILQG_MODEL_I32_ARRAYS(ILQG_K_A)
#undef ILQG_K_A
    key.insert(key.end(), pairs.begin(), pairs.end());
    static_id = match_static_model(key);
  }

  // the cooperative LDS layouts (host-side: model scalars only)
  void layouts() {
    const HostModel& h = host;
#define ILQG_SC_I(nm) dm.nm = h.nm;
#define ILQG_SC_F(nm) dm.nm = h.nm;
    ILQG_MODEL_I32_SCALARS(ILQG_SC_I)
    ILQG_MODEL_F64_SCALARS(ILQG_SC_F)
#undef ILQG_SC_I
#undef ILQG_SC_F
    dm.maxcon = h.maxcon;
    dm.maxefc = h.maxefc;
    dm.img_bytes = (int)img.size();
    dm.static_id = use_static() ? static_id : 0;
    Lc = make_layout(dm, npair);
    C = coop::make_coop_layout(dm, npair);
    // no LDS left for the model image (humanoid): the kernels read it from its
    // global copy (stage_model with C.imgd == 0)
    if (coop_lds_bytes(Lc, C) > kMaxLds) C.imgd = 0;
  }

  int upload(int device) {
    if (dev == device && buf.p) return ILQG_OK;
    HIPCHK(hipSetDevice(device));
    const HostModel& h = host;
    HIPCHK(buf.alloc(img.size()));
    HIPCHK(hipMemcpy(buf.p, img.data(), img.size(), hipMemcpyHostToDevice));
    for (auto& f : fix) *f.second = static_cast<unsigned char*>(buf.p) + f.first;
    layouts();
    dm.img = static_cast<const unsigned char*>(buf.p);
    X.isanc = reinterpret_cast<const int*>(static_cast<unsigned char*>(buf.p) + isanc_at);
    X.pair = reinterpret_cast<const int*>(static_cast<unsigned char*>(buf.p) + pair_at);
    X.npair = npair;
    X.pmask = h.nv <= 64 ? reinterpret_cast<const unsigned long long*>(static_cast<unsigned char*>(buf.p) + pmask_at)
                         : nullptr;
    X.haspm = X.pmask != nullptr;
    if (getenv("ILQG_VERBOSE"))
      fprintf(stderr, "ilqg: model nq=%d nv=%d static_id=%d lds/team=%zu B (ws %d + coop %d + image %d doubles, %d ints)\n",
              h.nq, h.nv, dm.static_id, coop_lds_bytes(Lc, C), Lc.nd, C.nd, C.imgd, Lc.ni + C.ni);
    if (!stream) HIPCHK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    dev = device;
    return ILQG_OK;
  }
  ~ilqg_model() {
    if (stream) (void)hipStreamDestroy(stream);
  }
};

struct ilqg_solver {
  const ilqg_model* model = nullptr;
  ilqg_solver_opts opts{};
  int S = 0, A = 0, P = 0, D = 0, nx = 0, ncol = 0;
  // FD records at a padded stride Dp (whole 128-byte lines: handoff.h); the
  // fused sweep (fd_fused) also streams the backward pass behind the FD teams
  int Dp = 0, WCp = 0, nut = 0;
  bool fused = false;
  int riccati = ILQG_RICCATI_EXACT;  // ilqg_solver_set_riccati
  int fdprec = ILQG_FD_F64;          // ilqg_solver_set_fd_precision
  hipStream_t stream = nullptr;
  DevBuf traj[5], cand[5], dinit[5];
  DevBuf qfrc_applied, xfrc_applied, K, k, deriv, warm_c, cost_c, V, v, cost_cand, cost_sel, sel, alphas, cost;
  DevBuf cw, sync, fault, plan_dur, plan_order, plan_pos;
  DevBuf snap;  // the centre teams' position/velocity workspace per point (FdFused.snap)
  int snapd = 0;
  DevBuf xq;    // the column halves' qacc exchange (FdFused.halves)
  int halves = 0;
  // schedule knobs, read once at creation (ILQG_FD_SNAP, ILQG_PLAN, ILQG_PLAN_K,
  // ILQG_PLAN_P0): the launch and the debug_plan hook use the same values
  bool snap_on = true, snap_poison = false, plan_on = false;
  float plan_k = 3.0f;
  int plan_p0 = 8;
  // debug_plant_schedule: one-shot (slot, item) pairs written into the next
  // fused launch's ticket map before it is validated
  std::vector<std::pair<unsigned, unsigned>> plants;
  std::vector<double> host_alphas;
  bool initialized = false;
  hipStream_t own_stream = nullptr;
  // pipelined iterate (one candidate per seed, unfused sweep): the rollout in
  // chunks of pipe_chunk points, the FD sweep of each finished chunk on
  // fd_stream behind it (ILQG_PIPE_CHUNK, read at creation; 0 = off)
  int pipe_chunk = 0;
  bool pipe_flat = false;  // ILQG_PIPE_FLAT: equal chunks to the end (A/B)
  static constexpr int kFdStreams = 4;  // chunk c's sweep on fd_stream[c % nfd]: the launches' tails overlap
  hipStream_t fd_stream[kFdStreams] = {};
  int nfd = 3;  // ILQG_PIPE_STREAMS (1 .. 4), read at creation
  std::vector<hipEvent_t> pipe_ev;
  DevBuf carry[5];  // the chunked rollout's state between launches, [S][...]
  bool pipe_ready = false;  // pipe_setup done (fd_stream, pipe_ev, carry)
  // seed groups (ilqg_solver_set_groups): the seeds as G contiguous ranges,
  // software-pipelined.  Group g has a rollout stream (CU-masked to an XCD of
  // its own: one rollout workgroup per CU) and a sweep stream (every CU but the
  // other groups' rollout XCDs); its rollout of iteration n waits for its own
  // sweep of n - 1 and for group g - 1's rollout of n.  In steady state a
  // group's fused sweep runs beside the next group's rollout, which uses a
  // quarter of the chip.  Launches, operands and results are the per-group
  // ones of the ungrouped iterate: the same bits.
  static constexpr int kMaxGroups = 4;
  int ngroups = 1;
  bool grp_join = true;  // the next grouped iterate waits for the solver's stream first
  // ilqg_solver_join_stream with candidates (A > 1): only the groups' selections
  // (which rewrite the selected costs, the nominal trajectory and setDInit) wait
  // for the caller's work on the solver's stream, so the next rollouts still
  // start behind their own sweeps (the pipeline survives the cost exchange)
  bool grp_sel_join = false;
  hipEvent_t grp_ext = nullptr;
  hipStream_t grp_roll[kMaxGroups] = {}, grp_fd[kMaxGroups] = {};
  hipEvent_t grp_sel[kMaxGroups] = {}, grp_done[kMaxGroups] = {};
  // Each group's recursion streams inside its own fused sweep launch: no
  // consumer ever spin-waits on a producer in another launch or stream (round 5
  // ran it as a launch of its own beside the sweep, which broke the rule below
  // and measured slower; removed in round 6).
  DevBuf grp_sync;  // one hand-off block per group
  size_t grp_sync_stride = 0;
  int grp_xcd = 0;  // ILQG_GROUP_XCD: 1 a whole XCD per group rollout, 0 spread over every XCD (default)
  int grp_rcus = 0;  // CUs per group rollout mask (0: unmasked streams)
  // (A split variant -- the Riccati recursion as a launch of its own on a second
  // stream, streaming a concurrent sweep launch's records -- deadlocked when the
  // two streams shared a hardware queue: HIP does not guarantee that two
  // launches run concurrently, so every producer/consumer pair stays inside one
  // ticketed launch.)
  // ilqg_solver_set_layout / ilqg_solver_set_value (device/kernels.h RicFlags)
  int layout = ILQG_LAYOUT_REFERENCE;
  bool vinit_pending = false;  // the next recursion starts from the uploaded V / v
  RicFlags flags() const { return RicFlags{layout, vinit_pending ? 1 : 0}; }
  bool timing = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev[ILQG_NKERNEL];
  std::vector<hipEvent_t> event_pool;

  hipEvent_t get_event() {
    if (!event_pool.empty()) {
      hipEvent_t e = event_pool.back();
      event_pool.pop_back();
      return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
  }
  // record an event pair around a launch when timing is on
  template <typename F>
  hipError_t timed(int kind, F&& launch, hipStream_t st = nullptr) {
    if (!timing) return launch();
    if (!st) st = stream;
    hipEvent_t a = get_event(), b = get_event();
    if (!a || !b) return hipErrorOutOfMemory;
    hipError_t e = hipEventRecord(a, st);
    if (e != hipSuccess) return e;
    e = launch();
    if (e != hipSuccess) return e;
    e = hipEventRecord(b, st);
    ev[kind].emplace_back(a, b);
    return e;
  }

  TrajDev tview(DevBuf* b) const {
    return TrajDev{b[0].as<double>(), b[1].as<double>(), b[2].as<double>(), b[3].as<double>(), b[4].as<double>()};
  }
  CostDev cview() const {
    const double* c = cost.as<double>();
    const int nq = model->host.nq, nv = model->host.nv, nu = model->host.nu;
    return CostDev{c, c + nq, c + 2 * nq, c + 3 * nq, c + 3 * nq + nv, c + 3 * nq + 2 * nv,
                   c + 3 * nq + 3 * nv, c + 3 * nq + 3 * nv + nu, c + 3 * nq + 3 * nv + 2 * nu};
  }
  // every stream the solver launches on
  hipError_t sync_all() {
    hipError_t e = hipStreamSynchronize(stream);
    for (auto fs : fd_stream)
      if (e == hipSuccess && fs) e = hipStreamSynchronize(fs);
    for (int g = 0; g < kMaxGroups; g++) {
      if (e == hipSuccess && grp_roll[g]) e = hipStreamSynchronize(grp_roll[g]);
      if (e == hipSuccess && grp_fd[g]) e = hipStreamSynchronize(grp_fd[g]);
    }
    return e;
  }
  void free_groups() {
    for (int g = 0; g < kMaxGroups; g++) {
      if (grp_roll[g]) (void)hipStreamDestroy(grp_roll[g]);
      if (grp_fd[g]) (void)hipStreamDestroy(grp_fd[g]);
      if (grp_sel[g]) (void)hipEventDestroy(grp_sel[g]);
      if (grp_done[g]) (void)hipEventDestroy(grp_done[g]);
      if (g == 0 && grp_ext) (void)hipEventDestroy(grp_ext), grp_ext = nullptr;
      grp_roll[g] = grp_fd[g] = nullptr;
      grp_sel[g] = grp_done[g] = nullptr;
    }
    grp_sync.release();
    ngroups = 1;
  }
  ~ilqg_solver() {
    (void)sync_all();
    for (auto& v : ev)
      for (auto& p : v) {
        (void)hipEventDestroy(p.first);
        (void)hipEventDestroy(p.second);
      }
    for (auto e : event_pool) (void)hipEventDestroy(e);
    for (auto e : pipe_ev) (void)hipEventDestroy(e);
    for (auto fs : fd_stream)
      if (fs) (void)hipStreamDestroy(fs);
    free_groups();
    if (own_stream) (void)hipStreamDestroy(own_stream);
  }
};

static std::vector<double> pack_cost(const HostModel& m, const ilqg_cost* c) {
  const int nq = m.nq, nv = m.nv, nu = m.nu;
  std::vector<double> out(3 * nq + 3 * nv + 3 * nu, 0.0);
  if (!c) return out;
  auto put = [&](const double* src, int n, size_t at) {
    if (src) std::copy(src, src + n, out.begin() + at);
  };
  put(c->wq, nq, 0); put(c->tq, nq, nq); put(c->lq, nq, 2 * nq);
  put(c->wv, nv, 3 * nq); put(c->tv, nv, 3 * nq + nv); put(c->lv, nv, 3 * nq + 2 * nv);
  put(c->wu, nu, 3 * nq + 3 * nv); put(c->tu, nu, 3 * nq + 3 * nv + nu); put(c->lu, nu, 3 * nq + 3 * nv + 2 * nu);
  return out;
}

extern "C" {

const char* ilqg_last_error(void) { return g_err.c_str(); }
int ilqg_version(void) { return 100; }

int ilqg_device_count(int* count) {
  if (!count) return fail(ILQG_ERR_ARG, "null count");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) { *count = 0; return hip_fail(e, "hipGetDeviceCount"); }
  *count = n;
  return ILQG_OK;
}

// ---------------------------------------------------------------- model --
static int finish_model(ilqg_model* m, ilqg_model** out) {
  m->blob = write_blob(m->host);
  m->prepare();
  // every device path runs one physics evaluation per workgroup with its
  // workspace in LDS: a model whose workspace exceeds one CU's 160 KB is
  // refused here, at load, rather than at the first launch
  m->layouts();
  if (coop_lds_bytes(m->Lc, m->C) > kMaxLds) {
    const size_t b = coop_lds_bytes(m->Lc, m->C);
    delete m;
    return fail(ILQG_ERR_UNSUPPORTED, "model workspace (" + std::to_string(b) +
                                          " B of LDS per physics evaluation) exceeds one CU's LDS (160 KB)");
  }
  *out = m;
  return ILQG_OK;
}

int ilqg_model_load_xml(const char* path, ilqg_model** out) {
  if (!path || !out) return fail(ILQG_ERR_ARG, "null argument");
  auto* m = new ilqg_model();
  std::string err;
  if (!compile_mjcf_file(path, m->host, err)) {
    delete m;
    return fail(ILQG_ERR_MODEL, err);
  }
  return finish_model(m, out);
}

int ilqg_model_load_xml_string(const char* xml, ilqg_model** out) {
  if (!xml || !out) return fail(ILQG_ERR_ARG, "null argument");
  auto* m = new ilqg_model();
  std::string err;
  if (!compile_mjcf_string(xml, m->host, err)) {
    delete m;
    return fail(ILQG_ERR_MODEL, err);
  }
  return finish_model(m, out);
}

void ilqg_model_free(ilqg_model* m) { delete m; }

int ilqg_model_sizes(const ilqg_model* m, int* s) {
  if (!m || !s) return fail(ILQG_ERR_ARG, "null argument");
  const HostModel& h = m->host;
  int v[10] = {h.nq, h.nv, h.nu, h.nbody, h.njnt, h.ngeom, h.maxcon, h.maxefc, h.nconmax, h.njmax};
  memcpy(s, v, sizeof(v));
  return ILQG_OK;
}

int ilqg_model_timestep(const ilqg_model* m, double* dt) {
  if (!m || !dt) return fail(ILQG_ERR_ARG, "null argument");
  *dt = m->host.opt_timestep;
  return ILQG_OK;
}

int ilqg_model_qpos0(const ilqg_model* m, double* q) {
  if (!m || !q) return fail(ILQG_ERR_ARG, "null argument");
  std::copy(m->host.qpos0.begin(), m->host.qpos0.end(), q);
  return ILQG_OK;
}

// cooperative kernels: LDS workspace within one CU's 160 KB, rollout record
// prefetch within 4 registers per lane (kernels_coop.hip)
static bool coop_ok(const ilqg_model* m) {
  return coop_lds_bytes(m->Lc, m->C) <= kMaxLds;
}
static int lds_fail() {
  return fail(ILQG_ERR_UNSUPPORTED, "model workspace exceeds one CU's LDS (160 KB)");
}

// fused FD sweep (kernels_coop.hip k_fd_fused_*): cooperative models whose
// centre warm start fits one lane per dof and whose FD record fits the
// backward role's prefetch registers
static bool fused_ok(const ilqg_model* m) {
  const HostModel& h = m->host;
  const int D = h.nv * (2 * h.nv + h.nu) + 2 * h.nv + h.nu;
  return coop_ok(m) && h.nv <= 64 && D <= 512 && getenv_int("ILQG_FUSED", 1) != 0;
}
static int round16(int n) { return (n + 15) / 16 * 16; }
// ctrl columns on teams of their own, min(nu, nv) of them (mjderivative.cpp:78-82)
static int fd_nut(const HostModel& h) { return std::min(h.nu, h.nv); }
// sync block: ticket, pad x3, cflag[npts], done[npts] (u32), padded to 16 bytes
// [4 + 3 npts + npts ntm] words: ticket, pad, cflag, done, snapshot flags, column pair counters
static size_t sync_bytes(size_t npts, size_t ntm) { return ((4 + 3 * npts + npts * ntm) * 4 + 15) / 16 * 16; }

int ilqg_model_static_key(const ilqg_model* m, int* key, int cap, int* n) {
  if (!m || !n) return fail(ILQG_ERR_ARG, "null argument");
  *n = (int)m->key.size();
  if (key) {
    if (cap < (int)m->key.size()) return fail(ILQG_ERR_ARG, "buffer too small");
    std::copy(m->key.begin(), m->key.end(), key);
  }
  return ILQG_OK;
}

int ilqg_model_static_id(const ilqg_model* m, int* id) {
  if (!m || !id) return fail(ILQG_ERR_ARG, "null argument");
  *id = use_static() ? m->static_id : 0;
  return ILQG_OK;
}

int ilqg_model_blob(const ilqg_model* m, void* buf, size_t cap, size_t* needed) {
  if (!m) return fail(ILQG_ERR_ARG, "null model");
  if (needed) *needed = m->blob.size();
  if (buf) {
    if (cap < m->blob.size()) return fail(ILQG_ERR_ARG, "buffer too small");
    memcpy(buf, m->blob.data(), m->blob.size());
  }
  return ILQG_OK;
}

// ------------------------------------------------------ batched physics --
namespace {
struct Scratch {
  DevBuf time, qpos, qvel, warm, ctrl, qa, xf, out, warm_c, cost_c, cost;
};
int prep_batch(ilqg_model* m, int n, Scratch& s, const double* time, const double* qpos,
               const double* qvel, const double* warm, const double* ctrl, const double* qfrc_applied,
               const double* xfrc_applied) {
  std::string why;
  int rc = check_device_support(m->host, false, why);
  if (rc) return fail(rc, why);
  rc = m->upload(0);
  if (rc) return rc;
  const HostModel& h = m->host;
  HIPCHK(s.time.alloc(n * 8));
  HIPCHK(s.qpos.alloc((size_t)n * h.nq * 8));
  HIPCHK(s.qvel.alloc((size_t)n * h.nv * 8));
  HIPCHK(s.warm.alloc((size_t)n * h.nv * 8));
  HIPCHK(s.ctrl.alloc((size_t)n * h.nu * 8));
  HIPCHK(s.qa.alloc((size_t)n * h.nv * 8));
  HIPCHK(s.xf.alloc((size_t)n * 6 * h.nbody * 8));
  if (!coop_ok(m)) return lds_fail();
  auto up = [&](DevBuf& b, const double* src, size_t cnt) -> hipError_t {
    if (!src) return hipSuccess;
    return hipMemcpy(b.p, src, cnt * 8, hipMemcpyHostToDevice);
  };
  HIPCHK(up(s.time, time, n));
  HIPCHK(up(s.qpos, qpos, (size_t)n * h.nq));
  HIPCHK(up(s.qvel, qvel, (size_t)n * h.nv));
  HIPCHK(up(s.warm, warm, (size_t)n * h.nv));
  HIPCHK(up(s.ctrl, ctrl, (size_t)n * h.nu));
  HIPCHK(up(s.qa, qfrc_applied, (size_t)n * h.nv));
  HIPCHK(up(s.xf, xfrc_applied, (size_t)n * 6 * h.nbody));
  return ILQG_OK;
}
}  // namespace

int ilqg_step_batch(const ilqg_model* mc, int n, int nstep, double* time, double* qpos, double* qvel, double* warm,
                    const double* ctrl, const double* qfrc_applied, const double* xfrc_applied) {
  auto* m = const_cast<ilqg_model*>(mc);
  if (!m || n <= 0 || nstep < 0 || !qpos || !qvel || !warm || !ctrl) return fail(ILQG_ERR_ARG, "bad argument");
  Scratch s;
  std::vector<double> t0(n, 0.0);
  int rc = prep_batch(m, n, s, time ? time : t0.data(), qpos, qvel, warm, ctrl, qfrc_applied, xfrc_applied);
  if (rc) return rc;
  TrajDev st{s.time.as<double>(), s.qpos.as<double>(), s.qvel.as<double>(), s.warm.as<double>(), s.ctrl.as<double>()};
  HIPCHK(launch_step_coop(m->dm, m->Lc, m->C, m->X, st, n, nstep, s.qa.as<double>(), s.xf.as<double>(), m->stream));
  HIPCHK(hipStreamSynchronize(m->stream));
  const HostModel& h = m->host;
  if (time) HIPCHK(hipMemcpy(time, s.time.p, n * 8, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(qpos, s.qpos.p, (size_t)n * h.nq * 8, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(qvel, s.qvel.p, (size_t)n * h.nv * 8, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(warm, s.warm.p, (size_t)n * h.nv * 8, hipMemcpyDeviceToHost));
  return ILQG_OK;
}

int ilqg_forward_batch(const ilqg_model* mc, int n, const double* qpos, const double* qvel, double* warm,
                       const double* ctrl, const double* qfrc_applied, const double* xfrc_applied, double* qacc) {
  auto* m = const_cast<ilqg_model*>(mc);
  if (!m || n <= 0 || !qpos || !qvel || !warm || !ctrl || !qacc) return fail(ILQG_ERR_ARG, "bad argument");
  Scratch s;
  std::vector<double> t0(n, 0.0);
  int rc = prep_batch(m, n, s, t0.data(), qpos, qvel, warm, ctrl, qfrc_applied, xfrc_applied);
  if (rc) return rc;
  const HostModel& h = m->host;
  HIPCHK(s.out.alloc((size_t)n * h.nv * 8));
  TrajDev st{s.time.as<double>(), s.qpos.as<double>(), s.qvel.as<double>(), s.warm.as<double>(), s.ctrl.as<double>()};
  HIPCHK(launch_forward_coop(m->dm, m->Lc, m->C, m->X, st, n, s.qa.as<double>(), s.xf.as<double>(),
                             s.out.as<double>(), m->stream));
  HIPCHK(hipStreamSynchronize(m->stream));
  HIPCHK(hipMemcpy(qacc, s.out.p, (size_t)n * h.nv * 8, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(warm, s.warm.p, (size_t)n * h.nv * 8, hipMemcpyDeviceToHost));
  return ILQG_OK;
}

int ilqg_fd_batch(const ilqg_model* mc, int n, const double* qpos, const double* qvel, const double* warm,
                  const double* ctrl, const double* qfrc_applied, const double* xfrc_applied, const ilqg_cost* cost,
                  double* deriv) {
  auto* m = const_cast<ilqg_model*>(mc);
  if (!m || n <= 0 || !qpos || !qvel || !warm || !ctrl || !deriv) return fail(ILQG_ERR_ARG, "bad argument");
  const HostModel& h = m->host;
  const int nctrl = std::min(h.nu, h.nv), ncol = nctrl + 2 * h.nv;
  const int D = h.nv * (2 * h.nv + h.nu) + 2 * h.nv + h.nu;
  Scratch s;
  std::vector<double> t0(n, 0.0);
  int rc = prep_batch(m, n, s, t0.data(), qpos, qvel, warm, ctrl, qfrc_applied, xfrc_applied);
  if (rc) return rc;
  std::vector<double> cp = pack_cost(h, cost);
  HIPCHK(s.cost.alloc(cp.size() * 8));
  HIPCHK(hipMemcpy(s.cost.p, cp.data(), cp.size() * 8, hipMemcpyHostToDevice));
  HIPCHK(s.warm_c.alloc((size_t)n * h.nv * 8));
  HIPCHK(s.cost_c.alloc((size_t)n * 8));
  HIPCHK(s.out.alloc((size_t)n * D * 8));
  const double* c = s.cost.as<double>();
  const int nq = h.nq, nv = h.nv, nu = h.nu;
  CostDev cd{c, c + nq, c + 2 * nq, c + 3 * nq, c + 3 * nq + nv, c + 3 * nq + 2 * nv,
             c + 3 * nq + 3 * nv, c + 3 * nq + 3 * nv + nu, c + 3 * nq + 3 * nv + 2 * nu};
  TrajDev st{s.time.as<double>(), s.qpos.as<double>(), s.qvel.as<double>(), s.warm.as<double>(), s.ctrl.as<double>()};
  if (fused_ok(m)) {
    // n points as n one-point trajectories through the fused sweep (no backward roles)
    const int Dp = round16(D), WCp = round16(h.nv + 1);
    DevBuf cw, sy, fl, outp;
    HIPCHK(cw.alloc((size_t)n * WCp * 8));
    HIPCHK(sy.alloc(sync_bytes(n, fd_nut(h) + 2 * h.nv)));
    HIPCHK(fl.alloc(16));
    HIPCHK(outp.alloc((size_t)n * Dp * 8));
    HIPCHK(hipMemsetAsync(fl.p, 0, 16, m->stream));
    HIPCHK(hipMemsetAsync(sy.p, 0, sync_bytes(n, fd_nut(h) + 2 * h.nv), m->stream));
    FdFused a{};
    a.tr = st; a.S = n; a.P = 1; a.nB = 0; a.nv = h.nv; a.nut = fd_nut(h);
    a.Dp = Dp; a.WCp = WCp; a.qfrc_applied = s.qa.as<double>(); a.xfrc_applied = s.xf.as<double>(); a.cost = cd;
    a.cw = cw.as<double>(); a.deriv = outp.as<double>(); a.sync = sy.as<unsigned>(); a.fault = fl.as<unsigned>();
    HIPCHK(launch_fd_fused_coop(m->dm, m->Lc, m->C, m->X, a, m->stream));
    HIPCHK(hipStreamSynchronize(m->stream));
    unsigned flt = 0;
    HIPCHK(hipMemcpy(&flt, fl.p, 4, hipMemcpyDeviceToHost));
    if (flt) return fail(ILQG_ERR_HIP, "fused FD sweep: a hand-off wait timed out");
    HIPCHK(hipMemcpy2D(deriv, (size_t)D * 8, outp.p, (size_t)Dp * 8, (size_t)D * 8, n, hipMemcpyDeviceToHost));
    return ILQG_OK;
  } else {
    HIPCHK(launch_fd_centre_coop(m->dm, m->Lc, m->C, m->X, st, n, 1, s.qa.as<double>(), s.xf.as<double>(), cd,
                                 s.warm_c.as<double>(), s.cost_c.as<double>(), m->stream));
    HIPCHK(launch_fd_cols_coop(m->dm, m->Lc, m->C, m->X, st, n, 1, s.qa.as<double>(), s.xf.as<double>(), cd,
                               s.warm_c.as<double>(), s.cost_c.as<double>(), s.out.as<double>(), D, m->stream));
  }
  HIPCHK(hipStreamSynchronize(m->stream));
  HIPCHK(hipMemcpy(deriv, s.out.p, (size_t)n * D * 8, hipMemcpyDeviceToHost));
  return ILQG_OK;
}

// --------------------------------------------------------------- solver --
int ilqg_solver_create(const ilqg_model* mc, const ilqg_solver_opts* o, const ilqg_cost* cost, ilqg_solver** out) {
  auto* m = const_cast<ilqg_model*>(mc);
  if (!m || !o || !out) return fail(ILQG_ERR_ARG, "null argument");
  if (o->horizon < 1 || o->nseed < 1 || o->nalpha < 1) return fail(ILQG_ERR_ARG, "horizon, nseed, nalpha must be >= 1");
  std::string why;
  int rc = check_device_support(m->host, true, why);
  if (rc) return fail(rc, why);
  rc = m->upload(o->device);
  if (rc) return rc;
  if (!coop_ok(m)) return lds_fail();
  const HostModel& h = m->host;
  auto* s = new ilqg_solver();
  s->model = m;
  s->opts = *o;
  s->S = o->nseed;
  s->A = o->nalpha;
  s->P = o->horizon + 1;
  s->nx = 2 * h.nv;
  s->D = h.nv * (2 * h.nv + h.nu) + 2 * h.nv + h.nu;
  s->ncol = std::min(h.nu, h.nv) + 2 * h.nv;
  s->Dp = round16(s->D);
  s->WCp = round16(h.nv + 1);
  s->fused = fused_ok(m);
  s->nut = fd_nut(h);
  s->host_alphas.assign(o->nalpha, 1.0);
  if (o->alphas) std::copy(o->alphas, o->alphas + o->nalpha, s->host_alphas.begin());
  s->opts.alphas = nullptr;
  const size_t S = s->S, A = s->A, P = s->P;
  auto fail_free = [&](hipError_t e, const char* w) {
    delete s;
    return hip_fail(e, w);
  };
#define ALLOC(b, bytes) do { hipError_t e_ = (b).alloc(bytes); if (e_ != hipSuccess) return fail_free(e_, #b); } while (0)
  hipError_t e = hipStreamCreateWithFlags(&s->own_stream, hipStreamNonBlocking);
  if (e != hipSuccess) return fail_free(e, "hipStreamCreate");
  s->stream = s->own_stream;
  const size_t fld[5] = {1, (size_t)h.nq, (size_t)h.nv, (size_t)h.nv, (size_t)h.nu};
  for (int f = 0; f < 5; f++) {
    ALLOC(s->traj[f], S * P * fld[f] * 8);
    ALLOC(s->dinit[f], S * fld[f] * 8);
    if (A > 1) ALLOC(s->cand[f], S * A * P * fld[f] * 8);
  }
  ALLOC(s->qfrc_applied, S * h.nv * 8);
  ALLOC(s->xfrc_applied, S * 6 * h.nbody * 8);
  ALLOC(s->K, S * P * h.nu * s->nx * 8);  // zero-initialised gains (quirk Q12)
  ALLOC(s->k, S * P * h.nu * 8);
  ALLOC(s->deriv, S * P * s->Dp * 8);
  if (s->fused) {
    ALLOC(s->cw, S * P * s->WCp * 8);
    const size_t ntm = (size_t)s->nut + 2 * (size_t)h.nv;
    ALLOC(s->sync, sync_bytes(S * P, ntm));
    // every column as two items (FdFused.halves): the qacc exchange
    s->halves = getenv_int("ILQG_FD_HALVES", 0) ? 1 : 0;  // opt-in: measured slower
    if (s->halves) ALLOC(s->xq, S * P * ntm * 2 * (size_t)h.nv * 8);
    // the ticket schedule, the per-item durations it is planned from (zero: no
    // history) and the validator's scratch
    const size_t items = S * P * (1 + (s->halves ? 2 : 1) * ntm);
    ALLOC(s->plan_dur, items * 4);
    ALLOC(s->plan_order, items * 4);
    ALLOC(s->plan_pos, items * 4);
    s->plan_on = getenv_int("ILQG_PLAN", 0) != 0;
    if (const char* pk = getenv("ILQG_PLAN_K")) s->plan_k = (float)atof(pk);
    s->plan_p0 = getenv_int("ILQG_PLAN_P0", 8);
    s->snap_on = getenv_int("ILQG_FD_SNAP", 1) != 0;
    s->snap_poison = getenv_int("ILQG_SNAP_POISON", 0) != 0;  // tests: see FdFused.poison
    if (s->snap_on) {
      const ilqg_model* mm = s->model;
      s->snapd = round16(mm->Lc.nd + mm->C.nd + (mm->Lc.ni + mm->C.ni + 1) / 2);
      ALLOC(s->snap, S * P * (size_t)s->snapd * 8);
    }
  }
  ALLOC(s->fault, 2 * ilqg_solver::kMaxGroups * sizeof(unsigned));  // one fault block (handoff.h) per seed group
  // chunks of 7 points to the end (flat): cfg 5 21.53-21.59 iterations/s
  // against 21.28-21.31 with 10, 21.51 with 9, 19.9 with 6, after round 6's
  // faster fp32 sweep and recursion (round 5: 10 best, with halving tail
  // chunks worse; profiles/r05_cfg5_pipeline.txt, r06_cfg5_chunks.txt)
  s->pipe_chunk = getenv_int("ILQG_PIPE_CHUNK", 7);
  s->pipe_flat = getenv_int("ILQG_PIPE_FLAT", 1) != 0;
  s->nfd = std::min(std::max(getenv_int("ILQG_PIPE_STREAMS", 3), 1), (int)ilqg_solver::kFdStreams);
  // the pipeline's streams, events and carry buffers are created by the first
  // pipelined iterate (pipe_setup): most solvers never take that path, and the
  // box gives a process 4 hardware queues
  if (!(s->A == 1 && s->pipe_chunk > 0 && s->pipe_chunk < (int)P)) s->pipe_chunk = 0;
  ALLOC(s->warm_c, S * P * h.nv * 8);
  ALLOC(s->cost_c, S * P * 8);
  ALLOC(s->V, S * s->nx * s->nx * 8);
  ALLOC(s->v, S * s->nx * 8);
  ALLOC(s->cost_cand, S * A * 8);
  ALLOC(s->cost_sel, S * 8);
  ALLOC(s->sel, S * 4);
  ALLOC(s->alphas, A * 8);
  std::vector<double> cp = pack_cost(h, cost);
  ALLOC(s->cost, cp.size() * 8);
  e = hipMemcpy(s->alphas.p, s->host_alphas.data(), A * 8, hipMemcpyHostToDevice);
  if (e != hipSuccess) return fail_free(e, "alphas");
  e = hipMemcpy(s->cost.p, cp.data(), cp.size() * 8, hipMemcpyHostToDevice);
  if (e != hipSuccess) return fail_free(e, "cost");
  size_t lds = backward_lds_bytes(h.nv, h.nu);
  if (lds > 160 * 1024) {
    delete s;
    return fail(ILQG_ERR_UNSUPPORTED, "backward pass LDS footprint exceeds 160 KiB (nx too large)");
  }
  *out = s;
  return ILQG_OK;
#undef ALLOC
}

void ilqg_solver_free(ilqg_solver* s) { delete s; }

static int upload_state(ilqg_solver* s, DevBuf* dst, size_t npts, const double* time, const double* qpos,
                        const double* qvel, const double* warm, const double* ctrl) {
  const HostModel& h = s->model->host;
  const double* src[5] = {time, qpos, qvel, warm, ctrl};
  const size_t fld[5] = {1, (size_t)h.nq, (size_t)h.nv, (size_t)h.nv, (size_t)h.nu};
  HIPCHK(s->sync_all());  // no launch still reading the buffers being replaced
  for (int f = 0; f < 5; f++)
    if (src[f]) HIPCHK(hipMemcpyAsync(dst[f].p, src[f], npts * fld[f] * 8, hipMemcpyHostToDevice, s->stream));
    else HIPCHK(hipMemsetAsync(dst[f].p, 0, npts * fld[f] * 8, s->stream));
  HIPCHK(s->sync_all());
  return ILQG_OK;
}

int ilqg_solver_init(ilqg_solver* s, const double* time, const double* qpos, const double* qvel, const double* warm,
                     const double* ctrl, const double* qfrc_applied, const double* xfrc_applied) {
  if (!s || !qpos || !qvel) return fail(ILQG_ERR_ARG, "bad argument");
  const ilqg_model* m = s->model;
  const HostModel& h = m->host;
  int rc = upload_state(s, s->dinit, s->S, time, qpos, qvel, warm, ctrl);
  if (rc) return rc;
  if (qfrc_applied)
    HIPCHK(hipMemcpy(s->qfrc_applied.p, qfrc_applied, (size_t)s->S * h.nv * 8, hipMemcpyHostToDevice));
  if (xfrc_applied)
    HIPCHK(hipMemcpy(s->xfrc_applied.p, xfrc_applied, (size_t)s->S * 6 * h.nbody * 8, hipMemcpyHostToDevice));
  // ILQR ctor: passive rollout with constant ctrl into dArray[N..0]
  TrajDev nom = s->tview(s->traj), di = s->tview(s->dinit);
  HIPCHK(launch_rollout_coop(m->dm, m->Lc, m->C, m->X, s->S, 1, s->P, nom, nom, 0, s->K.as<double>(),
                             s->k.as<double>(), nullptr, di, s->qfrc_applied.as<double>(),
                             s->xfrc_applied.as<double>(), 1, s->cview(), nullptr, s->stream));
  HIPCHK(s->sync_all());
  // setDInit(dmain) as the MPC driver does before iterating (src/inverted_pendulum/inverted_pendulum.cpp:21)
  s->initialized = true;
  return upload_state(s, s->dinit, s->S, time, qpos, qvel, warm, ctrl);
}

int ilqg_solver_set_dinit(ilqg_solver* s, const double* time, const double* qpos, const double* qvel,
                          const double* warm, const double* ctrl) {
  if (!s) return fail(ILQG_ERR_ARG, "null solver");
  return upload_state(s, s->dinit, s->S, time, qpos, qvel, warm, ctrl);
}

int ilqg_solver_set_traj(ilqg_solver* s, const double* time, const double* qpos, const double* qvel,
                         const double* warm, const double* ctrl) {
  if (!s) return fail(ILQG_ERR_ARG, "null solver");
  s->initialized = true;
  return upload_state(s, s->traj, (size_t)s->S * s->P, time, qpos, qvel, warm, ctrl);
}

int ilqg_solver_get_traj(ilqg_solver* s, double* time, double* qpos, double* qvel, double* warm, double* ctrl) {
  if (!s) return fail(ILQG_ERR_ARG, "null solver");
  const HostModel& h = s->model->host;
  double* dst[5] = {time, qpos, qvel, warm, ctrl};
  const size_t fld[5] = {1, (size_t)h.nq, (size_t)h.nv, (size_t)h.nv, (size_t)h.nu};
  HIPCHK(s->sync_all());
  for (int f = 0; f < 5; f++)
    if (dst[f]) HIPCHK(hipMemcpy(dst[f], s->traj[f].p, (size_t)s->S * s->P * fld[f] * 8, hipMemcpyDeviceToHost));
  return ILQG_OK;
}

int ilqg_solver_set_gains(ilqg_solver* s, const double* K, const double* k) {
  if (!s) return fail(ILQG_ERR_ARG, "null solver");
  HIPCHK(s->sync_all());
  if (K) HIPCHK(hipMemcpy(s->K.p, K, s->K.n, hipMemcpyHostToDevice));
  if (k) HIPCHK(hipMemcpy(s->k.p, k, s->k.n, hipMemcpyHostToDevice));
  return ILQG_OK;
}

int ilqg_solver_get_gains(ilqg_solver* s, double* K, double* k) {
  if (!s) return fail(ILQG_ERR_ARG, "null solver");
  HIPCHK(s->sync_all());
  if (K) HIPCHK(hipMemcpy(K, s->K.p, s->K.n, hipMemcpyDeviceToHost));
  if (k) HIPCHK(hipMemcpy(k, s->k.p, s->k.n, hipMemcpyDeviceToHost));
  return ILQG_OK;
}

int ilqg_solver_get_deriv(ilqg_solver* s, double* deriv) {
  if (!s || !deriv) return fail(ILQG_ERR_ARG, "bad argument");
  HIPCHK(s->sync_all());
  HIPCHK(hipMemcpy2D(deriv, (size_t)s->D * 8, s->deriv.p, (size_t)s->Dp * 8, (size_t)s->D * 8, (size_t)s->S * s->P,
                     hipMemcpyDeviceToHost));
  return ILQG_OK;
}

int ilqg_solver_get_deriv_point(ilqg_solver* s, int seed, int point, double* deriv) {
  if (!s || !deriv || seed < 0 || seed >= s->S || point < 0 || point >= s->P) return fail(ILQG_ERR_ARG, "bad argument");
  HIPCHK(s->sync_all());
  HIPCHK(hipMemcpy(deriv, s->deriv.as<double>() + ((size_t)seed * s->P + point) * s->Dp, (size_t)s->D * 8,
                   hipMemcpyDeviceToHost));
  return ILQG_OK;
}

int ilqg_solver_set_deriv(ilqg_solver* s, const double* deriv) {
  if (!s || !deriv) return fail(ILQG_ERR_ARG, "bad argument");
  HIPCHK(s->sync_all());
  HIPCHK(hipMemcpy2D(s->deriv.p, (size_t)s->Dp * 8, deriv, (size_t)s->D * 8, (size_t)s->D * 8, (size_t)s->S * s->P,
                     hipMemcpyHostToDevice));
  return ILQG_OK;
}

int ilqg_solver_get_value(ilqg_solver* s, double* V, double* v) {
  if (!s) return fail(ILQG_ERR_ARG, "null solver");
  HIPCHK(s->sync_all());
  if (V) HIPCHK(hipMemcpy(V, s->V.p, s->V.n, hipMemcpyDeviceToHost));
  if (v) HIPCHK(hipMemcpy(v, s->v.p, s->v.n, hipMemcpyDeviceToHost));
  return ILQG_OK;
}

int ilqg_solver_get_costs(ilqg_solver* s, double* cost, int* selected) {
  if (!s) return fail(ILQG_ERR_ARG, "null solver");
  HIPCHK(s->sync_all());
  if (cost) HIPCHK(hipMemcpy(cost, s->cost_cand.p, s->cost_cand.n, hipMemcpyDeviceToHost));
  if (selected) HIPCHK(hipMemcpy(selected, s->sel.p, s->sel.n, hipMemcpyDeviceToHost));
  return ILQG_OK;
}

// a contiguous seed range [s0, s0+ns) of the solver, launched on `st`; every
// per-seed array is seed-major, so a range is the same kernels on offset pointers
struct SeedRange {
  int s0, ns;
  hipStream_t st;
  unsigned* sync;  // the range's own hand-off block (fused sweep)
  int grp = 0;     // its fault block: s->fault + 2 grp (seed groups)
};
static SeedRange whole(ilqg_solver* s) { return {0, s->S, s->stream, s->sync.as<unsigned>(), 0}; }
static TrajDev toff(TrajDev t, size_t pts, const HostModel& h) {
  return TrajDev{t.time + pts, t.qpos + pts * h.nq, t.qvel + pts * h.nv, t.warm + pts * h.nv, t.ctrl + pts * h.nu};
}

// rollout of every (seed, alpha) candidate of the range, then selection + setDInit
static hipError_t rollout_launch(ilqg_solver* s, const SeedRange& r, RollChunk ch);
static hipError_t fd_range_launch(ilqg_solver* s, int p0, int np, hipStream_t st);
static hipError_t forward_range(ilqg_solver* s, const SeedRange& r, hipEvent_t before_select = nullptr) {
  const ilqg_model* m = s->model;
  const HostModel& h = m->host;
  const size_t s0 = r.s0, P = s->P, A = s->A, nx = s->nx;
  TrajDev nom = toff(s->tview(s->traj), s0 * P, h), di = toff(s->tview(s->dinit), s0, h);
  const bool multi = s->A > 1;
  TrajDev outv = multi ? toff(s->tview(s->cand), s0 * A * P, h) : nom;
  const double* K = s->K.as<double>() + s0 * P * h.nu * nx;
  const double* k = s->k.as<double>() + s0 * P * h.nu;
  const double* qa = s->qfrc_applied.as<double>() + s0 * h.nv;
  const double* xf = s->xfrc_applied.as<double>() + s0 * 6 * h.nbody;
  double* cc = s->cost_cand.as<double>() + s0 * A;
  hipError_t e = rollout_launch(s, r, RollChunk{});
  if (e != hipSuccess) return e;
  if (before_select) {
    e = hipStreamWaitEvent(r.st, before_select, 0);
    if (e != hipSuccess) return e;
  }
  return s->timed(1, [&] {
    return launch_select(m->dm, r.ns, s->A, s->P, s->opts.select_mode, multi ? 1 : 0, cc, s->sel.as<int>() + s0,
                         s->cost_sel.as<double>() + s0, outv, nom, di, r.st);
  }, r.st);
}

// the rollout of every (seed, alpha) candidate of the range over ch's points
static hipError_t rollout_launch(ilqg_solver* s, const SeedRange& r, RollChunk ch) {
  const ilqg_model* m = s->model;
  const HostModel& h = m->host;
  const size_t s0 = r.s0, P = s->P, A = s->A, nx = s->nx;
  TrajDev nom = toff(s->tview(s->traj), s0 * P, h), di = toff(s->tview(s->dinit), s0, h);
  const bool multi = s->A > 1;
  TrajDev outv = multi ? toff(s->tview(s->cand), s0 * A * P, h) : nom;
  const double* K = s->K.as<double>() + s0 * P * h.nu * nx;
  const double* k = s->k.as<double>() + s0 * P * h.nu;
  const double* qa = s->qfrc_applied.as<double>() + s0 * h.nv;
  const double* xf = s->xfrc_applied.as<double>() + s0 * 6 * h.nbody;
  double* cc = s->cost_cand.as<double>() + s0 * A;
  if (ch.n_hi >= 0) ch.carry = toff(s->tview(s->carry), s0 * A, h);
  return s->timed(0, [&] {
    return launch_rollout_coop(m->dm, m->Lc, m->C, m->X, r.ns, s->A, s->P, nom, outv, multi ? 1 : 0, K, k,
                               s->alphas.as<double>(), di, qa, xf, 0, s->cview(), cc, r.st, ch);
  }, r.st);
}

// the pipelined iterate's resources (ILQG_PIPE_STREAMS sweep streams CU-masked
// away from the rollout's CUs, the chunk events, the carried state), created
// on first use
static hipError_t pipe_setup(ilqg_solver* s) {
  if (s->pipe_ready) return hipSuccess;
  const HostModel& h = s->model->host;
  const size_t S = s->S, P = s->P;
  const size_t fld[5] = {1, (size_t)h.nq, (size_t)h.nv, (size_t)h.nv, (size_t)h.nu};
  // the sweep streams leave CUs to the rollout: a rollout chunk's workgroup
  // (the humanoid's: 147 KB of LDS, a CU to itself) waited up to 13 ms for
  // sweep teams to free a whole CU (rocprofv3 kernel trace); one CU per seed,
  // spread over the chip, is never given to the sweep
  int ncu = 0;
  hipError_t e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, s->opts.device);
  if (e != hipSuccess) return e;
  // (ILQG_PIPE_KEEP: how many; ILQG_PIPE_LOW: 1 the lowest-numbered mask
  // bits, which KFD deals round-robin over the XCDs (bit c -> XCD c % 8), so
  // ncu / 8 of them are four CUs on every XCD; 2 the CUs of one XCD (bits
  // c % 8 == 0), an L2 of the rollout's own; 0 spread evenly by bit).
  // Default: the lowest ncu / 8: cfg 5 rollout chunks 212 -> 177 us per step
  // beside the sweep (profiles/r05_cfg5_pipeline.txt)
  const int keep = std::min(getenv_int("ILQG_PIPE_KEEP", std::max((int)S, ncu / 8)), ncu / 4);
  const int low = getenv_int("ILQG_PIPE_LOW", 1);
  const int nxcd = (ncu >= 64 && ncu % 8 == 0) ? 8 : 1;
  std::vector<uint32_t> fmask((ncu + 31) / 32, 0);
  for (int c = 0, j = 0; c < ncu; c++) {
    bool r;
    if (low == 1) r = c < keep;
    else if (low == 2) r = j < keep && c % nxcd == 0;
    else r = j < keep && (long)c * keep / ncu >= j;  // spread evenly by bit
    if (r) j++;
    else fmask[c / 32] |= 1u << (c % 32);
  }
  for (int f = 0; f < s->nfd; f++) {
    hipStream_t& fs = s->fd_stream[f];
    if (fs) continue;  // (a retry after a failed setup)
    e = keep > 0 ? hipExtStreamCreateWithCUMask(&fs, (uint32_t)fmask.size(), fmask.data())
                 : hipStreamCreateWithFlags(&fs, hipStreamNonBlocking);
    if (e != hipSuccess) return e;
  }
  for (int f = 0; f < 5; f++) {
    if (s->carry[f].p) continue;
    e = s->carry[f].alloc(S * fld[f] * 8);
    if (e != hipSuccess) return e;
  }
  const int nch = ((int)P + s->pipe_chunk - 1) / s->pipe_chunk + 32 + ilqg_solver::kFdStreams;
  s->pipe_ev.resize(nch, nullptr);
  for (auto& ev : s->pipe_ev) {
    if (ev) continue;
    e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (e != hipSuccess) return e;
  }
  s->pipe_ready = true;
  return hipSuccess;
}

// the pipelined rollout's chunks in launch order, (lo, hi) point ranges
// descending from P - 1 (the rollout runs n = N .. 0, inc/ilqr.h:120): C
// points each (flat), or C halving toward the end (ILQG_PIPE_FLAT=0: a small
// last chunk's sweep takes about one team's latency)
static void pipe_chunks(int P, int C, bool flat, std::vector<std::pair<int, int>>& out) {
  out.clear();
  for (int hi = P - 1, n; hi >= 0; hi -= n) {
    const int rem = hi + 1;
    n = rem >= 2 * C ? C : (rem + 1) / 2;
    if (n < 1) n = 1;
    if (flat) n = C;
    out.emplace_back(hi - n + 1 > 0 ? hi - n + 1 : 0, hi);
  }
}

// Which of `world` ranks differentiates each point when one seed's FD sweep
// is sharded behind the pipelined rollout (flat chunks of C points): chunk c
// (launch order) goes to rank c % world, except the last kShardTail chunks --
// the sweep the recursion waits for once the rollout ends -- whose points
// [0, T) are dealt in contiguous blocks, rank r taking [T r / world,
// T (r + 1) / world).  Every rank sweeps behind the rollout as the one-GPU
// pipeline does, and the tail's latency is split world ways.
static constexpr int kShardTail = 2;
static void point_owners(int P, int C, int world, int* owner) {
  std::vector<std::pair<int, int>> ch;
  pipe_chunks(P, C, true, ch);
  const int nch = (int)ch.size(), tail = std::min(kShardTail, nch);
  const int T = ch[nch - tail].second + 1;
  for (int c = 0; c < nch; c++)
    for (int p = ch[c].first; p <= ch[c].second; p++)
      owner[p] = c < nch - tail ? c % world : (int)((long)p * world / T);
}

// iterate() with one candidate per seed and the unfused sweep: the rollout in
// chunks of pipe_chunk points (descending, as the rollout runs), and behind
// each chunk, on fd_stream, the FD sweep of the points it finished -- every
// point's record depends only on its own trajectory entry, so the sweep runs
// under the (latency-bound, one-workgroup-per-seed) rollout instead of after
// it; then selection / setDInit and the recursion once every record is in.
// The same launches' work as ilqg_forward + ilqg_fd_sweep + ilqg_backward:
// the same bits (tests/test_gpu_parity.py::test_pipelined_iterate).
//
// Point sharding (one seed's sweep over `world` ranks, BASELINE.json
// configs[4]): every rank runs the whole rollout and differentiates, behind
// each chunk, only the points it owns (point_owner); the records of the other
// points come from the other ranks (an all-gather by the caller), then
// ilqg_backward.  `backward` false stops after selection with the solver's
// stream behind every sweep launch.
static int iterate_pipelined(ilqg_solver* s, int rank = 0, int world = 1, bool backward = true) {
  const ilqg_model* m = s->model;
  const SeedRange r = whole(s);
  const int P = s->P, C = s->pipe_chunk;
  HIPCHK(pipe_setup(s));
  int ev = 0;
  std::vector<std::pair<int, int>> chunks;
  pipe_chunks(P, C, s->pipe_flat, chunks);
  std::vector<int> owner(P, 0);
  if (world > 1) point_owners(P, C, world, owner.data());
  for (const auto& c : chunks) {
    const int lo = c.first, hi = c.second;
    RollChunk ch;
    ch.n_hi = hi;
    ch.n_lo = lo;
    HIPCHK(rollout_launch(s, r, ch));
    // this rank's points of the chunk: all of them, none, or one contiguous run
    int plo = hi + 1, phi = lo - 1;
    for (int p = lo; p <= hi; p++)
      if (owner[p] == rank) plo = std::min(plo, p), phi = std::max(phi, p);
    if (plo > phi) continue;
    HIPCHK(hipEventRecord(s->pipe_ev[ev], s->stream));
    hipStream_t fs = s->fd_stream[ev % s->nfd];
    HIPCHK(hipStreamWaitEvent(fs, s->pipe_ev[ev], 0));
    ev++;
    HIPCHK(s->timed(3, [&] { return fd_range_launch(s, plo, phi - plo + 1, fs); }, fs));
  }
  // selection + setDInit (one candidate: the rollout wrote the nominal trajectory)
  const TrajDev nom = s->tview(s->traj), di = s->tview(s->dinit);
  HIPCHK(s->timed(1, [&] {
    return launch_select(m->dm, s->S, s->A, s->P, s->opts.select_mode, 0, s->cost_cand.as<double>(),
                         s->sel.as<int>(), s->cost_sel.as<double>(), nom, nom, di, s->stream);
  }));
  for (auto fs : s->fd_stream) {
    if (!fs) continue;
    HIPCHK(hipEventRecord(s->pipe_ev[ev], fs));
    HIPCHK(hipStreamWaitEvent(s->stream, s->pipe_ev[ev], 0));
    ev++;
  }
  if (!backward) {
    s->grp_join = true;
    return ILQG_OK;
  }
  return ilqg_backward(s);
}

int ilqg_forward_sharded(ilqg_solver* s, int rank, int world) {
  if (!s || !s->initialized) return fail(ILQG_ERR_ARG, "solver not initialised");
  if (world < 1 || rank < 0 || rank >= world) return fail(ILQG_ERR_ARG, "rank outside [0, world)");
  if (s->pipe_chunk <= 0 || !s->pipe_flat || s->fused)
    return fail(ILQG_ERR_UNSUPPORTED, "point sharding rides the pipelined iterate (one candidate per seed, the "
                                      "unfused sweep: fp32 FD or the MFMA recursion, flat chunks)");
  return iterate_pipelined(s, rank, world, false);
}

int ilqg_solver_point_owners(ilqg_solver* s, int world, int* owner) {
  if (!s || !owner || world < 1) return fail(ILQG_ERR_ARG, "bad argument");
  if (s->pipe_chunk <= 0 || !s->pipe_flat) return fail(ILQG_ERR_UNSUPPORTED, "no pipelined iterate on this solver");
  point_owners(s->P, s->pipe_chunk, world, owner);
  return ILQG_OK;
}

int ilqg_point_owners(int npoint, int chunk, int world, int* owner) {
  if (npoint < 1 || chunk < 1 || world < 1 || !owner) return fail(ILQG_ERR_ARG, "bad argument");
  point_owners(npoint, chunk, world, owner);
  return ILQG_OK;
}

int ilqg_forward(ilqg_solver* s) {
  if (!s || !s->initialized) return fail(ILQG_ERR_ARG, "solver not initialised");
  s->grp_join = true;
  HIPCHK(forward_range(s, whole(s)));
  return ILQG_OK;
}

// the fused sweep over a seed range: its hand-off words zeroed on the stream first
// mode: 0 the sweep alone, 1 the sweep with the backward roles streamed behind it
// the range's hand-off words and its launch fault word (handoff.h; the report
// word survives until read), zeroed on the range's stream
static hipError_t fused_zero(ilqg_solver* s, const SeedRange& r) {
  const size_t ntm = (size_t)s->nut + 2 * (size_t)s->model->host.nv;
  hipError_t e = hipMemsetAsync(r.sync, 0, sync_bytes((size_t)r.ns * s->P, ntm), r.st);
  if (e != hipSuccess) return e;
  return hipMemsetAsync(s->fault.as<unsigned>() + 2 * r.grp + 1, 0, sizeof(unsigned), r.st);
}
static hipError_t fused_launch(ilqg_solver* s, const SeedRange& r, int mode, bool zero = true) {
  const ilqg_model* m = s->model;
  const HostModel& h = m->host;
  const size_t s0 = r.s0, P = s->P, nx = s->nx;
  const size_t ntm = (size_t)s->nut + 2 * (size_t)h.nv;
  hipError_t e = zero ? fused_zero(s, r) : hipSuccess;
  if (e != hipSuccess) return e;
  unsigned* fault = s->fault.as<unsigned>() + 2 * r.grp;
  FdFused a{};
  a.tr = toff(s->tview(s->traj), s0 * P, h);
  a.S = r.ns;
  a.P = s->P;
  a.nB = mode ? r.ns : 0;
  a.nv = h.nv;
  a.nut = s->nut;
  a.Dp = s->Dp;
  a.WCp = s->WCp;
  a.qfrc_applied = s->qfrc_applied.as<double>() + s0 * h.nv;
  a.xfrc_applied = s->xfrc_applied.as<double>() + s0 * 6 * h.nbody;
  a.cost = s->cview();
  a.cw = s->cw.as<double>() + s0 * P * s->WCp;
  a.deriv = s->deriv.as<double>() + s0 * P * s->Dp;
  a.sync = r.sync;
  a.fault = fault;
  a.mu = s->opts.mu;
  a.K = s->K.as<double>() + s0 * P * h.nu * nx;
  a.k = s->k.as<double>() + s0 * P * h.nu;
  a.V = s->V.as<double>() + s0 * nx * nx;
  a.v = s->v.as<double>() + s0 * nx;
  a.fl = s->flags();
  {
    // FD teams' issue priority by ticket slot (permille of the FD items; 0 = off)
    const unsigned nit = (unsigned)(r.ns * s->P * (1 + (s->halves ? 2 : 1) * (s->nut + 2 * h.nv)));
    const int p1 = getenv_int("ILQG_FD_PRIO1", 0), p2 = getenv_int("ILQG_FD_PRIO2", 0);
    a.prio1 = p1 > 0 ? (unsigned)((unsigned long long)nit * p1 / 1000) : ~0u;
    a.prio2 = p2 > 0 ? (unsigned)((unsigned long long)nit * p2 / 1000) : ~0u;
  }
  if (s->snap.p && s->snap_on) {
    a.snap = s->snap.as<double>() + s0 * P * (size_t)s->snapd;
    a.snapd = s->snapd;
    a.poison = s->snap_poison ? 1 : 0;
  }
  if (s->halves) {
    a.halves = 1;
    a.xq = s->xq.as<double>() + s0 * P * ntm * 2 * h.nv;
    a.pairc = r.sync + 4 + 3 * (size_t)r.ns * P;
  }
  // ticket schedule from the previous launch's item durations: opt-in
  // (ILQG_PLAN=1); measured slower than the point-major order on the bench
  // workload ("Fused sweep ticket schedule")
  // Every map the sweep reads is validated first (launch_fd_order_check): an
  // invalid one is replaced by the identity and reported by ilqg_synchronize.
  const int nt = (s->halves ? 2 : 1) * (s->nut + 2 * h.nv);
  // (one ticket map per solver: seed groups run the identity order)
  if (s->plan_dur.p && (s->plan_on || !s->plants.empty()) && s->ngroups == 1) {
    if (s->plan_on) {
      e = launch_fd_plan(r.ns, s->P, nt, s->plan_p0, s->plan_k, s->plan_dur.as<unsigned>(),
                         s->plan_order.as<unsigned>(), r.st);
      if (e != hipSuccess) return e;
      a.dur = s->plan_dur.as<unsigned>();
    } else {
      std::vector<unsigned> id((size_t)r.ns * P * (1 + nt));
      for (size_t u = 0; u < id.size(); u++) id[u] = (unsigned)u;
      e = hipMemcpyAsync(s->plan_order.p, id.data(), id.size() * 4, hipMemcpyHostToDevice, r.st);
      if (e != hipSuccess) return e;
      e = hipStreamSynchronize(r.st);  // id is a host temporary
      if (e != hipSuccess) return e;
    }
    for (const auto& pl : s->plants) {
      e = hipMemcpyAsync(s->plan_order.as<unsigned>() + pl.first, &pl.second, 4, hipMemcpyHostToDevice, r.st);
      if (e != hipSuccess) return e;
    }
    if (!s->plants.empty()) {
      e = hipStreamSynchronize(r.st);
      s->plants.clear();
      if (e != hipSuccess) return e;
    }
    e = launch_fd_order_check(r.ns, s->P, nt, s->plan_order.as<unsigned>(), s->plan_pos.as<unsigned>(), fault,
                              r.st);
    if (e != hipSuccess) return e;
    a.order = s->plan_order.as<unsigned>();
  }
  return launch_fd_fused_coop(m->dm, m->Lc, m->C, m->X, a, r.st);
}

int ilqg_fd_sweep(ilqg_solver* s) {
  if (!s || !s->initialized) return fail(ILQG_ERR_ARG, "solver not initialised");
  s->grp_join = true;
  const ilqg_model* m = s->model;
  TrajDev nom = s->tview(s->traj);
  const int npts = s->S * s->P;
  if (s->fused) {
    HIPCHK(s->timed(3, [&] { return fused_launch(s, whole(s), 0); }));
    return ILQG_OK;
  }
  if (s->fdprec == ILQG_FD_F32) {
    HIPCHK(s->timed(3, [&] {
      return launch_fd_sweep_f32(m->dm, m->Lc, m->C, m->X, nom, npts, s->P, s->qfrc_applied.as<double>(),
                                 s->xfrc_applied.as<double>(), s->cview(), s->warm_c.as<double>(),
                                 s->cost_c.as<double>(), s->deriv.as<double>(), s->Dp, ILQG_FD32_EPS, s->stream);
    }));
    return ILQG_OK;
  }
  HIPCHK(s->timed(2, [&] {
    return launch_fd_centre_coop(m->dm, m->Lc, m->C, m->X, nom, npts, s->P, s->qfrc_applied.as<double>(),
                                 s->xfrc_applied.as<double>(), s->cview(), s->warm_c.as<double>(),
                                 s->cost_c.as<double>(), s->stream);
  }));
  HIPCHK(s->timed(3, [&] {
    return launch_fd_cols_coop(m->dm, m->Lc, m->C, m->X, nom, npts, s->P, s->qfrc_applied.as<double>(),
                               s->xfrc_applied.as<double>(), s->cview(), s->warm_c.as<double>(),
                               s->cost_c.as<double>(), s->deriv.as<double>(), s->Dp, s->stream);
  }));
  return ILQG_OK;
}

// calcMJDerivatives at points p0 .. p0 + np - 1 of every seed: the share of
// one rank in a point-sharded sweep (a single seed's FD sweep spread over
// GPUs; the records are then all-gathered and every rank runs the recursion).
// The unfused kernels of the solver's FD precision, one launch pair per seed;
// the same records the whole-trajectory sweep writes.
static hipError_t fd_range_launch(ilqg_solver* s, int p0, int np, hipStream_t st) {
  const ilqg_model* m = s->model;
  const HostModel& h = m->host;
  constexpr int kOneSeed = 1 << 30;  // the kernels' seed index pt / P is 0 for every point of the range
  for (int sd = 0; sd < s->S; sd++) {
    const size_t pt0 = (size_t)sd * s->P + p0;
    const TrajDev nom = toff(s->tview(s->traj), pt0, h);
    const double* qa = s->qfrc_applied.as<double>() + (size_t)sd * h.nv;
    const double* xa = s->xfrc_applied.as<double>() + (size_t)sd * 6 * h.nbody;
    double* wc = s->warm_c.as<double>() + pt0 * h.nv;
    double* cc = s->cost_c.as<double>() + pt0;
    double* dv = s->deriv.as<double>() + pt0 * s->Dp;
    hipError_t e;
    if (s->fdprec == ILQG_FD_F32) {
      e = launch_fd_sweep_f32(m->dm, m->Lc, m->C, m->X, nom, np, kOneSeed, qa, xa, s->cview(), wc, cc, dv, s->Dp,
                              ILQG_FD32_EPS, st);
    } else {
      e = launch_fd_centre_coop(m->dm, m->Lc, m->C, m->X, nom, np, kOneSeed, qa, xa, s->cview(), wc, cc, st);
      if (e == hipSuccess)
        e = launch_fd_cols_coop(m->dm, m->Lc, m->C, m->X, nom, np, kOneSeed, qa, xa, s->cview(), wc, cc, dv, s->Dp,
                                st);
    }
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

int ilqg_fd_sweep_range(ilqg_solver* s, int p0, int np) {
  if (!s || !s->initialized) return fail(ILQG_ERR_ARG, "solver not initialised");
  if (p0 < 0 || np < 0 || p0 + np > s->P) return fail(ILQG_ERR_ARG, "point range outside the trajectory");
  if (!np) return ILQG_OK;
  s->grp_join = true;
  HIPCHK(s->timed(3, [&] { return fd_range_launch(s, p0, np, s->stream); }));
  return ILQG_OK;
}

int ilqg_solver_device_deriv(ilqg_solver* s, double** dptr, int* stride) {
  if (!s || !dptr) return fail(ILQG_ERR_ARG, "bad argument");
  *dptr = s->deriv.as<double>();
  if (stride) *stride = s->Dp;
  return ILQG_OK;
}

int ilqg_backward(ilqg_solver* s) {
  if (!s || !s->initialized) return fail(ILQG_ERR_ARG, "solver not initialised");
  s->grp_join = true;
  const ilqg_model* m = s->model;
  HIPCHK(s->timed(4, [&] {
    if (s->riccati == ILQG_RICCATI_MFMA)
      return launch_backward_mfma(m->dm, s->S, s->P, s->opts.mu, s->deriv.as<double>(), s->Dp, s->tview(s->traj),
                                  s->K.as<double>(), s->k.as<double>(), s->V.as<double>(), s->v.as<double>(),
                                  s->flags(), s->stream);
    return launch_backward(m->dm, s->S, s->P, s->opts.mu, s->deriv.as<double>(), s->Dp, s->tview(s->traj),
                           s->K.as<double>(), s->k.as<double>(), s->V.as<double>(), s->v.as<double>(), s->flags(),
                           s->stream);
  }));
  s->vinit_pending = false;
  return ILQG_OK;
}

// iterate() over seed groups (ilqg_solver_set_groups): per group, its rollout +
// selection on its rollout stream, then its fused sweep on its sweep stream;
// the group's next rollout waits for that sweep (the gains), and group g's
// rollout for group g - 1's (which re-creates the stagger after any drain).
// The solver's stream waits for every group, so work enqueued on it after
// iterate() sees this iteration's results; the groups wait for the solver's
// stream only on the first grouped iterate after work was enqueued on it
// through the solver (grp_join) -- see INTEGRATION.md.
static int iterate_groups(ilqg_solver* s) {
  const int G = s->ngroups;
  if (s->grp_join) {
    for (int g = 0; g < G; g++) HIPCHK(hipEventRecord(s->grp_done[g], s->stream));
    s->grp_join = false;
    s->grp_sel_join = false;
  }
  hipEvent_t sel_wait = nullptr;
  if (s->grp_sel_join) {
    HIPCHK(hipEventRecord(s->grp_ext, s->stream));
    sel_wait = s->grp_ext;
    s->grp_sel_join = false;
  }
  for (int g = 0; g < G; g++) {
    const int s0 = s->S * g / G, s1 = s->S * (g + 1) / G;
    SeedRange r{s0, s1 - s0, s->grp_roll[g],
                reinterpret_cast<unsigned*>(static_cast<char*>(s->grp_sync.p) + g * s->grp_sync_stride), g};
    HIPCHK(hipStreamWaitEvent(r.st, s->grp_done[g], 0));
    if (g > 0) HIPCHK(hipStreamWaitEvent(r.st, s->grp_sel[g - 1], 0));
    HIPCHK(forward_range(s, r, sel_wait));
    HIPCHK(hipEventRecord(s->grp_sel[g], r.st));
    r.st = s->grp_fd[g];
    HIPCHK(hipStreamWaitEvent(r.st, s->grp_sel[g], 0));
    // the sweep with the group's recursion streamed behind it: one launch
    HIPCHK(s->timed(5, [&] { return fused_launch(s, r, 1); }, r.st));
    HIPCHK(hipEventRecord(s->grp_done[g], r.st));
  }
  for (int g = 0; g < G; g++) HIPCHK(hipStreamWaitEvent(s->stream, s->grp_done[g], 0));
  s->vinit_pending = false;
  return ILQG_OK;
}

int ilqg_iterate(ilqg_solver* s) {
  if (!s || !s->initialized) return fail(ILQG_ERR_ARG, "solver not initialised");
  if (s->ngroups > 1 && s->fused) return iterate_groups(s);
  if (!s->fused && s->pipe_chunk > 0) return iterate_pipelined(s);
  int rc = ilqg_forward(s);
  if (rc) return rc;
  if (s->fused) {
    // FD sweep with the Riccati recursion of every seed streamed behind it (one launch)
    HIPCHK(s->timed(5, [&] { return fused_launch(s, whole(s), 1); }));
    s->vinit_pending = false;
    return ILQG_OK;
  }
  rc = ilqg_fd_sweep(s);
  if (rc) return rc;
  return ilqg_backward(s);
}

int ilqg_synchronize(ilqg_solver* s) {
  if (!s) return fail(ILQG_ERR_ARG, "null solver");
  HIPCHK(s->sync_all());
  // every seed group's report word (fault block g at 2 g)
  unsigned blk[2 * ilqg_solver::kMaxGroups] = {};
  HIPCHK(hipMemcpy(blk, s->fault.p, sizeof(blk), hipMemcpyDeviceToHost));
  unsigned flt = 0;
  for (int g = 0; g < ilqg_solver::kMaxGroups; g++) flt |= blk[2 * g];
  if (flt) {
    // reported once: cleared by the read (the next launch waits normally)
    for (int g = 0; g < ilqg_solver::kMaxGroups; g++) HIPCHK(hipMemset(s->fault.as<unsigned>() + 2 * g, 0, 4));
    if (flt == 2u)
      return fail(ILQG_ERR_HIP, "fused FD sweep: invalid ticket schedule (item out of range, repeated, or a column "
                                "before its centre); the sweep ran in the identity order");
    return fail(ILQG_ERR_HIP, "fused FD sweep: a hand-off wait timed out");
  }
  return ILQG_OK;
}

int ilqg_solver_device_traj(ilqg_solver* s, int field, double** dptr) {
  if (!s || !dptr || field < 0 || field > 4) return fail(ILQG_ERR_ARG, "bad argument");
  *dptr = s->traj[field].as<double>();
  return ILQG_OK;
}

int ilqg_selftest_div(const double* a, const double* b, double* q, double* q2, int n) {
  if (!a || !b || !q || n < 0 || n > (1 << 24)) return fail(ILQG_ERR_ARG, "bad argument");
  if (!n) return ILQG_OK;
  const size_t bytes = (size_t)n * 8;
  DevBuf da, db, dq, dq2;
  HIPCHK(da.alloc(bytes));
  HIPCHK(db.alloc(bytes));
  HIPCHK(dq.alloc(bytes));
  if (q2) HIPCHK(dq2.alloc(bytes));
  HIPCHK(hipMemcpy(da.p, a, bytes, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(db.p, b, bytes, hipMemcpyHostToDevice));
  HIPCHK(launch_selftest_div((const double*)da.p, (const double*)db.p, (double*)dq.p, (double*)dq2.p, n, nullptr));
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(q, dq.p, bytes, hipMemcpyDeviceToHost));
  if (q2) HIPCHK(hipMemcpy(q2, dq2.p, bytes, hipMemcpyDeviceToHost));
  return ILQG_OK;
}

int ilqg_solver_debug_set_fault(ilqg_solver* s, unsigned value) {
  if (!s) return fail(ILQG_ERR_ARG, "null solver");
  HIPCHK(s->sync_all());
  HIPCHK(hipMemcpy(s->fault.p, &value, 4, hipMemcpyHostToDevice));
  return ILQG_OK;
}

void* ilqg_solver_stream(ilqg_solver* s) { return s ? (void*)s->stream : nullptr; }

int ilqg_solver_debug_plan(ilqg_solver* s, unsigned* order, unsigned* dur, int* nitems) {
  if (!s || !nitems) return fail(ILQG_ERR_ARG, "bad argument");
  const HostModel& h = s->model->host;
  const int n = s->plan_dur.p ? (int)(s->plan_dur.n / 4) : 0;
  *nitems = n;
  if (!n || (!order && !dur)) return ILQG_OK;
  HIPCHK(s->sync_all());
  HIPCHK(launch_fd_plan(s->S, s->P, (s->halves ? 2 : 1) * (s->nut + 2 * h.nv), s->plan_p0, s->plan_k,
                        s->plan_dur.as<unsigned>(), s->plan_order.as<unsigned>(), s->stream));
  HIPCHK(s->sync_all());
  if (order) HIPCHK(hipMemcpy(order, s->plan_order.p, (size_t)n * 4, hipMemcpyDeviceToHost));
  if (dur) HIPCHK(hipMemcpy(dur, s->plan_dur.p, (size_t)n * 4, hipMemcpyDeviceToHost));
  return ILQG_OK;
}

int ilqg_solver_debug_plant_schedule(ilqg_solver* s, unsigned slot, unsigned item) {
  if (!s) return fail(ILQG_ERR_ARG, "null solver");
  if (!s->plan_order.p) return fail(ILQG_ERR_UNSUPPORTED, "no fused sweep on this solver");
  if ((size_t)slot >= s->plan_order.n / 4) return fail(ILQG_ERR_ARG, "slot out of range");
  s->plants.emplace_back(slot, item);
  return ILQG_OK;
}

int ilqg_solver_set_mu(ilqg_solver* s, double mu) {
  if (!s || !(mu == mu)) return fail(ILQG_ERR_ARG, "bad argument");
  HIPCHK(s->sync_all());  // launches already enqueued keep the value they were given
  s->opts.mu = mu;
  return ILQG_OK;
}

int ilqg_solver_set_stream(ilqg_solver* s, void* stream) {
  if (!s) return fail(ILQG_ERR_ARG, "null solver");
  HIPCHK(s->sync_all());
  s->stream = stream ? (hipStream_t)stream : s->own_stream;
  s->grp_join = true;
  return ILQG_OK;
}

int ilqg_solver_set_timing(ilqg_solver* s, int enable) {
  if (!s) return fail(ILQG_ERR_ARG, "null solver");
  s->timing = enable != 0;
  return ILQG_OK;
}

int ilqg_solver_get_timing(ilqg_solver* s, double* ms, int* launches) {
  if (!s) return fail(ILQG_ERR_ARG, "null solver");
  HIPCHK(s->sync_all());
  for (int k = 0; k < ILQG_NKERNEL; k++) {
    double tot = 0;
    for (auto& p : s->ev[k]) {
      float t = 0;
      HIPCHK(hipEventElapsedTime(&t, p.first, p.second));
      tot += t;
      s->event_pool.push_back(p.first);
      s->event_pool.push_back(p.second);
    }
    if (ms) ms[k] = tot;
    if (launches) launches[k] = (int)s->ev[k].size();
    s->ev[k].clear();
  }
  return ILQG_OK;
}

int ilqg_solver_set_riccati(ilqg_solver* s, int mode) {
  if (!s || (mode != ILQG_RICCATI_EXACT && mode != ILQG_RICCATI_MFMA)) return fail(ILQG_ERR_ARG, "bad argument");
  const HostModel& h = s->model->host;
  if (mode == ILQG_RICCATI_MFMA) {
    if (!backward_mfma_supported(h.nv, h.nu))
      return fail(ILQG_ERR_UNSUPPORTED, "MFMA Riccati: nu <= 32, 2 nv + 1 <= 256, FD record <= 4096 doubles, LDS <= 160 KB");
  }
  HIPCHK(s->sync_all());
  s->riccati = mode;
  // the fused sweep streams the bit-exact recursion; the MFMA one runs after a
  // plain sweep (its workspace -- the hand-off block -- is allocated either way)
  s->fused = mode == ILQG_RICCATI_EXACT && s->fdprec == ILQG_FD_F64 && fused_ok(s->model) && s->sync.p;
  return ILQG_OK;
}

int ilqg_solver_set_fd_precision(ilqg_solver* s, int prec) {
  if (!s || (prec != ILQG_FD_F64 && prec != ILQG_FD_F32)) return fail(ILQG_ERR_ARG, "bad argument");
  if (prec == ILQG_FD_F32 && coop_lds_bytes_f32(s->model->Lc, s->model->C) > kMaxLds) return lds_fail();
  HIPCHK(s->sync_all());
  s->fdprec = prec;
  // the fused sweep is the fp64 one: fp32 FD runs the two-kernel sweep, then the recursion
  s->fused = s->riccati == ILQG_RICCATI_EXACT && prec == ILQG_FD_F64 && fused_ok(s->model) && s->sync.p;
  return ILQG_OK;
}

int ilqg_solver_set_layout(ilqg_solver* s, int layout) {
  if (!s || (layout != ILQG_LAYOUT_REFERENCE && layout != ILQG_LAYOUT_CORRECTED))
    return fail(ILQG_ERR_ARG, "bad argument");
  HIPCHK(s->sync_all());
  s->layout = layout;
  return ILQG_OK;
}

int ilqg_solver_set_value(ilqg_solver* s, const double* V, const double* v) {
  if (!s || !V || !v) return fail(ILQG_ERR_ARG, "bad argument");
  HIPCHK(s->sync_all());
  HIPCHK(hipMemcpy(s->V.p, V, s->V.n, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(s->v.p, v, s->v.n, hipMemcpyHostToDevice));
  s->vinit_pending = true;
  return ILQG_OK;
}

int ilqg_solver_set_groups(ilqg_solver* s, int ngroups) {
  if (!s || ngroups < 1 || ngroups > ilqg_solver::kMaxGroups || ngroups > s->S)
    return fail(ILQG_ERR_ARG, "ngroups must be in 1 .. min(4, nseed)");
  HIPCHK(s->sync_all());
  s->free_groups();
  s->grp_join = true;
  if (ngroups == 1) return ILQG_OK;
  if (!s->fused)
    return fail(ILQG_ERR_UNSUPPORTED, "seed groups pipeline the fused sweep (fp64 FD with the exact recursion)");
  const HostModel& h = s->model->host;
  const int G = ngroups;
  hipError_t e;
  auto bail = [&](hipError_t err, const char* w) {
    s->free_groups();
    return hip_fail(err, w);
  };
  // the CU masks: KFD deals mask bit c to XCD c % nxcd (MI355X: 8 XCDs of 32
  // CUs); a rollout workgroup holds a CU (k_rollout2: 480 registers a lane, one
  // wave per SIMD), so group g's rollout gets the XCDs [g k, g k + k) that hold
  // its ns * A workgroups, and every group's sweep all CUs but the other
  // groups' rollout XCDs.  Unmasked streams when the rollouts would take the
  // whole chip.
  int ncu = 0;
  e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, s->opts.device);
  if (e != hipSuccess) return bail(e, "hipDeviceGetAttribute");
  const int nxcd = (ncu >= 64 && ncu % 8 == 0) ? 8 : 1, per = ncu / nxcd;
  const int need = ((s->S + G - 1) / G) * s->A;
  const int k = (need + per - 1) / per;
  // default: the lowest mask bits (the group's rollout spread over every XCD):
  // measured ahead of a whole XCD per group (profiles/r05_seed_groups.txt)
  s->grp_xcd = getenv_int("ILQG_GROUP_XCD", 0);
  const bool masked = getenv_int("ILQG_GROUP_MASK", 1) != 0 && G * k < nxcd;
  s->grp_rcus = masked ? k * per : 0;
  auto rolls = [&](int g, int c) {  // CU c in group g's rollout set
    if (s->grp_xcd) return (c % nxcd) / k == g;
    return c / (k * per) == g;  // the lowest bits: spread over every XCD
  };
  for (int g = 0; g < G; g++) {
    if (masked) {
      std::vector<uint32_t> rm((ncu + 31) / 32, 0), fm((ncu + 31) / 32, 0);
      for (int c = 0; c < ncu; c++) {
        bool other = false;
        for (int o = 0; o < G; o++)
          if (o != g && rolls(o, c)) other = true;
        if (rolls(g, c)) rm[c / 32] |= 1u << (c % 32);
        if (!other) fm[c / 32] |= 1u << (c % 32);
      }
      e = hipExtStreamCreateWithCUMask(&s->grp_roll[g], (uint32_t)rm.size(), rm.data());
      if (e == hipSuccess) e = hipExtStreamCreateWithCUMask(&s->grp_fd[g], (uint32_t)fm.size(), fm.data());
    } else {
      e = hipStreamCreateWithFlags(&s->grp_roll[g], hipStreamNonBlocking);
      if (e == hipSuccess) e = hipStreamCreateWithFlags(&s->grp_fd[g], hipStreamNonBlocking);
    }
    if (e != hipSuccess) return bail(e, "hipStreamCreate");
    e = hipEventCreateWithFlags(&s->grp_sel[g], hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&s->grp_done[g], hipEventDisableTiming);
    if (e == hipSuccess && g == 0) e = hipEventCreateWithFlags(&s->grp_ext, hipEventDisableTiming);
    if (e != hipSuccess) return bail(e, "hipEventCreate");
  }
  const size_t ntm = (size_t)s->nut + 2 * (size_t)h.nv;
  s->grp_sync_stride = (sync_bytes((size_t)((s->S + G - 1) / G) * s->P, ntm) + 255) / 256 * 256;
  e = s->grp_sync.alloc(G * s->grp_sync_stride);
  if (e != hipSuccess) return bail(e, "hipMalloc");
  s->ngroups = G;
  return ILQG_OK;
}

int ilqg_solver_get_groups(ilqg_solver* s, int* ngroups, int* rollout_cus) {
  if (!s || !ngroups) return fail(ILQG_ERR_ARG, "bad argument");
  *ngroups = s->ngroups;
  if (rollout_cus) *rollout_cus = s->ngroups > 1 ? s->grp_rcus : 0;
  return ILQG_OK;
}

int ilqg_solver_join_stream(ilqg_solver* s) {
  if (!s) return fail(ILQG_ERR_ARG, "null solver");
  // with candidates the rollout writes only the candidate buffers, so the
  // selection is the first launch that rewrites what the caller may read;
  // with one candidate the rollout rewrites the nominal trajectory itself
  if (s->ngroups > 1 && s->A > 1 && s->grp_ext) s->grp_sel_join = true;
  else s->grp_join = true;
  return ILQG_OK;
}

int ilqg_solver_device_costs(ilqg_solver* s, double** dptr) {
  if (!s || !dptr) return fail(ILQG_ERR_ARG, "bad argument");
  *dptr = s->cost_sel.as<double>();
  return ILQG_OK;
}

}  // extern "C"
