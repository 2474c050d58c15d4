// Body of the cooperative device physics, included by dcoop.h (namespace
// coop, real = double: the bit-exact fp64 pipeline) and dcoop_f32.h
// (namespace coopf, real = float: the fp32 FD sweep of BASELINE.json cfg 5).
// Not a standalone header: the includer opens the namespace and defines
// `real`.  Model data stays fp64 (read and rounded where used); workspace,
// state and arithmetic on workspace values are `real`.
using namespace dev;

struct Team {
  real* w;   // WsLayout doubles (stride 1)
  int* iw;     // WsLayout ints
  real* c;   // CoopLayout doubles
  int* ci;     // CoopLayout ints
  int tid, nt;
};

// Team synchronisation: team_sync() (dsmall.h).
#define TSYNC() team_sync()

// diagnostic build only (-DILQG_STAMPS): per-stage s_memtime deltas of
// workgroup 0, lane 0, accumulated in LDS (a global read-modify-write per
// stamp would itself wait on memory) and flushed once at kernel end
#ifdef ILQG_STAMPS
#define STAMP_N 60  // ids 0..43 waves 0 and 1, 48..59 wave 2 (44..47: per-kernel counters)
#define STAMP_NG 64
// (per translation unit: the rollout and the FD kernels each read their own copy)
static __device__ unsigned long long g_stamp_acc[STAMP_NG];
static __device__ unsigned long long g_stamp_cnt[STAMP_NG];
static __device__ unsigned long long g_newton_iters;  // all workgroups: Newton iterations
static __device__ unsigned long long g_newton_calls;  // all workgroups: solver calls
// line searches of the wave-parallel Newton solver: [0] calls, [1] iterations,
// [2] calls that ran to LS_ITER, [3] constraint rows summed over the calls,
// [4] calls on the uniform-row form (ne <= LS_NE), [5] cycles in line searches,
// [6] cycles in fwd_constraint_fast, [7] FD team lifetimes (kernels_fd.hip)
static __device__ unsigned long long g_ls[8];
// the same counted per workgroup in LDS (lane 0 of wave 0) and added to the
// globals once when the workgroup ends: per-event global atomics from
// thousands of teams distorted the timings they measure ([8], [9]: Newton
// iterations and solver calls)
__shared__ unsigned long long s_cnt[10];
__device__ __forceinline__ void cnt_add_g(unsigned long long* g, unsigned long long v) {
  if (v) __hip_atomic_fetch_add(g, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void cnt_flush() {
  const unsigned long long c0 = s_cnt[0], c1 = s_cnt[1], c2 = s_cnt[2], c3 = s_cnt[3], c4 = s_cnt[4];
  const unsigned long long c5 = s_cnt[5], c6 = s_cnt[6], c7 = s_cnt[7], c8 = s_cnt[8], c9 = s_cnt[9];
  cnt_add_g(g_ls + 0, c0); cnt_add_g(g_ls + 1, c1); cnt_add_g(g_ls + 2, c2); cnt_add_g(g_ls + 3, c3);
  cnt_add_g(g_ls + 4, c4); cnt_add_g(g_ls + 5, c5); cnt_add_g(g_ls + 6, c6); cnt_add_g(g_ls + 7, c7);
  cnt_add_g(&g_newton_iters, c8); cnt_add_g(&g_newton_calls, c9);
}
#define CNT_ADD(i, v)                     \
  do {                                    \
    if (threadIdx.x == 0) __hip_atomic_fetch_add(&s_cnt[i], (unsigned long long)(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); \
  } while (0)
// the workgroups whose stamps are taken: block 0, or (ILQG_STAMP_SAMPLE = k) every
// 2^k-th block (the FD sweeps: a sample of all team roles)
#ifndef ILQG_STAMP_SAMPLE
#define ILQG_STAMP_SAMPLE 0
#endif
#define STAMP_BLOCK() ((blockIdx.x & ((1u << ILQG_STAMP_SAMPLE) - 1u)) == 0)
__shared__ unsigned long long s_stamp_acc[STAMP_N], s_stamp_cnt[STAMP_N], s_stamp_prev, s_stamp_prevb, s_stamp_prevc;
#define STAMP_AT(lane, prev, id)                                             \
  do {                                                                       \
    if (threadIdx.x == (lane) && STAMP_BLOCK()) {                            \
      unsigned long long t_ = __builtin_amdgcn_s_memtime();                  \
      if ((id) >= 0) {                                                       \
        s_stamp_acc[(id) < 0 ? 0 : (id)] += t_ - prev;                       \
        s_stamp_cnt[(id) < 0 ? 0 : (id)]++;                                  \
      }                                                                      \
      prev = t_;                                                             \
    }                                                                        \
  } while (0)
// wave 0 lane 0; STAMPB: lane 0 of the helper wave of a two-wave team
#define STAMP(id) STAMP_AT(0, s_stamp_prev, id)
#define STAMPB(id) STAMP_AT(64, s_stamp_prevb, id)
// STAMPC: lane 0 of the third wave of a three-wave team (ids 48..59)
#define STAMPC(id) STAMP_AT(128, s_stamp_prevc, id)
#define STAMP_INIT()                                                         \
  do {                                                                       \
    if (threadIdx.x == 0) {                                                  \
      for (int i_ = 0; i_ < 10; i_++) s_cnt[i_] = 0;                         \
      if (STAMP_BLOCK()) {                                                   \
        for (int i_ = 0; i_ < STAMP_N; i_++) s_stamp_acc[i_] = s_stamp_cnt[i_] = 0; \
        s_stamp_prev = s_stamp_prevb = s_stamp_prevc = __builtin_amdgcn_s_memtime();         \
      }                                                                      \
    }                                                                        \
  } while (0)
#define STAMP_FLUSH()                                                        \
  do {                                                                       \
    if (threadIdx.x == 0) {                                                  \
      cnt_flush();                                                           \
      if (STAMP_BLOCK())                                                     \
        for (int i_ = 0; i_ < STAMP_N; i_++)                                 \
          if (s_stamp_cnt[i_]) {                                             \
            cnt_add_g(&g_stamp_acc[i_], s_stamp_acc[i_]);                    \
            cnt_add_g(&g_stamp_cnt[i_], s_stamp_cnt[i_]);                    \
          }                                                                  \
    }                                                                        \
  } while (0)
#else
#define CNT_ADD(i, v) \
  do {                \
  } while (0)
#define STAMP(id) \
  do {            \
  } while (0)
#define STAMPB(id) STAMP(id)
#define STAMPC(id) STAMP(id)
#define STAMP_INIT() STAMP(-1)
#define STAMP_FLUSH() STAMP(-1)
#endif
#define FOR_T(v, n) for (int v = T.tid; v < (n); v += T.nt)

#ifndef KIN_SPLIT
#define KIN_SPLIT 1
#endif
// below this many dofs the small factorizations run on lane 0 (fewer LDS round trips)
constexpr int SERIAL_NV = 12;
// the Newton Hessian's build for compile-time dof counts: a lane per row block
// (HessLanes) instead of a lane per entry (0: the per-entry form, A/B)
#ifndef ILQG_HESS_ROWS
#define ILQG_HESS_ROWS 1
#endif
// the Newton Hessian's Cholesky in row registers up to 32 dofs (cholesky_rows32)
#ifndef ILQG_CHOL32
#define ILQG_CHOL32 1
#endif
// the Newton search-direction substitution for RMAX < nv <= 32: 0 chol_solve_wave,
// 1 chol_solve_rows32 (solution in registers), 2 chol_solve_u2 (compile-time steps)
#ifndef ILQG_CHOLS
#define ILQG_CHOLS 2
#endif

__device__ __forceinline__ real tdot(const real* a, const real* b, int n) {
  real r = 0;
  for (int i = 0; i < n; i++) r += a[i] * b[i];
  return r;
}
// sum_j (Ma_j - qfs_j)(qa_j - qas_j) in ascending order, four terms' loads in flight
__device__ __forceinline__ real gauss_w(const real* Ma, const real* qfs, const real* qa, const real* qas, int n) {
  real g = 0;
  int j = 0;
  for (; j + 4 <= n; j += 4) {
    real a[4], b[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      a[k] = Ma[j + k] - qfs[j + k];
      b[k] = qa[j + k] - qas[j + k];
    }
#pragma unroll
    for (int k = 0; k < 4; k++) g += a[k] * b[k];
  }
  for (; j < n; j++) g += (Ma[j] - qfs[j]) * (qa[j] - qas[j]);
  return g;
}
// the same sum for run-time n over LDS operands: the loads of eight terms are
// issued together (one LDS latency per eight terms instead of per term), the
// additions stay in ascending order from +0
__device__ __forceinline__ real tdotw(const real* a, const real* b, int n) {
  real r = 0;
  int i = 0;
  for (; i + 8 <= n; i += 8) {
    real x[8], y[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
      x[k] = a[i + k];
      y[k] = b[i + k];
    }
#pragma unroll
    for (int k = 0; k < 8; k++) r += x[k] * y[k];
  }
  for (; i < n; i++) r += a[i] * b[i];
  return r;
}

// ------------------------------------------------------ position stage ---
// model traits with compile-time sizes and tables (static_models.h)
template <class M>
concept StaticModel = requires { std::integral_constant<int, M::nbody>{}; };
// a run-time model whose dof count alone is a compile-time constant (the
// generic rollout kernel's instance for 27-dof models: the humanoid); the
// Newton Hessian's Cholesky and its substitution drop their size guards
template <int NV_>
struct DevModelNV : DevModel {
  static constexpr int kNV = NV_;
};
template <class M>
constexpr int nv_const() {
  if constexpr (requires { std::integral_constant<int, M::kNV>{}; }) return M::kNV;
  else return 0;
}

// rot_vec_quat / normalize4 with their special cases as selects instead of
// branches: the same doubles in every case (the general formula is computed
// and discarded where MuJoCo takes the shortcut), no exec-mask round trips on
// the serial chain
__device__ __forceinline__ void rot_vec_quat_sel(real* r, const real* v, const real* q) {
  const bool vz = v[0] == 0 && v[1] == 0 && v[2] == 0;
  const bool qi = q[0] == 1 && q[1] == 0 && q[2] == 0 && q[3] == 0;
  const real t0 = q[0] * v[0] + q[2] * v[2] - q[3] * v[1];
  const real t1 = q[0] * v[1] + q[3] * v[0] - q[1] * v[2];
  const real t2 = q[0] * v[2] + q[1] * v[1] - q[2] * v[0];
  const real r0 = v[0] + 2 * (q[2] * t2 - q[3] * t1);
  const real r1 = v[1] + 2 * (q[3] * t0 - q[1] * t2);
  const real r2 = v[2] + 2 * (q[1] * t1 - q[2] * t0);
  r[0] = vz ? 0.0 : (qi ? v[0] : r0);
  r[1] = vz ? 0.0 : (qi ? v[1] : r1);
  r[2] = vz ? 0.0 : (qi ? v[2] : r2);
}
__device__ __forceinline__ void normalize4_sel(real* q) {
  const real norm = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  const bool tiny = norm < MINVAL;
  const bool scale = !tiny && fabs(norm - 1) > MINVAL;
  const real inv = 1 / norm;
  const real s0 = q[0] * inv, s1 = q[1] * inv, s2 = q[2] * inv, s3 = q[3] * inv;
  q[0] = tiny ? 1.0 : (scale ? s0 : q[0]);
  q[1] = tiny ? 0.0 : (scale ? s1 : q[1]);
  q[2] = tiny ? 0.0 : (scale ? s2 : q[2]);
  q[3] = tiny ? 0.0 : (scale ? s3 : q[3]);
}

// normalize4_sel when the squared norm already decides that q stays as it is:
// |fl(sqrt(s)) - 1| <= MINVAL exactly for s in [S_LO, S_HI] (sqrt correctly
// rounded and monotone; the bounds are the ends of that run of doubles,
// tests/test_oracle_physics.py::test_normalize4_window).  Unit quaternion
// products land there almost always, so the chain skips the sqrt and divide.
constexpr real NORM4_S_LO = 0x1.fffffffffffeep-1, NORM4_S_HI = 0x1.0000000000009p+0;
__device__ __forceinline__ void normalize4_fast(real* q) {
  const real s = q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3];
  if (s >= NORM4_S_LO && s <= NORM4_S_HI) return;
  normalize4_sel(q);
}

// The kinematic chain of a compile-time model on lane 0 with every body frame
// in registers (no store->load round trip through LDS between a body and its
// children): the tree walk is unrolled with compile-time parent indices and
// joint types.  Same operations in the same order as the loop in kinematics().
template <class M>
__device__ inline void kin_chain_static(const M& m, const real* qpos, const real* qloc, real* xpos,
                                        real* xquat, real* xanchor, real* xaxis) {
  constexpr int NB = M::nbody;
  real xp[NB][3], xq[NB][4];
  xp[0][0] = xp[0][1] = xp[0][2] = 0;
  xq[0][0] = 1;
  xq[0][1] = xq[0][2] = xq[0][3] = 0;
  sfor<1, NB>(SLAM(ii) {
    constexpr int i = SK(ii);
    constexpr int pid = M::body_parentid[i];
    real tmp[3], bpos[3], bquat[4];
    ldm<3>(bpos, m.body_pos + 3 * i);
    ldm<4>(bquat, m.body_quat + 4 * i);
    rot_vec_quat_sel(tmp, bpos, xq[pid]);
    xp[i][0] = xp[pid][0] + tmp[0];
    xp[i][1] = xp[pid][1] + tmp[1];
    xp[i][2] = xp[pid][2] + tmp[2];
    quat_mul(xq[i], xq[pid], bquat);
    sfor<0, M::body_jntnum[i]>(SLAM(jj) {
      constexpr int jid = M::body_jntadr[i] + SK(jj);
      constexpr int type = M::jnt_type[jid], qadr = M::jnt_qposadr[jid];
      real jpos[3], jaxis[3];
      ldm<3>(jpos, m.jnt_pos + 3 * jid);
      ldm<3>(jaxis, m.jnt_axis + 3 * jid);
      if constexpr (type == JNT_FREE) {
        for (int k = 0; k < 3; k++) xp[i][k] = qpos[qadr + k];
        for (int k = 0; k < 4; k++) xq[i][k] = qpos[qadr + 3 + k];
        normalize4_sel(xq[i]);
        for (int k = 0; k < 3; k++) { xanchor[3 * jid + k] = xp[i][k]; xaxis[3 * jid + k] = jaxis[k]; }
      } else {
        real anc[3], ax[3];
        rot_vec_quat_sel(anc, jpos, xq[i]);
        anc[0] += xp[i][0]; anc[1] += xp[i][1]; anc[2] += xp[i][2];
        rot_vec_quat_sel(ax, jaxis, xq[i]);
        if constexpr (type == JNT_SLIDE) {
          const real dq = qpos[qadr] - m.qpos0[qadr];
          xp[i][0] += ax[0] * dq; xp[i][1] += ax[1] * dq; xp[i][2] += ax[2] * dq;
        } else {
          real ql[4];
          ldm<4>(ql, qloc + 4 * jid);
          quat_mul(xq[i], xq[i], ql);
          rot_vec_quat_sel(tmp, jpos, xq[i]);
          xp[i][0] = anc[0] - tmp[0];
          xp[i][1] = anc[1] - tmp[1];
          xp[i][2] = anc[2] - tmp[2];
        }
        for (int k = 0; k < 3; k++) { xanchor[3 * jid + k] = anc[k]; xaxis[3 * jid + k] = ax[k]; }
      }
    });
    normalize4_sel(xq[i]);
    for (int k = 0; k < 3; k++) xpos[3 * i + k] = xp[i][k];
    for (int k = 0; k < 4; k++) xquat[4 * i + k] = xq[i][k];
  });
  for (int k = 0; k < 3; k++) xpos[k] = 0;
  xquat[0] = 1;
  xquat[1] = xquat[2] = xquat[3] = 0;
}

// The same chain as kin_chain_static, split by dependency (compile-time models):
//   1. lane 0 walks the quaternion chain alone (body quat products, joint
//      rotations, normalisation) -- it never reads a position -- and parks
//      every quaternion a rotation below needs;
//   2. every vector rotation of the walk (body offsets, joint anchors, axes and
//      post-rotation anchors) runs on a lane of its own;
//   3. lane 0 walks the position chain: additions only.
// Each output is produced by the same operations in the same order as in
// kin_chain_static (and the oracle), only on another lane or earlier.
template <class M>
struct KinPlan {
  // rotation r: vector kind (0 body_pos, 1 jnt_pos, 2 jnt_axis) and index, quaternion
  // source (>= 0: parked slot, < 0: final quaternion of body -1 - src), role
  // (0 body offset, 1 anchor, 2 axis, 3 post-rotation anchor) and its joint
  static constexpr int MAXR = 64;
  int nrot = 0, nslot = 0;
  int vkind[MAXR] = {}, vidx[MAXR] = {}, qsrc[MAXR] = {}, role[MAXR] = {}, jnt[MAXR] = {};
  int body_rot[M::nbody > 0 ? M::nbody : 1] = {};            // rotation of body i's offset
  int anc_rot[M::njnt > 0 ? M::njnt : 1] = {}, ax_rot[M::njnt > 0 ? M::njnt : 1] = {},
      tmp_rot[M::njnt > 0 ? M::njnt : 1] = {};
  int qb_slot[M::nbody > 0 ? M::nbody : 1] = {};             // quat after the body quat (-1: not parked)
  int qj_slot[M::njnt > 0 ? M::njnt : 1] = {};               // quat after joint j's rotation (-1)
  bool ok = true;
  struct Packed {
    unsigned long long w[MAXR / 4];
    __host__ __device__ constexpr unsigned long long operator[](int i) const { return w[i]; }
  };
  constexpr Packed packed() const {
    Packed p{};
    for (int r = 0; r < nrot; r++) {
      const unsigned long long d = (unsigned long long)(vkind[r] | (vidx[r] << 2) | ((qsrc[r] + 64) << 9));
      p.w[r / 4] |= d << (16 * (r % 4));
    }
    return p;
  }
  constexpr KinPlan() {
    auto add = [&](int kind, int idx, int q, int rl, int j) {
      if (nrot >= MAXR) { ok = false; return 0; }
      vkind[nrot] = kind; vidx[nrot] = idx; qsrc[nrot] = q; role[nrot] = rl; jnt[nrot] = j;
      return nrot++;
    };
    for (int i = 0; i < M::nbody; i++) qb_slot[i] = -1;
    for (int j = 0; j < M::njnt; j++) qj_slot[j] = anc_rot[j] = ax_rot[j] = tmp_rot[j] = -1;
    for (int i = 1; i < M::nbody; i++) {
      body_rot[i] = add(0, i, -1 - M::body_parentid[i], 0, -1);
      int cur = -2;  // quaternion the next joint starts from: -2 = q_b (not parked yet)
      for (int jj = 0; jj < M::body_jntnum[i]; jj++) {
        const int j = M::body_jntadr[i] + jj, type = M::jnt_type[j];
        if (type == JNT_FREE) { cur = -3; continue; }  // no rotations; later joints unsupported
        if (cur == -3) { ok = false; continue; }
        if (cur == -2) { qb_slot[i] = nslot++; cur = qb_slot[i]; }
        anc_rot[j] = add(1, j, cur, 1, j);
        ax_rot[j] = add(2, j, cur, 2, j);
        if (type != JNT_SLIDE) {
          if (nslot >= 63 || j >= 127 || i >= 64) ok = false;
          qj_slot[j] = nslot++;
          cur = qj_slot[j];
          tmp_rot[j] = add(1, j, cur, 3, j);
        }
      }
    }
  }
};

template <class M, class F>
__device__ inline void kin_chain_par(const M& m, const Team& T, const real* qpos, const real* qloc, real* xpos,
                                     real* xquat, real* xanchor, real* xaxis, real* scratch,
                                     F&& after_quats) {
  static constexpr KinPlan<M> P{};
  constexpr int NB = M::nbody;
  real* QS = scratch;                 // parked quaternions, 4 per slot
  real* RS = scratch + 4 * P.nslot;   // rotation results, 3 per rotation
  // 1. quaternion chain (lane 0)
  if (T.tid == 0) {
    // every LDS operand of the walk is loaded up front: one wait, none inside the walk
    real bq[NB][4], ql[M::njnt > 0 ? M::njnt : 1][4];
    sfor<1, NB>(SLAM(ii) { ldm<4>(bq[SK(ii)], m.body_quat + 4 * SK(ii)); });
    sfor<0, M::njnt>(SLAM(jj) {
      constexpr int j = SK(jj);
      if constexpr (M::jnt_type[j] != JNT_FREE && M::jnt_type[j] != JNT_SLIDE) ldm<4>(ql[j], qloc + 4 * j);
    });
    real xq[NB][4];
    xq[0][0] = 1;
    xq[0][1] = xq[0][2] = xq[0][3] = 0;
    sfor<1, NB>(SLAM(ii) {
      constexpr int i = SK(ii);
      constexpr int pid = M::body_parentid[i];
      quat_mul(xq[i], xq[pid], bq[i]);
      if constexpr (P.qb_slot[i] >= 0)
        for (int k = 0; k < 4; k++) QS[4 * P.qb_slot[i] + k] = xq[i][k];
      sfor<0, M::body_jntnum[i]>(SLAM(jj) {
        constexpr int jid = M::body_jntadr[i] + SK(jj);
        constexpr int type = M::jnt_type[jid], qadr = M::jnt_qposadr[jid];
        if constexpr (type == JNT_FREE) {
          for (int k = 0; k < 4; k++) xq[i][k] = qpos[qadr + 3 + k];
          normalize4_fast(xq[i]);
        } else if constexpr (type != JNT_SLIDE) {
          quat_mul(xq[i], xq[i], ql[jid]);
          for (int k = 0; k < 4; k++) QS[4 * P.qj_slot[jid] + k] = xq[i][k];
        }
      });
      normalize4_fast(xq[i]);
      for (int k = 0; k < 4; k++) xquat[4 * i + k] = xq[i][k];
    });
    xquat[0] = 1;
    xquat[1] = xquat[2] = xquat[3] = 0;
  }
  team_sync();
  after_quats();  // every body quaternion is final
  STAMP(22);
  // 2. every rotation on a lane of its own
  if (T.tid < P.nrot) {
    // lane -> plan entry: 16-bit descriptors packed 4 per 64-bit immediate
    // (kind 2 bits | vector index 7 bits | quaternion source + 64 7 bits)
    static constexpr auto D = P.packed();
    const int l = T.tid;
    unsigned long long w = D[0];
    sfor<1, (P.nrot + 3) / 4>(SLAM(kk) { w = (l >> 2) == SK(kk) ? D[SK(kk)] : w; });
    const unsigned d = (unsigned)(w >> (16 * (l & 3))) & 0xffffu;
    const int kind = d & 3, idx = (d >> 2) & 127, q = (int)(d >> 9) - 64, j = idx;
    const int rl = kind == 2 ? 2 : 0;
    // integer offsets from one base each (a select between pointers becomes a
    // lookup table in scratch and a flat load)
    const int d1 = (int)(m.jnt_pos - m.body_pos), d2 = (int)(m.jnt_axis - m.body_pos);
    const real* v = m.body_pos + (3 * idx + (kind == 1 ? d1 : 0) + (kind == 2 ? d2 : 0));
    const int dq = (int)(xquat - QS);
    const real* qq = QS + (q >= 0 ? 4 * q : dq + 4 * (-1 - q));
    real vv[3], q4[4], r3[3];
    ldm<3>(vv, v);
    ldm<4>(q4, qq);
    rot_vec_quat_sel(r3, vv, q4);
    for (int k = 0; k < 3; k++) RS[3 * T.tid + k] = r3[k];
    if (rl == 2)
      for (int k = 0; k < 3; k++) xaxis[3 * j + k] = r3[k];
  }
  team_sync();
  STAMP(23);
  // 3. position chain (lane 0): the additions of kin_chain_static in its order
  if (T.tid == 0) {
    real R[P.nrot][3];
    sfor<0, P.nrot>(SLAM(rr) { ldm<3>(R[SK(rr)], RS + 3 * SK(rr)); });
    real xp[NB][3];
    xp[0][0] = xp[0][1] = xp[0][2] = 0;
    sfor<1, NB>(SLAM(ii) {
      constexpr int i = SK(ii);
      constexpr int pid = M::body_parentid[i];
      const real* tmp = R[P.body_rot[i]];
      xp[i][0] = xp[pid][0] + tmp[0];
      xp[i][1] = xp[pid][1] + tmp[1];
      xp[i][2] = xp[pid][2] + tmp[2];
      sfor<0, M::body_jntnum[i]>(SLAM(jj) {
        constexpr int jid = M::body_jntadr[i] + SK(jj);
        constexpr int type = M::jnt_type[jid], qadr = M::jnt_qposadr[jid];
        if constexpr (type == JNT_FREE) {
          real jaxis[3];
          ldm<3>(jaxis, m.jnt_axis + 3 * jid);
          for (int k = 0; k < 3; k++) xp[i][k] = qpos[qadr + k];
          for (int k = 0; k < 3; k++) { xanchor[3 * jid + k] = xp[i][k]; xaxis[3 * jid + k] = jaxis[k]; }
        } else {
          const real* ra = R[P.anc_rot[jid]];
          real anc[3];
          anc[0] = ra[0] + xp[i][0]; anc[1] = ra[1] + xp[i][1]; anc[2] = ra[2] + xp[i][2];
          if constexpr (type == JNT_SLIDE) {
            const real* ax = R[P.ax_rot[jid]];
            const real dq = qpos[qadr] - m.qpos0[qadr];
            xp[i][0] += ax[0] * dq; xp[i][1] += ax[1] * dq; xp[i][2] += ax[2] * dq;
          } else {
            const real* tmp2 = R[P.tmp_rot[jid]];
            xp[i][0] = anc[0] - tmp2[0];
            xp[i][1] = anc[1] - tmp2[1];
            xp[i][2] = anc[2] - tmp2[2];
          }
          for (int k = 0; k < 3; k++) xanchor[3 * jid + k] = anc[k];
        }
      });
      for (int k = 0; k < 3; k++) xpos[3 * i + k] = xp[i][k];
    });
    xpos[0] = xpos[1] = xpos[2] = 0;
  }
}

__device__ inline void kinematics(const auto& m, const auto& L, const auto& C, const Team& T) {
  real* qpos = T.w + L.qpos;
  real* xpos = T.w + L.xpos;
  real* xquat = T.w + L.xquat;
  real* xmat = T.w + L.xmat;
  real* xipos = T.w + L.xipos;
  real* ximat = T.w + L.ximat;
  real* xanchor = T.w + L.xanchor;
  real* xaxis = T.w + L.xaxis;
  real* qloc = T.c + C.qloc;
  // joint-local rotations depend on qpos only: all joints at once
  FOR_T(j, m.njnt) {
    int type = m.jnt_type[j], qadr = m.jnt_qposadr[j];
    real q[4], ja[3];
    if (type == JNT_HINGE) {
      ldm<3>(ja, m.jnt_axis + 3 * j);
      axis_angle2quat(q, ja, qpos[qadr] - m.qpos0[qadr]);
      for (int k = 0; k < 4; k++) qloc[4 * j + k] = q[k];
    } else if (type == JNT_BALL) {
      q[0] = qpos[qadr]; q[1] = qpos[qadr + 1]; q[2] = qpos[qadr + 2]; q[3] = qpos[qadr + 3];
      normalize4(q);
      for (int k = 0; k < 4; k++) qloc[4 * j + k] = q[k];
    }
  }
  TSYNC();
  STAMP(11);
  // the kinematic chain: lane 0
  using MT = std::remove_cvref_t<decltype(m)>;
  if constexpr (StaticModel<MT>) {
    static constexpr KinPlan<MT> plan{};
    // the split chain needs its scratch in the union (dead until collision) and a lane per rotation
    if constexpr (plan.ok && 4 * plan.nslot + 3 * plan.nrot <= 12 * MT::nbody + 10 * MT::nv && KIN_SPLIT)
      kin_chain_par(m, T, qpos, qloc, xpos, xquat, xanchor, xaxis, T.w + L.con, []() {});
    else if (T.tid == 0)
      kin_chain_static(m, qpos, qloc, xpos, xquat, xanchor, xaxis);
  } else {
    // body i from its parent's frame (the oracle's loop body)
    auto walk_body = [&](int i) {
      int pid = m.body_parentid[i];
      real xp[3], xq[4], tmp[3], pq[4], bp[3], bq[4];
      ldm<4>(pq, xquat + 4 * pid);
      ldm<3>(bp, m.body_pos + 3 * i);
      ldm<4>(bq, m.body_quat + 4 * i);
      rot_vec_quat(tmp, bp, pq);
      xp[0] = xpos[3 * pid] + tmp[0];
      xp[1] = xpos[3 * pid + 1] + tmp[1];
      xp[2] = xpos[3 * pid + 2] + tmp[2];
      quat_mul(xq, pq, bq);
      for (int j = 0; j < m.body_jntnum[i]; j++) {
        int jid = m.body_jntadr[i] + j;
        int qadr = m.jnt_qposadr[jid];
        int type = m.jnt_type[jid];
        real anc[3], ax[3], jp[3], ja[3];
        ldm<3>(jp, m.jnt_pos + 3 * jid);
        ldm<3>(ja, m.jnt_axis + 3 * jid);
        if (type == JNT_FREE) {
          xp[0] = qpos[qadr]; xp[1] = qpos[qadr + 1]; xp[2] = qpos[qadr + 2];
          xq[0] = qpos[qadr + 3]; xq[1] = qpos[qadr + 4]; xq[2] = qpos[qadr + 5]; xq[3] = qpos[qadr + 6];
          normalize4(xq);
          for (int k = 0; k < 3; k++) { xanchor[3 * jid + k] = xp[k]; xaxis[3 * jid + k] = ja[k]; }
          continue;
        }
        rot_vec_quat(anc, jp, xq);
        anc[0] += xp[0]; anc[1] += xp[1]; anc[2] += xp[2];
        rot_vec_quat(ax, ja, xq);
        if (type == JNT_SLIDE) {
          real dq = qpos[qadr] - m.qpos0[qadr];
          xp[0] += ax[0] * dq; xp[1] += ax[1] * dq; xp[2] += ax[2] * dq;
        } else {
          real ql[4];
          ldm<4>(ql, qloc + 4 * jid);
          quat_mul(xq, xq, ql);
          rot_vec_quat(tmp, jp, xq);
          xp[0] = anc[0] - tmp[0];
          xp[1] = anc[1] - tmp[1];
          xp[2] = anc[2] - tmp[2];
        }
        for (int k = 0; k < 3; k++) { xanchor[3 * jid + k] = anc[k]; xaxis[3 * jid + k] = ax[k]; }
      }
      normalize4(xq);
      for (int k = 0; k < 3; k++) xpos[3 * i + k] = xp[k];
      for (int k = 0; k < 4; k++) xquat[4 * i + k] = xq[k];
    };
    const int nb = m.nbody;
    if (nb <= TEAM_SIZE && T.nt == TEAM_SIZE) {
      // level by level: every body at depth d at once (its parent, at depth
      // d - 1, is final); each body's operations are the oracle's
      const int i = T.tid;
      int dep = 0;
      if (i < nb)
        for (int p = i; p > 0; p = m.body_parentid[p]) dep++;
      if (i == 0) {
        xpos[0] = xpos[1] = xpos[2] = 0;
        xquat[0] = 1; xquat[1] = xquat[2] = xquat[3] = 0;
      }
      TSYNC();
      for (int d = 1; __ballot(i < nb && dep >= d); d++) {
        if (i < nb && dep == d) walk_body(i);
        TSYNC();
      }
    } else if (T.tid == 0) {
      xpos[0] = xpos[1] = xpos[2] = 0;
      xquat[0] = 1; xquat[1] = xquat[2] = xquat[3] = 0;
      for (int i = 1; i < nb; i++) walk_body(i);
    }
  }
  TSYNC();
  STAMP(12);
  // body frames and inertial frames: one lane per body
  FOR_T(i, m.nbody) {
    real xq[4], mat[9], tmp[3], ip[3], iq[4], q2[4];
    ldm<4>(xq, xquat + 4 * i);
    quat2mat(mat, xq);
    for (int k = 0; k < 9; k++) xmat[9 * i + k] = mat[k];
    if (i == 0) {
      xipos[0] = xipos[1] = xipos[2] = 0;
      for (int k = 0; k < 9; k++) ximat[k] = mat[k];
    } else {
      ldm<3>(ip, m.body_ipos + 3 * i);
      ldm<4>(iq, m.body_iquat + 4 * i);
      rot_vec_mat(tmp, ip, mat);
      xipos[3 * i] = tmp[0] + xpos[3 * i];
      xipos[3 * i + 1] = tmp[1] + xpos[3 * i + 1];
      xipos[3 * i + 2] = tmp[2] + xpos[3 * i + 2];
      quat_mul(q2, xq, iq);
      quat2mat(mat, q2);
      for (int k = 0; k < 9; k++) ximat[9 * i + k] = mat[k];
    }
  }
  TSYNC();
  STAMP(13);
  real* gxpos = T.w + L.gxpos;
  real* gxmat = T.w + L.gxmat;
  FOR_T(g, m.ngeom) {
    int b = m.geom_bodyid[g];
    real tmp[3], q[4], bm[9], bq[4], gp[3], gq[4], mat[9];
    ldm<9>(bm, xmat + 9 * b);
    ldm<4>(bq, xquat + 4 * b);
    ldm<3>(gp, m.geom_pos + 3 * g);
    ldm<4>(gq, m.geom_quat + 4 * g);
    rot_vec_mat(tmp, gp, bm);
    gxpos[3 * g] = tmp[0] + xpos[3 * b];
    gxpos[3 * g + 1] = tmp[1] + xpos[3 * b + 1];
    gxpos[3 * g + 2] = tmp[2] + xpos[3 * b + 2];
    quat_mul(q, bq, gq);
    quat2mat(mat, q);
    for (int k = 0; k < 9; k++) gxmat[9 * g + k] = mat[k];
  }
  TSYNC();
}

// the compile-time models whose kinematics() takes the split chain (kin_chain_par)
template <class MT>
constexpr bool kin_split_ok() {
  if constexpr (StaticModel<MT>) {
    constexpr KinPlan<MT> p{};
    return p.ok && 4 * p.nslot + 3 * p.nrot <= 12 * MT::nbody + 10 * MT::nv && KIN_SPLIT;
  } else {
    return false;
  }
}

// Hand-off between two waves of a team through an LDS word, without the third
// wave (unlike __syncthreads): the signaller's earlier LDS stores are ordered
// before the flag (workgroup release), the waiter's later loads after it
// (acquire).  Flags carry an increasing step id; the wait is bounded.
__device__ inline void wave_signal(int* f, int v) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if ((threadIdx.x & (TEAM_SIZE - 1)) == 0) __hip_atomic_store(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ inline void wave_wait(const int* f, int v) {
  for (int it = 0; it < (1 << 22); it++) {
    if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= v) break;
    __builtin_amdgcn_s_sleep(1);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// kinematics() of a compile-time model on two waves (three-wave rollout):
// the primary computes the joint rotations and walks the quaternion chain,
// signals, then walks the positions; the helper waits for the quaternions
// and computes every frame rotation -- xmat, ximat, gxmat are functions of the
// quaternions alone -- which the primary's xipos / geom positions then read.
// Each value is the expression kinematics() evaluates, on another wave.
__device__ inline void kinematics_primary(const auto& m, const auto& L, const auto& C, const Team& T, int* fq,
                                          const int* ff, int sid) {
  real* qpos = T.w + L.qpos;
  real* xpos = T.w + L.xpos;
  real* xquat = T.w + L.xquat;
  real* xmat = T.w + L.xmat;
  real* xipos = T.w + L.xipos;
  real* xanchor = T.w + L.xanchor;
  real* xaxis = T.w + L.xaxis;
  real* qloc = T.c + C.qloc;
  FOR_T(j, m.njnt) {
    int type = m.jnt_type[j], qadr = m.jnt_qposadr[j];
    real q[4], ja[3];
    if (type == JNT_HINGE) {
      ldm<3>(ja, m.jnt_axis + 3 * j);
      axis_angle2quat(q, ja, qpos[qadr] - m.qpos0[qadr]);
      for (int k = 0; k < 4; k++) qloc[4 * j + k] = q[k];
    } else if (type == JNT_BALL) {
      q[0] = qpos[qadr]; q[1] = qpos[qadr + 1]; q[2] = qpos[qadr + 2]; q[3] = qpos[qadr + 3];
      normalize4(q);
      for (int k = 0; k < 4; k++) qloc[4 * j + k] = q[k];
    }
  }
  TSYNC();
  STAMP(11);
  kin_chain_par(m, T, qpos, qloc, xpos, xquat, xanchor, xaxis, T.w + L.con, [&]() { wave_signal(fq, sid); });
  TSYNC();
  STAMP(12);
  wave_wait(ff, sid);
  // body inertial positions and geom positions (body frame rotations from the helper)
  real* gxpos = T.w + L.gxpos;
  FOR_T(e, m.nbody + m.ngeom) {
    if (e < m.nbody) {
      const int i = e;
      if (i == 0) {
        xipos[0] = xipos[1] = xipos[2] = 0;
      } else {
        real mat[9], tmp[3], ip[3];
        ldm<9>(mat, xmat + 9 * i);
        ldm<3>(ip, m.body_ipos + 3 * i);
        rot_vec_mat(tmp, ip, mat);
        xipos[3 * i] = tmp[0] + xpos[3 * i];
        xipos[3 * i + 1] = tmp[1] + xpos[3 * i + 1];
        xipos[3 * i + 2] = tmp[2] + xpos[3 * i + 2];
      }
    } else {
      const int g = e - m.nbody;
      const int b = m.geom_bodyid[g];
      real bm[9], gp[3], tmp[3];
      ldm<9>(bm, xmat + 9 * b);
      ldm<3>(gp, m.geom_pos + 3 * g);
      rot_vec_mat(tmp, gp, bm);
      gxpos[3 * g] = tmp[0] + xpos[3 * b];
      gxpos[3 * g + 1] = tmp[1] + xpos[3 * b + 1];
      gxpos[3 * g + 2] = tmp[2] + xpos[3 * b + 2];
    }
  }
  TSYNC();
}
__device__ inline void kinematics_frames(const auto& m, const auto& L, const Team& T, const int* fq, int* ff,
                                         int sid) {
  real* xquat = T.w + L.xquat;
  real* xmat = T.w + L.xmat;
  real* ximat = T.w + L.ximat;
  real* gxmat = T.w + L.gxmat;
  wave_wait(fq, sid);
  FOR_T(e, m.nbody + m.ngeom) {
    if (e < m.nbody) {
      const int i = e;
      real xq[4], mat[9], iq[4], q2[4];
      ldm<4>(xq, xquat + 4 * i);
      quat2mat(mat, xq);
      for (int k = 0; k < 9; k++) xmat[9 * i + k] = mat[k];
      if (i == 0) {
        for (int k = 0; k < 9; k++) ximat[k] = mat[k];
      } else {
        ldm<4>(iq, m.body_iquat + 4 * i);
        quat_mul(q2, xq, iq);
        quat2mat(mat, q2);
        for (int k = 0; k < 9; k++) ximat[9 * i + k] = mat[k];
      }
    } else {
      const int g = e - m.nbody;
      const int b = m.geom_bodyid[g];
      real bq[4], gq[4], q[4], mat[9];
      ldm<4>(bq, xquat + 4 * b);
      ldm<4>(gq, m.geom_quat + 4 * g);
      quat_mul(q, bq, gq);
      quat2mat(mat, q);
      for (int k = 0; k < 9; k++) gxmat[9 * g + k] = mat[k];
    }
  }
  TSYNC();
  wave_signal(ff, sid);
}

__device__ inline void com_pos(const auto& m, const auto& L, const Team& T) {
  const int nb = m.nbody;
  real* xipos = T.w + L.xipos;
  real* scom = T.w + L.scom;
  real* cinert = T.w + L.cinert;
  real* ximat = T.w + L.ximat;
  real* cdof = T.w + L.cdof;
  real* xanchor = T.w + L.xanchor;
  real* xaxis = T.w + L.xaxis;
  real* xmat = T.w + L.xmat;
  FOR_T(i, nb) {
    real ms = m.body_mass[i];
    scom[3 * i] = xipos[3 * i] * ms;
    scom[3 * i + 1] = xipos[3 * i + 1] * ms;
    scom[3 * i + 2] = xipos[3 * i + 2] * ms;
  }
  TSYNC();
  FOR_T(k, 3) {
    for (int i = nb - 1; i > 0; i--) scom[3 * m.body_parentid[i] + k] += scom[3 * i + k];
  }
  TSYNC();
  FOR_T(i, nb) {
    if (m.body_subtreemass[i] < MINVAL) {
      scom[3 * i] = xipos[3 * i];
      scom[3 * i + 1] = xipos[3 * i + 1];
      scom[3 * i + 2] = xipos[3 * i + 2];
    } else {
      real inv = 1 / m.body_subtreemass[i];
      scom[3 * i] *= inv;
      scom[3 * i + 1] *= inv;
      scom[3 * i + 2] *= inv;
    }
  }
  TSYNC();
  FOR_T(i, nb) {
    if (i == 0) {
      for (int k = 0; k < 10; k++) cinert[k] = 0;
    } else {
      real off[3], mat[9], in[3], res[10];
      const real* rc = scom + 3 * m.body_rootid[i];
      off[0] = xipos[3 * i] - rc[0];
      off[1] = xipos[3 * i + 1] - rc[1];
      off[2] = xipos[3 * i + 2] - rc[2];
      ldm<9>(mat, ximat + 9 * i);
      ldm<3>(in, m.body_inertia + 3 * i);
      inert_com(res, in, mat, off, m.body_mass[i]);
      for (int k = 0; k < 10; k++) cinert[10 * i + k] = res[k];
    }
  }
  FOR_T(j, m.njnt) {
    int da = 6 * m.jnt_dofadr[j];
    int bi = m.jnt_bodyid[j];
    const real* rc = scom + 3 * m.body_rootid[bi];
    real off[3] = {rc[0] - xanchor[3 * j], rc[1] - xanchor[3 * j + 1], rc[2] - xanchor[3 * j + 2]};
    real out[6];
    int type = m.jnt_type[j];
    int skip = 0;
    if (type == JNT_FREE) {
      for (int k = 0; k < 18; k++) cdof[da + k] = 0;
      for (int i = 0; i < 3; i++) cdof[da + 3 + 7 * i] = 1;
      skip = 18;
    }
    if (type == JNT_FREE || type == JNT_BALL) {
      for (int i = 0; i < 3; i++) {
        real axis[3] = {xmat[9 * bi + i], xmat[9 * bi + i + 3], xmat[9 * bi + i + 6]};
        out[0] = axis[0]; out[1] = axis[1]; out[2] = axis[2];
        cross3(out + 3, axis, off);
        for (int k = 0; k < 6; k++) cdof[da + skip + 6 * i + k] = out[k];
      }
    } else if (type == JNT_SLIDE) {
      out[0] = out[1] = out[2] = 0;
      out[3] = xaxis[3 * j]; out[4] = xaxis[3 * j + 1]; out[5] = xaxis[3 * j + 2];
      for (int k = 0; k < 6; k++) cdof[da + k] = out[k];
    } else {
      real ax[3] = {xaxis[3 * j], xaxis[3 * j + 1], xaxis[3 * j + 2]};
      out[0] = ax[0]; out[1] = ax[1]; out[2] = ax[2];
      cross3(out + 3, ax, off);
      for (int k = 0; k < 6; k++) cdof[da + k] = out[k];
    }
  }
  TSYNC();
}

#ifndef ILQG_COM_U
#define ILQG_COM_U 1
#endif
// com_pos for a compile-time model on one wave with the subtree centres of
// mass in wave-uniform registers (the rollout's primary chain): every lane
// forms every body's mass-weighted position, the subtree sums (per component,
// bodies descending, com_pos' order) and the normalisation, so the three LDS
// exchange phases before the per-body / per-joint phase disappear; each
// value is com_pos' expression in com_pos' order.
template <class MT>
__device__ inline void com_pos_u(const auto& m, const auto& L, const Team& T) {
  constexpr int NB = MT::nbody;
  const real* xipos = T.w + L.xipos;
  real* scom = T.w + L.scom;
  real* cinert = T.w + L.cinert;
  const real* ximat = T.w + L.ximat;
  real* cdof = T.w + L.cdof;
  const real* xanchor = T.w + L.xanchor;
  const real* xaxis = T.w + L.xaxis;
  const real* xmat = T.w + L.xmat;
  real xi[NB][3], sc[NB][3];
  sfor<0, NB>(SLAM(ii) {
    constexpr int i = SK(ii);
    const real ms = m.body_mass[i];
    sfor<0, 3>(SLAM(kk) {
      xi[i][SK(kk)] = xipos[3 * i + SK(kk)];
      sc[i][SK(kk)] = xi[i][SK(kk)] * ms;
    });
  });
  sfor<0, NB - 1>(SLAM(ii) {
    constexpr int i = NB - 1 - SK(ii);
    constexpr int p = MT::body_parentid[i];
    sfor<0, 3>(SLAM(kk) { sc[p][SK(kk)] += sc[i][SK(kk)]; });
  });
  sfor<0, NB>(SLAM(ii) {
    constexpr int i = SK(ii);
    const real stm = m.body_subtreemass[i];
    const bool tiny = stm < MINVAL;
    const real inv = 1 / (tiny ? 1.0 : stm);
    sfor<0, 3>(SLAM(kk) { sc[i][SK(kk)] = tiny ? xi[i][SK(kk)] : sc[i][SK(kk)] * inv; });
  });
  // scom out: lane e < 3 NB writes entry e
  if (T.tid < 3 * NB) {
    real v = sc[0][0];
    sfor<1, 3 * NB>(SLAM(ee) { v = T.tid == SK(ee) ? sc[SK(ee) / 3][SK(ee) % 3] : v; });
    scom[T.tid] = v;
  }
  // the subtree centre of a body's root, selected from the registers
  auto root_com = [&](int b, real (&rc)[3]) __attribute__((always_inline)) {
    const int rid = m.body_rootid[b];
    sfor<0, 3>(SLAM(kk) { rc[SK(kk)] = sc[0][SK(kk)]; });
    sfor<1, NB>(SLAM(bb) {
      sfor<0, 3>(SLAM(kk) { rc[SK(kk)] = rid == SK(bb) ? sc[SK(bb)][SK(kk)] : rc[SK(kk)]; });
    });
  };
  FOR_T(i, NB) {
    if (i == 0) {
      for (int k = 0; k < 10; k++) cinert[k] = 0;
    } else {
      real off[3], mat[9], in[3], res[10], rc[3];
      root_com(i, rc);
      off[0] = xipos[3 * i] - rc[0];
      off[1] = xipos[3 * i + 1] - rc[1];
      off[2] = xipos[3 * i + 2] - rc[2];
      ldm<9>(mat, ximat + 9 * i);
      ldm<3>(in, m.body_inertia + 3 * i);
      inert_com(res, in, mat, off, m.body_mass[i]);
      for (int k = 0; k < 10; k++) cinert[10 * i + k] = res[k];
    }
  }
  FOR_T(j, MT::njnt) {
    const int da = 6 * m.jnt_dofadr[j];
    const int bi = m.jnt_bodyid[j];
    real rc[3];
    root_com(bi, rc);
    real off[3] = {rc[0] - xanchor[3 * j], rc[1] - xanchor[3 * j + 1], rc[2] - xanchor[3 * j + 2]};
    real out[6];
    const int type = m.jnt_type[j];
    int skip = 0;
    if (type == JNT_FREE) {
      for (int k = 0; k < 18; k++) cdof[da + k] = 0;
      for (int i = 0; i < 3; i++) cdof[da + 3 + 7 * i] = 1;
      skip = 18;
    }
    if (type == JNT_FREE || type == JNT_BALL) {
      for (int i = 0; i < 3; i++) {
        real axis[3] = {xmat[9 * bi + i], xmat[9 * bi + i + 3], xmat[9 * bi + i + 6]};
        out[0] = axis[0]; out[1] = axis[1]; out[2] = axis[2];
        cross3(out + 3, axis, off);
        for (int k = 0; k < 6; k++) cdof[da + skip + 6 * i + k] = out[k];
      }
    } else if (type == JNT_SLIDE) {
      out[0] = out[1] = out[2] = 0;
      out[3] = xaxis[3 * j]; out[4] = xaxis[3 * j + 1]; out[5] = xaxis[3 * j + 2];
      for (int k = 0; k < 6; k++) cdof[da + k] = out[k];
    } else {
      real ax[3] = {xaxis[3 * j], xaxis[3 * j + 1], xaxis[3 * j + 2]};
      out[0] = ax[0]; out[1] = ax[1]; out[2] = ax[2];
      cross3(out + 3, ax, off);
      for (int k = 0; k < 6; k++) cdof[da + k] = out[k];
    }
  }
  TSYNC();
}

__device__ inline void crb(const auto& m, const auto& L, const auto& C, const auto& X,
                           const Team& T) {
  const int nv = m.nv, nb = m.nbody;
  real* crbv = T.w + L.crb;
  real* cinert = T.w + L.cinert;
  real* qM = T.w + L.qM;
  real* cdof = T.w + L.cdof;
  real* buf = T.c + C.buf6;
  FOR_T(e, 10 * nb) crbv[e] = cinert[e];
  TSYNC();
  FOR_T(k, 10) {
    for (int i = nb - 1; i > 0; i--) {
      int p = m.body_parentid[i];
      if (p > 0) crbv[10 * p + k] += crbv[10 * i + k];
    }
  }
  TSYNC();
  FOR_T(i, nv) {
    real ci[10], cd[6], r[6];
    ldm<10>(ci, crbv + 10 * m.dof_bodyid[i]);
    ldm<6>(cd, cdof + 6 * i);
    mul_inert_vec(r, ci, cd);
    for (int k = 0; k < 6; k++) buf[6 * i + k] = r[k];
  }
  TSYNC();
  FOR_T(e, nv * nv) {
    int i = e / nv, j = e % nv;
    if (j <= i) {
      real v = (i == j) ? m.dof_armature[i] : 0.0;
      if (X.isanc[e]) v += tdot(cdof + 6 * j, buf + 6 * i, 6);
      qM[e] = v;
      qM[j * nv + i] = v;
    }
  }
  TSYNC();
}

// crb for a compile-time model with the composite inertias in wave-uniform
// registers (the rollout's primary chain): every lane loads every body's
// cinert and forms the subtree sums (per component, bodies descending, crb's
// order), so the copy and tree-sum phases disappear; each dof lane then
// selects its body's composite inertia.  Same expressions, same order.
template <class MT>
__device__ inline void crb_u(const auto& m, const auto& L, const auto& C, const auto& X, const Team& T) {
  constexpr int NB = MT::nbody, NV = MT::nv;
  const real* cinert = T.w + L.cinert;
  real* qM = T.w + L.qM;
  const real* cdof = T.w + L.cdof;
  real* buf = T.c + C.buf6;
  real cr[NB][10];
  sfor<1, NB>(SLAM(ii) {
    sfor<0, 10>(SLAM(kk) { cr[SK(ii)][SK(kk)] = cinert[10 * SK(ii) + SK(kk)]; });
  });
  sfor<0, NB - 1>(SLAM(ii) {
    constexpr int i = NB - 1 - SK(ii);
    constexpr int p = MT::body_parentid[i];
    if constexpr (p > 0) sfor<0, 10>(SLAM(kk) { cr[p][SK(kk)] += cr[i][SK(kk)]; });
  });
  if (T.tid < NV) {
    const int i = T.tid;
    const int b = m.dof_bodyid[i];
    real ci[10], cd[6], r[6];
    sfor<0, 10>(SLAM(kk) { ci[SK(kk)] = cr[1][SK(kk)]; });
    sfor<2, NB>(SLAM(bb) {
      sfor<0, 10>(SLAM(kk) { ci[SK(kk)] = b == SK(bb) ? cr[SK(bb)][SK(kk)] : ci[SK(kk)]; });
    });
    ldm<6>(cd, cdof + 6 * i);
    mul_inert_vec(r, ci, cd);
    for (int k = 0; k < 6; k++) buf[6 * i + k] = r[k];
  }
  TSYNC();
  FOR_T(e, NV * NV) {
    int i = e / NV, j = e % NV;
    if (j <= i) {
      real v = (i == j) ? m.dof_armature[i] : 0.0;
      if (X.isanc[e]) v += tdot(cdof + 6 * j, buf + 6 * i, 6);
      qM[e] = v;
      qM[j * NV + i] = v;
    }
  }
  TSYNC();
}

// tree L'DL (oracle factor_ld), parallel over ancestor pairs for each k
// compile-time models small enough for factor_ld_lanes (nv <= RMAX: the
// register-row models); ILQG_FLD_LANES=0 keeps the register-row broadcasts
#ifndef ILQG_FLD_LANES
#define ILQG_FLD_LANES 1
#endif
template <class MT>
constexpr bool fld_lanes_ok() {
  if constexpr (StaticModel<MT> && ILQG_FLD_LANES) return MT::nv <= RMAX;
  return false;
}
__device__ inline void factor_ld(const auto& m, const auto& X, const Team& T, const real* mat, real* LD,
                                 real* diaginv, real* tmpv) {
  const int nv = m.nv;
  using MT = std::remove_cvref_t<decltype(m)>;
  if constexpr (fld_lanes_ok<MT>()) {
    // compile-time tree: the factor serially in lane 0's registers
    const real zero[MT::nv] = {};
    factor_ld_lanes<std::remove_cvref_t<decltype(X)>, MT::nv>(T.tid, mat, zero, false, LD, diaginv, 0, 0);
    return;
  }
  if (nv <= RMAX && has_pmask(X)) {
    factor_ld_rows(nv, X.pmask, T.tid, mat, LD, diaginv);
    return;
  }
  FOR_T(e, nv * nv) {
    int i = e / nv, j = e % nv;
    LD[e] = (j <= i) ? mat[e] : 0;
  }
  TSYNC();
  if (nv > SERIAL_NV && nv <= TEAM_SIZE && has_pmask(X) && T.nt == TEAM_SIZE) {
    // lane i owns row i.  For each k (descending) every proper ancestor i of k
    // at once: tmp = LD[k][i] / LD[k][k], LD[i][j] -= tmp * LD[k][j] over j in
    // {i} u anc(i) (descending, as the oracle), then LD[k][i] = tmp.  Within
    // one k the oracle reads LD[k][j] only for j not yet rescaled (the walk
    // goes up the tree and j lies above i), and each LD[i][j] is updated once,
    // so the rows are independent: the same operations on the same operands.
    const int i = T.tid;
    const unsigned long long pm = i < nv ? X.pmask[i] : 0ull;  // one load; broadcast per k
    const unsigned long long self = i < nv ? (pm | (1ull << i)) : 0ull;
    for (int k = nv - 1; k >= 0; k--) {
      const unsigned long long ak = bcast_u64(pm, k);
      if (!ak) continue;  // a root dof: nothing to eliminate (the clamp below still runs)
      real dk = LD[k * nv + k];
      if (dk < MINVAL) dk = MINVAL;
      TSYNC();
      if (i == k) LD[k * nv + k] = dk;
      const bool act = i < nv && ((ak >> i) & 1);
      real tmp = 0;
      if (act) {
        tmp = LD[k * nv + i] / dk;
        for (unsigned long long mj = self; mj;) {
          const int j = 63 - __builtin_clzll(mj);
          mj &= ~(1ull << j);
          LD[i * nv + j] -= tmp * LD[k * nv + j];
        }
      }
      TSYNC();
      if (act) LD[k * nv + i] = tmp;
      TSYNC();
    }
    // the clamp of root dofs (no ancestors), as the oracle's loop does for every k
    if (i < nv && !pm && LD[i * nv + i] < MINVAL) LD[i * nv + i] = MINVAL;
    TSYNC();
    FOR_T(r, nv) diaginv[r] = 1 / LD[r * nv + r];
    TSYNC();
    return;
  }
  if (nv <= SERIAL_NV) {
    // small trees: the oracle's loop on lane 0 beats 4 LDS round trips per k
    if (T.tid == 0) {
      if (has_pmask(X)) {
        // ancestor bitmasks replace the dependent parent-pointer chase
        for (int k = nv - 1; k >= 0; k--) {
          if (LD[k * nv + k] < MINVAL) LD[k * nv + k] = MINVAL;
          const real dk = LD[k * nv + k];
          for (unsigned long long mi = X.pmask[k]; mi;) {
            const int i = 63 - __builtin_clzll(mi);
            mi &= ~(1ull << i);
            real tmp = LD[k * nv + i] / dk;
            // the ancestors of k below i are exactly i's ancestors (one root path)
            for (unsigned long long mj = mi | (1ull << i); mj;) {
              const int j = 63 - __builtin_clzll(mj);
              mj &= ~(1ull << j);
              LD[i * nv + j] -= tmp * LD[k * nv + j];
            }
            LD[k * nv + i] = tmp;
          }
        }
      } else {
        for (int k = nv - 1; k >= 0; k--) {
          if (LD[k * nv + k] < MINVAL) LD[k * nv + k] = MINVAL;
          for (int i = m.dof_parentid[k]; i >= 0; i = m.dof_parentid[i]) {
            real tmp = LD[k * nv + i] / LD[k * nv + k];
            for (int j = i; j >= 0; j = m.dof_parentid[j]) LD[i * nv + j] -= tmp * LD[k * nv + j];
            LD[k * nv + i] = tmp;
          }
        }
      }
      for (int i = 0; i < nv; i++) diaginv[i] = 1 / LD[i * nv + i];
    }
    TSYNC();
    return;
  }
  for (int k = nv - 1; k >= 0; k--) {
    if (T.tid == 0 && LD[k * nv + k] < MINVAL) LD[k * nv + k] = MINVAL;
    TSYNC();
    FOR_T(i, nv) {
      if (i != k && X.isanc[k * nv + i]) tmpv[i] = LD[k * nv + i] / LD[k * nv + k];
    }
    TSYNC();
    FOR_T(e, nv * nv) {
      int i = e / nv, j = e % nv;
      if (i != k && X.isanc[k * nv + i] && X.isanc[i * nv + j]) LD[e] -= tmpv[i] * LD[k * nv + j];
    }
    TSYNC();
    FOR_T(i, nv) {
      if (i != k && X.isanc[k * nv + i]) LD[k * nv + i] = tmpv[i];
    }
    TSYNC();
  }
  FOR_T(i, nv) diaginv[i] = 1 / LD[i * nv + i];
  TSYNC();
}

// oracle solve_ld on lane 0 (ends with a barrier)
__device__ inline void solve_ld(const auto& m, const auto& X, const Team& T, const real* LD,
                                const real* diaginv, real* x) {
  const int nv = m.nv;
  if (nv <= RMAX && has_pmask(X)) {
    solve_ld_rows(nv, X.pmask, T.tid, LD, diaginv, x);
    return;
  }
  if (nv > SERIAL_NV && nv <= TEAM_SIZE && has_pmask(X) && T.nt == TEAM_SIZE) {
    // lane j owns x[j]; the products LD[i][j] * x[.] are formed by the lane
    // holding the operand (one coalesced row read per step) and applied in the
    // oracle's order: the same operations on the same operands
    const int j = T.tid;
    const bool own = j < nv;
    const unsigned long long anc = own ? X.pmask[j] : 0ull;
    real xj = own ? x[j] : (real)0;
    TSYNC();  // every lane has read x before it is overwritten
    for (int i = nv - 1; i >= 0; i--) {  // x[j] -= LD[i][j] * x[i], j in anc(i)
      const real tmp = bcast(xj, i);
      const real lij = own ? LD[i * nv + j] : (real)0;
      if (tmp != 0 && own && ((bcast_u64(anc, i) >> j) & 1)) xj -= lij * tmp;
    }
    if (own) xj *= diaginv[j];
    for (int i = 0; i < nv; i++) {  // x[i] -= LD[i][j] * x[j], j in anc(i) descending
      const unsigned long long ai = bcast_u64(anc, i);
      if (!ai) continue;
      const real pr = own ? LD[i * nv + j] * xj : (real)0;
      real xi = bcast(xj, i);
      for (unsigned long long mj = ai; mj;) {
        const int q = 63 - __builtin_clzll(mj);
        mj &= ~(1ull << q);
        xi -= bcast(pr, q);
      }
      xj = j == i ? xi : xj;
    }
    if (own) x[j] = xj;
    TSYNC();
    return;
  }
  if (T.tid == 0) {
    if (has_pmask(X)) {
      for (int i = nv - 1; i >= 0; i--) {
        real tmp = x[i];
        if (tmp != 0)
          for (unsigned long long mj = X.pmask[i]; mj;) {
            const int j = 63 - __builtin_clzll(mj);
            mj &= ~(1ull << j);
            x[j] -= LD[i * nv + j] * tmp;
          }
      }
      for (int i = 0; i < nv; i++) x[i] *= diaginv[i];
      for (int i = 0; i < nv; i++) {
        real xi = x[i];
        for (unsigned long long mj = X.pmask[i]; mj;) {
          const int j = 63 - __builtin_clzll(mj);
          mj &= ~(1ull << j);
          xi -= LD[i * nv + j] * x[j];
        }
        x[i] = xi;
      }
    } else {
      for (int i = nv - 1; i >= 0; i--) {
        real tmp = x[i];
        if (tmp != 0)
          for (int j = m.dof_parentid[i]; j >= 0; j = m.dof_parentid[j]) x[j] -= LD[i * nv + j] * tmp;
      }
      for (int i = 0; i < nv; i++) x[i] *= diaginv[i];
      for (int i = 0; i < nv; i++)
        for (int j = m.dof_parentid[i]; j >= 0; j = m.dof_parentid[j]) x[i] -= LD[i * nv + j] * x[j];
    }
  }
  TSYNC();
}

__device__ inline void jac_col(const auto& m, const auto& X, const real* scom, const real* cdof,
                               const real* point, int body, int k, real* out3) {
  // one dof column of jac_point (oracle): zero unless dof k lies on the chain of `body`
  const int nv = m.nv;
  out3[0] = out3[1] = out3[2] = 0;
  const real* rc = scom + 3 * m.body_rootid[body];
  real off[3] = {point[0] - rc[0], point[1] - rc[1], point[2] - rc[2]};
  while (body && !m.body_dofnum[body]) body = m.body_parentid[body];
  if (!body) return;
  int last = m.body_dofadr[body] + m.body_dofnum[body] - 1;
  if (!X.isanc[last * nv + k]) return;
  real tmp[3], cd[6];
  ldm<6>(cd, cdof + 6 * k);
  cross3(tmp, cd, off);
  out3[0] = cd[3] + tmp[0];
  out3[1] = cd[4] + tmp[1];
  out3[2] = cd[5] + tmp[2];
}

// collision's narrow phase for pair p (its contacts into pcon, its count into
// pcnt).  Always inlined: as an outlined call (flat pointer arguments) ROCm's
// backend emits an illegal is-shared compare (V_CMP_NE_U32_e32 0, src_shared_base)
__device__ __forceinline__ void collision_pair(const auto& m, const auto& L, const auto& C, const auto& X, const Team& T,
                                      int p) {
  real* gxpos = T.w + L.gxpos;
  real* gxmat = T.w + L.gxmat;
  real* pcon = T.w + L.pcon;
  int* pcnt = T.ci + C.pcnt;
  int g1 = X.pair[2 * p], g2 = X.pair[2 * p + 1];
  int n = 0;
  real margin = maxd(m.geom_margin[g1], m.geom_margin[g2]);
  bool ok = true;
  if (m.geom_rbound[g1] > 0 && m.geom_rbound[g2] > 0) {
    real dd[3] = {gxpos[3 * g1] - gxpos[3 * g2], gxpos[3 * g1 + 1] - gxpos[3 * g2 + 1],
                    gxpos[3 * g1 + 2] - gxpos[3 * g2 + 2]};
    if (sqrt(dot3(dd, dd)) > m.geom_rbound[g1] + m.geom_rbound[g2] + margin) ok = false;
  }
  if (ok) {
    int ga = g1, gb = g2;
    if (m.geom_type[g1] > m.geom_type[g2]) { ga = g2; gb = g1; }
    real pos1[3], mat1[9], sz1[3], pos2[3], mat2[9], sz2[3];
    ldm<3>(pos1, gxpos + 3 * ga);
    ldm<9>(mat1, gxmat + 9 * ga);
    ldm<3>(sz1, m.geom_size + 3 * ga);
    ldm<3>(pos2, gxpos + 3 * gb);
    ldm<9>(mat2, gxmat + 9 * gb);
    ldm<3>(sz2, m.geom_size + 3 * gb);
    // contacts straight into the pair's LDS records
    n = narrow(m, m.geom_type[ga], m.geom_type[gb], pos1, mat1, sz1, pos2, mat2, sz2, margin,
               LdsConSinkT<real>{pcon + 14 * p});
  }
  pcnt[p] = n;
}

__device__ __forceinline__ void collision_finish(const auto& m, const auto& L, const auto& C, const auto& X,
                                                const Team& T);
__device__ inline void collision(const auto& m, const auto& L, const auto& C, const auto& X,
                                 const Team& T) {
  FOR_T(p, X.npair) collision_pair(m, L, C, X, T, p);
  collision_finish(m, L, C, X, T);
}

// the ordered compaction and the contact records (after every pair's narrow phase)
__device__ __forceinline__ void collision_finish(const auto& m, const auto& L, const auto& C, const auto& X,
                                                const Team& T) {
  real* con = T.w + L.con;
  int* coni = T.iw + L.coni;
  real* pcon = T.w + L.pcon;
  int* pcnt = T.ci + C.pcnt;
  TSYNC();
  // ordered compaction with the oracle's truncation at nconmax
  const int lim = m.nconmax < m.maxcon ? m.nconmax : m.maxcon;
  // offsets as ballot prefix counts when nothing is truncated (n <= 2 per pair),
  // else the oracle's loop on lane 0
  bool par = X.npair <= TEAM_SIZE;
  if (par) {
    const int t = T.tid;
    const int n = t < X.npair ? pcnt[t] : 0;
    const unsigned long long b0 = __ballot(n & 1), b1 = __ballot(n & 2);
    const int total = __popcll(b0) + 2 * __popcll(b1);
    par = total <= lim && __ballot(n > 3) == 0ull;
    if (par) {
      const unsigned long long below = t < 64 ? (1ull << t) - 1 : ~0ull;
      if (t < X.npair) pcnt[t] = ((__popcll(b0 & below) + 2 * __popcll(b1 & below)) << 8) | n;
      if (t == 0) T.iw[L.ncon] = total;
    }
  }
  if (!par && T.tid == 0) {
    int ncon = 0;
    for (int p = 0; p < X.npair; p++) {
      int n = pcnt[p];
      int take = 0;
      for (int k = 0; k < n; k++)
        if (ncon + take < lim) take++;
      pcnt[p] = (ncon << 8) | take;  // offset, count
      ncon += take;
    }
    T.iw[L.ncon] = ncon;
  }
  TSYNC();
  FOR_T(e, 2 * X.npair) {
    int p = e >> 1, k = e & 1;
    int off = pcnt[p] >> 8, take = pcnt[p] & 255;
    if (k < take) {
      int g1 = X.pair[2 * p], g2 = X.pair[2 * p + 1];
      int ga = g1, gb = g2;
      if (m.geom_type[g1] > m.geom_type[g2]) { ga = g2; gb = g1; }
      real margin = maxd(m.geom_margin[g1], m.geom_margin[g2]);
      real gap = maxd(m.geom_gap[ga], m.geom_gap[gb]);
      real s1 = m.geom_solmix[ga], s2 = m.geom_solmix[gb], mix;
      if (s1 < MINVAL && s2 < MINVAL) mix = 0.5;
      else if (s1 < MINVAL) mix = 0;
      else if (s2 < MINVAL) mix = 1;
      else mix = s1 / (s1 + s2);
      const real* pc = pcon + 14 * p + 7 * k;
      real* c = con + CON_ND * (off + k);
      real fr[9];
      fr[0] = pc[4]; fr[1] = pc[5]; fr[2] = pc[6];
      make_frame(fr);
      c[CON_DIST] = pc[0];
      c[CON_POS] = pc[1]; c[CON_POS + 1] = pc[2]; c[CON_POS + 2] = pc[3];
      for (int r = 0; r < 9; r++) c[CON_FRAME + r] = fr[r];
      c[CON_INCLM] = margin - gap;
      real f0 = maxd(m.geom_friction[3 * ga], m.geom_friction[3 * gb]);
      real f1 = maxd(m.geom_friction[3 * ga + 1], m.geom_friction[3 * gb + 1]);
      real f2 = maxd(m.geom_friction[3 * ga + 2], m.geom_friction[3 * gb + 2]);
      c[CON_FRIC] = f0; c[CON_FRIC + 1] = f0; c[CON_FRIC + 2] = f1; c[CON_FRIC + 3] = f2; c[CON_FRIC + 4] = f2;
      for (int r = 0; r < 2; r++)
        c[CON_SOLREF + r] = mix * m.geom_solref[2 * ga + r] + (1 - mix) * m.geom_solref[2 * gb + r];
      for (int r = 0; r < 5; r++)
        c[CON_SOLIMP + r] = mix * m.geom_solimp[5 * ga + r] + (1 - mix) * m.geom_solimp[5 * gb + r];
      int cd1 = m.geom_condim[ga], cd2 = m.geom_condim[gb];
      int* ci = coni + CON_NI * (off + k);
      ci[CONI_DIM] = cd1 > cd2 ? cd1 : cd2;
      ci[CONI_G1] = ga;
      ci[CONI_G2] = gb;
      ci[CONI_EFCADR] = -1;
    }
  }
  TSYNC();
}

// make_constraint, in pieces the two-wave rollout schedules separately
// (step_dual_split); make_constraint() runs them in the oracle's order.

// which limit sides are violated (bit 0 lower, bit 1 upper): qpos only
__device__ inline void mc_limit_masks(const auto& m, const auto& L, const auto& C, const Team& T) {
  real* qpos = T.w + L.qpos;
  int* jcnt = T.ci + C.jcnt;
  FOR_T(j, m.njnt) {
    int type = m.jnt_type[j], mask = 0;
    if (m.jnt_limited[j] && (type == JNT_SLIDE || type == JNT_HINGE)) {
      real value = qpos[m.jnt_qposadr[j]];
      for (int side = -1; side <= 1; side += 2) {
        real dist = side * (m.jnt_range[2 * j + (side + 1) / 2] - value);
        if (dist < m.jnt_margin[j]) mask |= (side < 0 ? 1 : 2);
      }
    }
    jcnt[j] = mask;
  }
}

// contact jacobians in the contact frame: one lane per (contact, dof)
__device__ inline void mc_contact_jac(const auto& m, const auto& L, const auto& X, const Team& T) {
  const int nv = m.nv;
  real* con = T.w + L.con;
  int* coni = T.iw + L.coni;
  real* jc = T.w + L.jc;
  real* scom = T.w + L.scom;
  real* cdof = T.w + L.cdof;
  const int ncon = T.iw[L.ncon];
  FOR_T(e, ncon * nv) {
    int c = e / nv, k = e % nv;
    const real* cc = con + CON_ND * c;
    int b1 = m.geom_bodyid[coni[CON_NI * c + CONI_G1]], b2 = m.geom_bodyid[coni[CON_NI * c + CONI_G2]];
    real pos[3] = {cc[CON_POS], cc[CON_POS + 1], cc[CON_POS + 2]}, a[3], b[3];
    jac_col(m, X, scom, cdof, pos, b1, k, a);
    jac_col(m, X, scom, cdof, pos, b2, k, b);
    b[0] -= a[0]; b[1] -= a[1]; b[2] -= a[2];
    for (int r = 0; r < 3; r++)
      jc[(c * 3 + r) * nv + k] = cc[CON_FRAME + 3 * r] * b[0] + cc[CON_FRAME + 3 * r + 1] * b[1] +
                                 cc[CON_FRAME + 3 * r + 2] * b[2];
  }
}

// row allocation in the oracle's order (limits, then contacts).  When every
// row fits (no njmax truncation) the offsets are prefix counts over ballots,
// one lane per joint / contact; otherwise the oracle's loop on lane 0.
// Returns whether the parallel branch ran (wave-uniform).
__device__ inline bool mc_alloc(const auto& m, const auto& L, const auto& C, const Team& T) {
  int* coni = T.iw + L.coni;
  int* efc_type = T.iw + L.efc_type;
  int* efc_id = T.iw + L.efc_id;
  int* rsub = T.ci + C.rsub;
  int* jcnt = T.ci + C.jcnt;
  const int ncon = T.iw[L.ncon];
  const int njmax = m.njmax < m.maxefc ? m.njmax : m.maxefc;
  bool par = m.njnt <= TEAM_SIZE && ncon <= TEAM_SIZE;
  if (par) {
    const int t = T.tid;
    const int jm = t < m.njnt ? jcnt[t] : 0;
    const unsigned long long blo = __ballot(jm & 1), bhi = __ballot(jm & 2);
    const int nlim = __popcll(blo) + __popcll(bhi);
    const int dim = t < ncon ? coni[CON_NI * t + CONI_DIM] : 0;
    const int nrow = t < ncon ? (dim == 1 ? 1 : 2 * (dim - 1)) : 0;
    int before = 0, total = 0;  // contact rows of lanes below t, of all lanes
    for (int b = 0; b < 5; b++) {
      const unsigned long long bb = __ballot((nrow >> b) & 1);
      before += (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bb >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bb, 0u)) << b;
      total += __popcll(bb) << b;
    }
    par = nrow < 32 && __ballot(nrow >= 32) == 0ull && nlim + total <= njmax;
    if (par) {
      if (t < m.njnt && jm) {
        const unsigned long long below = (1ull << t) - 1;
        int r = __popcll(blo & below) + __popcll(bhi & below);
        for (int side = -1; side <= 1; side += 2) {
          if (!(jm & (side < 0 ? 1 : 2))) continue;
          efc_type[r] = C_LIMIT;
          efc_id[r] = t;
          rsub[r] = side;
          r++;
        }
      }
      if (t < ncon) {
        const int r0 = nlim + before;
        coni[CON_NI * t + CONI_EFCADR] = r0;
        for (int r = 0; r < nrow; r++) {
          efc_type[r0 + r] = dim == 1 ? C_FRICTIONLESS : C_PYRAMIDAL;
          efc_id[r0 + r] = t;
          rsub[r0 + r] = r;
        }
      }
      if (t == 0) T.iw[L.nefc] = nlim + total;
    }
  }
  if (!par && T.tid == 0) {
    int nefc = 0;
    for (int j = 0; j < m.njnt; j++) {
      int mask = jcnt[j];
      for (int side = -1; side <= 1; side += 2) {
        if (!(mask & (side < 0 ? 1 : 2))) continue;
        if (nefc + 1 > njmax) break;
        efc_type[nefc] = C_LIMIT;
        efc_id[nefc] = j;
        rsub[nefc] = side;
        nefc++;
      }
    }
    for (int c = 0; c < ncon; c++) {
      int dim = coni[CON_NI * c + CONI_DIM];
      int nrow = dim == 1 ? 1 : 2 * (dim - 1);
      if (nefc + nrow > njmax) continue;
      coni[CON_NI * c + CONI_EFCADR] = nefc;
      for (int r = 0; r < nrow; r++) {
        efc_type[nefc] = dim == 1 ? C_FRICTIONLESS : C_PYRAMIDAL;
        efc_id[nefc] = c;
        rsub[nefc] = r;
        nefc++;
      }
    }
    T.iw[L.nefc] = nefc;
  }
  return par;
}

// jacobian rows and row parameters (impedance, K/B, D) of rows [r0, r1)
__device__ inline void mc_rows(const auto& m, const auto& L, const auto& C, const Team& T, int r0, int r1) {
  const int nv = m.nv;
  real* qpos = T.w + L.qpos;
  real* con = T.w + L.con;
  real* efcJ = T.w + L.efc_J;
  real* efc_pos = T.w + L.efc_pos;
  real* efc_margin = T.w + L.efc_margin;
  real* efc_D = T.w + L.efc_D;
  real* KBIP = T.w + L.efc_KBIP;
  int* coni = T.iw + L.coni;
  int* efc_type = T.iw + L.efc_type;
  int* efc_id = T.iw + L.efc_id;
  int* rsub = T.ci + C.rsub;
  real* jc = T.w + L.jc;
  FOR_T(e0, (r1 - r0) * nv) {
    const int e = e0 + r0 * nv;
    int i = e / nv, k = e % nv;
    int type = efc_type[i], id = efc_id[i], sub = rsub[i];
    real v;
    if (type == C_LIMIT) {
      v = (k == m.jnt_dofadr[id]) ? (real)(-sub) : 0.0;
    } else if (type == C_FRICTIONLESS) {
      v = jc[(id * 3 + 0) * nv + k];
    } else {
      int kk = sub / 2 + 1;
      real f = con[CON_ND * id + CON_FRIC + kk - 1];
      real j0 = jc[(id * 3 + 0) * nv + k], jk = jc[(id * 3 + kk) * nv + k];
      v = (sub & 1) ? j0 + (-f) * jk : j0 + f * jk;
    }
    efcJ[i * nv + k] = v;
  }
  FOR_T(i0, r1 - r0) {
    const int i = i0 + r0;
    int type = efc_type[i], id = efc_id[i];
    real solref[2], solimp[5], dA, imp, tc, dr, dmax, K, B, pos, mar;
    if (type == C_LIMIT) {
      real value = qpos[m.jnt_qposadr[id]];
      int side = rsub[i];
      pos = side * (m.jnt_range[2 * id + (side + 1) / 2] - value);
      mar = m.jnt_margin[id];
      ldm<2>(solref, m.jnt_solref + 2 * id);
      ldm<5>(solimp, m.jnt_solimp + 5 * id);
      dA = m.dof_invweight0[m.jnt_dofadr[id]];
    } else {
      const real* cc = con + CON_ND * id;
      int b1 = m.geom_bodyid[coni[CON_NI * id + CONI_G1]], b2 = m.geom_bodyid[coni[CON_NI * id + CONI_G2]];
      real tran = m.body_invweight0[2 * b1] + m.body_invweight0[2 * b2];
      pos = cc[CON_DIST];
      mar = cc[CON_INCLM];
      ldm<2>(solref, cc + CON_SOLREF);
      ldm<5>(solimp, cc + CON_SOLIMP);
      if (type == C_FRICTIONLESS) {
        dA = tran;
      } else {
        int k = (i - coni[CON_NI * id + CONI_EFCADR]) / 2;
        real f = cc[CON_FRIC + k];
        dA = tran + f * f * tran;
      }
    }
    efc_pos[i] = pos;
    efc_margin[i] = mar;
    imp = get_impedance(solimp, pos, mar);
    dmax = clipd(solimp[1], MINIMP, MAXIMP);
    tc = solref[0];
    dr = solref[1];
    if (tc > 0) {
      if (tc < 2 * m.opt_timestep) tc = 2 * m.opt_timestep;
      K = 1 / (dmax * dmax * tc * tc * dr * dr);
      B = 2 / (dmax * tc);
    } else {
      K = -tc / (dmax * dmax);
      B = -dr / dmax;
    }
    KBIP[L.kstr * i] = K;
    KBIP[L.kstr * i + 1] = B;
    KBIP[L.kstr * i + 2] = imp;
    real R = maxd(MINVAL, (1 - imp) * dA / imp);
    efc_D[i] = 1 / R;
  }
}

__device__ inline void make_constraint(const auto& m, const auto& L, const auto& C, const auto& X,
                                       const Team& T) {
  mc_limit_masks(m, L, C, T);
  mc_contact_jac(m, L, X, T);
  TSYNC();
  (void)mc_alloc(m, L, C, T);
  TSYNC();
  mc_rows(m, L, C, T, 0, T.iw[L.nefc]);
  TSYNC();
}

// The limit rows -- the first rows of the constraint arrays -- from qpos alone,
// ahead of make_constraint (two-wave rollout, beside the kinematics): masks,
// allocation and rows [0, nlim) exactly as make_constraint computes them.
// Returns nlim (-1 when the limits alone exceed njmax: make_constraint then
// takes its serial branch and computes every row).
__device__ inline int limit_rows_pre(const auto& m, const auto& L, const auto& C, const Team& T) {
  mc_limit_masks(m, L, C, T);
  TSYNC();
  if (m.njnt > TEAM_SIZE) return -1;
  const int njmax = m.njmax < m.maxefc ? m.njmax : m.maxefc;
  int* efc_type = T.iw + L.efc_type;
  int* efc_id = T.iw + L.efc_id;
  int* rsub = T.ci + C.rsub;
  const int t = T.tid;
  const int jm = t < m.njnt ? T.ci[C.jcnt + t] : 0;
  const unsigned long long blo = __ballot(jm & 1), bhi = __ballot(jm & 2);
  const int nlim = __popcll(blo) + __popcll(bhi);
  if (nlim > njmax) return -1;
  if (t < m.njnt && jm) {
    const unsigned long long below = (1ull << t) - 1;
    int r = __popcll(blo & below) + __popcll(bhi & below);
    for (int side = -1; side <= 1; side += 2) {
      if (!(jm & (side < 0 ? 1 : 2))) continue;
      efc_type[r] = C_LIMIT;
      efc_id[r] = t;
      rsub[r] = side;
      r++;
    }
  }
  TSYNC();
  mc_rows(m, L, C, T, 0, nlim);
  TSYNC();
  return nlim;
}

// transmission: actuator_moment (joint transmissions)
__device__ inline void transmission(const auto& m, const auto& L, const Team& T) {
  real* amom = T.w + L.amom;
  FOR_T(e, m.nu * m.nv) {
    int i = e / m.nv, k = e % m.nv;
    int j = m.actuator_trnid[i];
    amom[e] = (k == m.jnt_dofadr[j]) ? m.actuator_gear[i] : 0.0;
  }
}

__device__ inline void fwd_position(const auto& m, const auto& L, const auto& C, const auto& X,
                                    const Team& T) {
  kinematics(m, L, C, T);
  STAMP(14 - 14 + 0);
  com_pos(m, L, T);
  STAMP(1);
  transmission(m, L, T);
  crb(m, L, C, X, T);
  STAMP(2);
  factor_ld(m, X, T, T.w + L.qM, T.w + L.qLD, T.w + L.qLDinv, T.c + C.ftmp);
  STAMP(3);
  collision(m, L, C, X, T);
  STAMP(4);
  make_constraint(m, L, C, X, T);
  STAMP(5);
}

// ------------------------------------------------------ velocity stage ---
// part 0: the whole stage; 1: com velocities + RNE (primary wave of a
// two-wave step); 2: passive forces + constraint reference (helper wave)
// passive forces: one lane per dof (hinge/slide springs; ball/free rejected on the host)
__device__ inline void passive_forces(const auto& m, const auto& L, const Team& T) {
  real* qvel = T.w + L.qvel;
  real* qpos = T.w + L.qpos;
  real* qp = T.w + L.qfrc_passive;
  FOR_T(i, m.nv) {
    int j = m.dof_jntid[i];
    real v = 0;
    real k = m.jnt_stiffness[j];
    if (k != 0) {
      int pa = m.jnt_qposadr[j];
      v = -k * (qpos[pa] - m.qpos_spring[pa]);
    }
    v -= m.dof_damping[i] * qvel[i];
    qp[i] = v;
  }
}

// constraint velocities and reference accelerations: one lane per row
__device__ inline void constraint_ref(const auto& m, const auto& L, const Team& T) {
  const int nv = m.nv;
  real* qvel = T.w + L.qvel;
  const int nefc = T.iw[L.nefc];
  real* KBIP = T.w + L.efc_KBIP;
  real* efc_vel = T.w + L.efc_vel;
  real* aref = T.w + L.efc_aref;
  real* J = T.w + L.efc_J;
  real* pos = T.w + L.efc_pos;
  real* mar = T.w + L.efc_margin;
  FOR_T(i, nefc) {
    real k0 = KBIP[L.kstr * i], k1 = KBIP[L.kstr * i + 1], k2 = KBIP[L.kstr * i + 2];
    real v = tdot(J + i * nv, qvel, nv);
    efc_vel[i] = v;
    aref[i] = -k1 * v - k0 * k2 * (pos[i] - mar[i]);
  }
}

// actuator forces and qfrc_actuator = moment' * force (the first part of the
// acceleration stage; ctrl and the joint transmissions only)
__device__ inline void actuator_force(const auto& m, const auto& L, const Team& T) {
  const int nv = m.nv, nu = m.nu;
  real* ctrl = T.w + L.ctrl;
  real* af = T.w + L.afrc;
  real* amom = T.w + L.amom;
  real* qa = T.w + L.qfrc_act;
  FOR_T(i, nu) {
    real c = ctrl[i], f;
    if (m.actuator_ctrllimited[i]) c = clipd(c, m.actuator_ctrlrange[2 * i], m.actuator_ctrlrange[2 * i + 1]);
    f = m.actuator_gainprm[i] * c;
    if (m.actuator_forcelimited[i]) f = clipd(f, m.actuator_forcerange[2 * i], m.actuator_forcerange[2 * i + 1]);
    af[i] = f;
  }
  TSYNC();
  FOR_T(j, nv) {
    real s = 0;
    for (int i = 0; i < nu; i++) s += amom[i * nv + j] * af[i];
    qa[j] = s;
  }
}

__device__ inline void fwd_velocity(const auto& m, const auto& L, const auto& C, const Team& T, int part = 0) {
  const int nv = m.nv, nb = m.nbody;
  real* cvelw = T.w + L.cvel;
  real* cdof = T.w + L.cdof;
  real* cdd = T.w + L.cdof_dot;
  real* qvel = T.w + L.qvel;
  real* qpos = T.w + L.qpos;
  if (part != 2) {
  // com velocities.  The recursion cvel_i = cvel_parent + sum_dof cdof*qvel is
  // component-wise, so it runs as 6 parallel chains (lane k = component k);
  // each dof's pre-update cvel is recorded (s_con) and the cdof_dot cross
  // products, which mix components but feed nothing back, follow one lane per
  // dof.  Per component the operations are the oracle's, in its order.
  real* cvb = T.w + L.s_con;  // 6 x nv: cvel seen by each dof
  FOR_T(k, 6) {
    cvelw[k] = 0;
    real cv = 0;
    int prev = 0;
    for (int i = 1; i < nb; i++) {
      const int bda = m.body_dofadr[i], pid = m.body_parentid[i];
      if (pid != prev) cv = cvelw[6 * pid + k];
      for (int j = 0; j < m.body_dofnum[i]; j++) {
        const int type = m.jnt_type[m.dof_jntid[bda + j]];
        if (type == JNT_FREE) {
          real t = 0;
          for (int q = 0; q < 3; q++) t += cdof[6 * (bda + q) + k] * qvel[bda + q];
          cv += t;
          j += 3;
        }
        if (type == JNT_FREE || type == JNT_BALL) {
          for (int q = 0; q < 3; q++) cvb[6 * (bda + j + q) + k] = cv;
          real t = 0;
          for (int q = 0; q < 3; q++) t += cdof[6 * (bda + j + q) + k] * qvel[bda + j + q];
          cv += t;
          j += 2;
        } else {
          cvb[6 * (bda + j) + k] = cv;
          real t = 0;
          t += cdof[6 * (bda + j) + k] * qvel[bda + j];
          cv += t;
        }
      }
      cvelw[6 * i + k] = cv;
      prev = i;
    }
  }
  TSYNC();
  FOR_T(d, nv) {
    const int jid = m.dof_jntid[d];
    if (m.jnt_type[jid] == JNT_FREE && d < m.jnt_dofadr[jid] + 3) {
      for (int q = 0; q < 6; q++) cdd[6 * d + q] = 0;
    } else {
      real cv[6], cd[6], r[6];
      ldm<6>(cv, cvb + 6 * d);
      ldm<6>(cd, cdof + 6 * d);
      cross_motion(r, cv, cd);
      for (int q = 0; q < 6; q++) cdd[6 * d + q] = r[q];
    }
  }
  }
  if (part != 1) {
    passive_forces(m, L, T);
    constraint_ref(m, L, T);
  }
  TSYNC();
  if (part == 2) return;
  // RNE: per (body, component) dof-velocity terms, then the chain per component
  real* rt = T.c + C.rtmp;
  real* cacc = T.w + L.s_rne;
  real* cfrc = cacc + 6 * nb;
  FOR_T(e, 6 * nb) {
    int i = e / 6, k = e % 6;
    if (i > 0) {
      int bda = m.body_dofadr[i], nd = m.body_dofnum[i];
      real sum = 0;
      for (int j = 0; j < nd; j++) sum += cdd[6 * (bda + j) + k] * qvel[bda + j];
      rt[e] = nd ? sum : 0;
    }
  }
  TSYNC();
  FOR_T(k, 6) {
    cacc[k] = k < 3 ? 0.0 : (k == 3 ? -m.opt_gravity0 : (k == 4 ? -m.opt_gravity1 : -m.opt_gravity2));
    for (int i = 1; i < nb; i++) cacc[6 * i + k] = cacc[6 * m.body_parentid[i] + k] + rt[6 * i + k];
  }
  TSYNC();
  real* cinert = T.w + L.cinert;
  FOR_T(i, nb) {
    if (i == 0) {
      for (int k = 0; k < 6; k++) cfrc[k] = 0;
    } else {
      real ci[10], a[6], f[6], cv[6], tmp[6], tmp1[6];
      ldm<10>(ci, cinert + 10 * i);
      ldm<6>(a, cacc + 6 * i);
      ldm<6>(cv, cvelw + 6 * i);
      mul_inert_vec(f, ci, a);
      mul_inert_vec(tmp, ci, cv);
      cross_force(tmp1, cv, tmp);
      for (int k = 0; k < 6; k++) cfrc[6 * i + k] = f[k] + tmp1[k];
    }
  }
  TSYNC();
  FOR_T(k, 6) {
    for (int i = nb - 1; i > 0; i--) {
      int p = m.body_parentid[i];
      if (p) cfrc[6 * p + k] += cfrc[6 * i + k];
    }
  }
  TSYNC();
  real* bias = T.w + L.qfrc_bias;
  FOR_T(i, nv) bias[i] = tdot(cdof + 6 * i, cfrc + 6 * m.dof_bodyid[i], 6);
  TSYNC();
}

#ifndef ILQG_VEL_U
#define ILQG_VEL_U 1
#endif
// fwd_velocity's part 1 (com velocities, cdof_dot, RNE -> qfrc_bias) for a
// compile-time model whose joints are all hinges and slides, in wave-uniform
// registers (the rollout's primary chain): every lane loads qvel and cdof once
// and runs the whole chain -- cvel per component down the tree, cdof_dot,
// the per-body dof terms, cacc, cfrc, the subtree sums, the bias rows -- with
// no LDS exchange in between; lane d < nv stores qfrc_bias[d] (cvel, cdof_dot
// and the RNE scratch have no reader outside this stage).  Every value is
// fwd_velocity's expression, in its order (the "t = 0; t += x" forms kept).
template <class MT>
constexpr bool vel_regs_ok() {
  if constexpr (StaticModel<MT> && ILQG_VEL_U) {
    if constexpr (MT::nv <= RMAX && MT::nbody <= 8) {
      for (int j = 0; j < MT::njnt; j++)
        if (MT::jnt_type[j] != JNT_SLIDE && MT::jnt_type[j] != JNT_HINGE) return false;
      return true;
    }
  }
  return false;
}
template <class MT>
__device__ inline void fwd_velocity_u(const auto& m, const auto& L, const Team& T) {
  constexpr int NV = MT::nv, NB = MT::nbody;
  const real* cdofw = T.w + L.cdof;
  const real* cinert = T.w + L.cinert;
  real qv[NV], cd[NV][6];
  sfor<0, NV>(SLAM(dd) {
    qv[SK(dd)] = T.w[L.qvel + SK(dd)];
    sfor<0, 6>(SLAM(kk) { cd[SK(dd)][SK(kk)] = cdofw[6 * SK(dd) + SK(kk)]; });
  });
  // com velocities; cvb[d]: the cvel dof d sees (fwd_velocity's chain)
  real cvel[NB][6], cvb[NV][6];
  sfor<0, 6>(SLAM(kk) { cvel[0][SK(kk)] = 0; });
  sfor<1, NB>(SLAM(ii) {
    constexpr int i = SK(ii);
    constexpr int pid = MT::body_parentid[i], bda = MT::body_dofadr[i], nd = MT::body_dofnum[i];
    sfor<0, 6>(SLAM(kk) {
      constexpr int k = SK(kk);
      real cv = cvel[pid][k];
      sfor<0, nd>(SLAM(jj) {
        constexpr int d = bda + SK(jj);
        cvb[d][k] = cv;
        real t = 0;
        t += cd[d][k] * qv[d];
        cv += t;
      });
      cvel[i][k] = cv;
    });
  });
  // cdof_dot
  real cdd[NV][6];
  sfor<0, NV>(SLAM(dd) { cross_motion(cdd[SK(dd)], cvb[SK(dd)], cd[SK(dd)]); });
  // RNE: per-body dof terms, cacc down the tree
  real cacc[NB][6];
  cacc[0][0] = cacc[0][1] = cacc[0][2] = 0.0;
  cacc[0][3] = -m.opt_gravity0;
  cacc[0][4] = -m.opt_gravity1;
  cacc[0][5] = -m.opt_gravity2;
  sfor<1, NB>(SLAM(ii) {
    constexpr int i = SK(ii);
    constexpr int pid = MT::body_parentid[i], bda = MT::body_dofadr[i], nd = MT::body_dofnum[i];
    sfor<0, 6>(SLAM(kk) {
      constexpr int k = SK(kk);
      real sum = 0;
      sfor<0, nd>(SLAM(jj) { sum += cdd[bda + SK(jj)][k] * qv[bda + SK(jj)]; });
      const real rt = nd ? sum : 0;
      cacc[i][k] = cacc[pid][k] + rt;
    });
  });
  // cfrc per body, subtree sums
  real cf[NB][6];
  sfor<1, NB>(SLAM(ii) {
    constexpr int i = SK(ii);
    real ci[10], f[6], tmp[6], tmp1[6];
    sfor<0, 10>(SLAM(kk) { ci[SK(kk)] = cinert[10 * i + SK(kk)]; });
    mul_inert_vec(f, ci, cacc[i]);
    mul_inert_vec(tmp, ci, cvel[i]);
    cross_force(tmp1, cvel[i], tmp);
    sfor<0, 6>(SLAM(kk) { cf[i][SK(kk)] = f[SK(kk)] + tmp1[SK(kk)]; });
  });
  sfor<0, NB - 1>(SLAM(ii) {
    constexpr int i = NB - 1 - SK(ii);
    constexpr int p = MT::body_parentid[i];
    if constexpr (p != 0) sfor<0, 6>(SLAM(kk) { cf[p][SK(kk)] += cf[i][SK(kk)]; });
  });
  // qfrc_bias[d] = tdot(cdof_d, cfrc_body(d)) on lane d
  real b = 0;
  sfor<0, NV>(SLAM(dd) {
    constexpr int d = SK(dd);
    constexpr int bi = MT::dof_bodyid[d];
    real r = 0;
    sfor<0, 6>(SLAM(kk) { r += cd[d][SK(kk)] * cf[bi][SK(kk)]; });
    b = T.tid == d ? r : b;
  });
  if (T.tid < NV) T.w[L.qfrc_bias + T.tid] = b;
  TSYNC();
}

#ifndef ILQG_VEL_H
#define ILQG_VEL_H 1
#endif
// fwd_velocity_u's values with its independent work spread over lanes: a
// wave-uniform stage executes every scalar operation as a full wave
// instruction, so the ≈700 operations of the velocity stage cost their count
// in issue cycles.  Here each phase runs one output per lane and the phases
// exchange through LDS (five wave fences):
//   1. lane k < 6: component k of the com velocities down the tree (the cvel
//      each dof sees, cvb, and every body's cvel);
//   2. lane 6 d + c: component c of cdof_dot[d] = cross_motion(cvb[d], cdof[d]);
//   3. lane k < 6: component k of the per-body dof terms and cacc down the tree;
//   4. lane i (body): cfrc_i = I_i cacc_i + cvel_i x* (I_i cvel_i);
//   5. lane k < 6: the subtree sums; then lane d: qfrc_bias[d] = cdof_d . cfrc_body(d).
// Every value is the expression fwd_velocity_u evaluates, in its order
// (cross_motion's terms as a lane-selected pair or pair of pairs: -x*y is
// -(x*y) exactly, and x - y is x + (-y)).
template <class MT>
__device__ inline void fwd_velocity_h(const auto& m, const auto& L, const Team& T) {
  constexpr int NV = MT::nv, NB = MT::nbody;
  static_assert(6 * NV <= TEAM_SIZE && NB <= TEAM_SIZE, "one output per lane");
  const int t = T.tid;
  real* cvw = T.w + L.cvel;      // [NB][6]
  real* cvb = T.w + L.s_con;     // [NV][6]: the cvel dof d sees
  real* cdw = T.w + L.cdof_dot;  // [NV][6]
  real* cac = T.w + L.s_rne;     // [NB][6]
  real* cfw = cac + 6 * NB;      // [NB][6]
  const real* cdofw = T.w + L.cdof;
  const real* qvw = T.w + L.qvel;
  real qv[NV];
  sfor<0, NV>(SLAM(dd) { qv[SK(dd)] = qvw[SK(dd)]; });
  // 1. com velocities
  if (t < 6) {
    const int k = t;
    real cdk[NV];
    sfor<0, NV>(SLAM(dd) { cdk[SK(dd)] = cdofw[6 * SK(dd) + k]; });
    real cvel[NB];
    cvel[0] = 0;
    sfor<1, NB>(SLAM(ii) {
      constexpr int i = SK(ii);
      constexpr int pid = MT::body_parentid[i], bda = MT::body_dofadr[i], nd = MT::body_dofnum[i];
      real cv = cvel[pid];
      sfor<0, nd>(SLAM(jj) {
        constexpr int d = bda + SK(jj);
        cvb[6 * d + k] = cv;
        real tt = 0;
        tt += cdk[d] * qv[d];
        cv += tt;
      });
      cvel[i] = cv;
    });
    sfor<0, NB>(SLAM(ii) { cvw[6 * SK(ii) + k] = cvel[SK(ii)]; });
  }
  TSYNC();
  // 2. cdof_dot: r[c] = (s1 v[a1] x[b1] + s2 v[a2] x[b2]) [+ (s3 .. + s4 ..) for c >= 3]
  if (t < 6 * NV) {
    const int d = t / 6, c = t - 6 * (t / 6);
    // cross_motion's operand indices and signs per component, 4 bits per c
    constexpr unsigned long long A1 = 0x122122, B1 = 0x334001, A2 = 0x001001, B2 = 0x455122;
    constexpr unsigned long long A3 = 0x455000, B3 = 0x001000, A4 = 0x334000, B4 = 0x122000;
    constexpr unsigned N1 = 0b101101, N2 = 0b010010, N3 = 0b101000, N4 = 0b010000;
    auto f4 = [&](unsigned long long P) { return (int)((P >> (4 * c)) & 15); };
    const real* v = cvb + 6 * d;
    const real* x = cdofw + 6 * d;
    const real p1 = v[f4(A1)] * x[f4(B1)], p2 = v[f4(A2)] * x[f4(B2)];
    const real p3 = v[f4(A3)] * x[f4(B3)], p4 = v[f4(A4)] * x[f4(B4)];
    const real s1 = ((N1 >> c) & 1 ? -p1 : p1) + ((N2 >> c) & 1 ? -p2 : p2);
    const real s2 = ((N3 >> c) & 1 ? -p3 : p3) + ((N4 >> c) & 1 ? -p4 : p4);
    cdw[t] = c < 3 ? s1 : s1 + s2;
  }
  TSYNC();
  // 3. per-body dof terms and cacc down the tree
  if (t < 6) {
    const int k = t;
    real cdd[NV];
    sfor<0, NV>(SLAM(dd) { cdd[SK(dd)] = cdw[6 * SK(dd) + k]; });
    real cacc[NB];
    cacc[0] = k < 3 ? 0.0 : (k == 3 ? -m.opt_gravity0 : (k == 4 ? -m.opt_gravity1 : -m.opt_gravity2));
    sfor<1, NB>(SLAM(ii) {
      constexpr int i = SK(ii);
      constexpr int pid = MT::body_parentid[i], bda = MT::body_dofadr[i], nd = MT::body_dofnum[i];
      real sum = 0;
      sfor<0, nd>(SLAM(jj) { sum += cdd[bda + SK(jj)] * qv[bda + SK(jj)]; });
      const real rt = nd ? sum : 0;
      cacc[i] = cacc[pid] + rt;
    });
    sfor<0, NB>(SLAM(ii) { cac[6 * SK(ii) + k] = cacc[SK(ii)]; });
  }
  TSYNC();
  // 4. cfrc per body
  if (t >= 1 && t < NB) {
    const int i = t;
    real ci[10], a[6], cv[6], f[6], tmp[6], tmp1[6];
    ldm<10>(ci, T.w + L.cinert + 10 * i);
    ldm<6>(a, cac + 6 * i);
    ldm<6>(cv, cvw + 6 * i);
    mul_inert_vec(f, ci, a);
    mul_inert_vec(tmp, ci, cv);
    cross_force(tmp1, cv, tmp);
    sfor<0, 6>(SLAM(kk) { cfw[6 * i + SK(kk)] = f[SK(kk)] + tmp1[SK(kk)]; });
  }
  TSYNC();
  // 5. subtree sums (children before parents), then the bias rows
  if (t < 6) {
    const int k = t;
    real cf[NB];
    sfor<1, NB>(SLAM(ii) { cf[SK(ii)] = cfw[6 * SK(ii) + k]; });
    sfor<0, NB - 1>(SLAM(ii) {
      constexpr int i = NB - 1 - SK(ii);
      constexpr int p = MT::body_parentid[i];
      if constexpr (p != 0) cf[p] += cf[i];
    });
    sfor<1, NB>(SLAM(ii) { cfw[6 * SK(ii) + k] = cf[SK(ii)]; });
  }
  TSYNC();
  if (t < NV) {
    const int d = t;
    int bi = 0;
    sfor<0, NV>(SLAM(dd) { bi = d == SK(dd) ? MT::dof_bodyid[SK(dd)] : bi; });
    real cd[6], cf[6];
    ldm<6>(cd, cdofw + 6 * d);
    ldm<6>(cf, cfw + 6 * bi);
    real r = 0;
    sfor<0, 6>(SLAM(kk) { r += cd[SK(kk)] * cf[SK(kk)]; });
    T.w[L.qfrc_bias + d] = r;
  }
  TSYNC();
}

// -------------------------------------------------- acceleration stage ---
// act_pre: actuator_force() already ran (two-wave rollout: on the helper wave)
__device__ inline void fwd_acceleration(const auto& m, const auto& L, const auto& X, const Team& T,
                                        bool act_pre = false) {
  const int nv = m.nv, nu = m.nu;
  real* ctrl = T.w + L.ctrl;
  real* af = T.w + L.afrc;
  real* amom = T.w + L.amom;
  real* qa = T.w + L.qfrc_act;
  if (!act_pre) {
    FOR_T(i, nu) {
      real c = ctrl[i], f;
      if (m.actuator_ctrllimited[i]) c = clipd(c, m.actuator_ctrlrange[2 * i], m.actuator_ctrlrange[2 * i + 1]);
      f = m.actuator_gainprm[i] * c;
      if (m.actuator_forcelimited[i]) f = clipd(f, m.actuator_forcerange[2 * i], m.actuator_forcerange[2 * i + 1]);
      af[i] = f;
    }
    TSYNC();
  }
  real* sm = T.w + L.qfrc_smooth;
  real* qp = T.w + L.qfrc_passive;
  real* qb = T.w + L.qfrc_bias;
  real* qap = T.w + L.qfrc_applied;
  real* xf = T.w + L.xfrc_applied;
  real* xipos = T.w + L.xipos;
  real* scom = T.w + L.scom;
  real* cdof = T.w + L.cdof;
  real* qs = T.w + L.qacc_smooth;
  // any nonzero xfrc_applied on a non-world body? (else the per-body loop below
  // skips every body, so leaving it out changes nothing)
  unsigned long long fmask = 0;
  for (int i0 = 6; i0 < 6 * m.nbody; i0 += TEAM_SIZE) fmask |= __ballot(i0 + T.tid < 6 * m.nbody && xf[i0 + T.tid] != 0);
  const bool anyf = fmask != 0ull;
  FOR_T(j, nv) {
    real s;
    if (act_pre) {
      s = qa[j];
    } else {
      s = 0;
      for (int i = 0; i < nu; i++) s += amom[i * nv + j] * af[i];
      qa[j] = s;
    }
    real v = qp[j] - qb[j];
    v += qap[j];
    v += s;
    // xfrc_applied: jac columns of dof j at each loaded body's COM
    for (int b = 1; anyf && b < m.nbody; b++) {
      real f[6];
      ldm<6>(f, xf + 6 * b);
      if (f[0] == 0 && f[1] == 0 && f[2] == 0 && f[3] == 0 && f[4] == 0 && f[5] == 0) continue;
      real p[3] = {xipos[3 * b], xipos[3 * b + 1], xipos[3 * b + 2]}, jp[3], jr[3] = {0, 0, 0};
      jac_col(m, X, scom, cdof, p, b, j, jp);
      int bb = b;
      while (bb && !m.body_dofnum[bb]) bb = m.body_parentid[bb];
      if (bb && X.isanc[(m.body_dofadr[bb] + m.body_dofnum[bb] - 1) * nv + j]) {
        jr[0] = cdof[6 * j]; jr[1] = cdof[6 * j + 1]; jr[2] = cdof[6 * j + 2];
      }
      real t1 = jp[0] * f[0] + jp[1] * f[1] + jp[2] * f[2];
      real t2 = jr[0] * f[3] + jr[1] * f[4] + jr[2] * f[5];
      v += t1 + t2;
    }
    sm[j] = v;
    qs[j] = v;
  }
  TSYNC();
  solve_ld(m, X, T, T.w + L.qLD, T.w + L.qLDinv, qs);
}

// s0 + v[lane 0] + v[lane 1] + ... + v[lane n-1], in that order
// fwd_acceleration(act_pre = true) for a compile-time model with the dof
// ancestor masks compiled in (the rollout's primary chain), in wave-uniform
// registers: qfrc_smooth's rows and the tree L'DL solve of qacc_smooth
// (solve_ld_rows' sequence, as euler_finish_u runs it) with one LDS read
// phase and one write.  Returns false, having done nothing, when a body
// carries xfrc_applied (the general path forms those Jacobian columns).
template <class MT>
__device__ inline bool fwd_acceleration_u(const auto& m, const auto& L, const auto& X, const Team& T) {
  constexpr int NV = MT::nv, NB = MT::nbody;
  using XT = std::remove_cvref_t<decltype(X)>;
  (void)X;
  const real* xf = T.w + L.xfrc_applied;
  static_assert(6 * NB <= TEAM_SIZE, "one ballot over xfrc_applied");
  if (__ballot(T.tid >= 6 && T.tid < 6 * NB && xf[T.tid] != 0) != 0ull) return false;
  const real *qp = T.w + L.qfrc_passive, *qb = T.w + L.qfrc_bias, *qap = T.w + L.qfrc_applied;
  const real* qa = T.w + L.qfrc_act;
  const real *LD = T.w + L.qLD, *LDinv = T.w + L.qLDinv;
  real v[NV], x[NV], dinv[NV], LDr[NV][NV];
  sfor<0, NV>(SLAM(jj) {
    constexpr int j = SK(jj);
    real t = qp[j] - qb[j];
    t += qap[j];
    t += qa[j];
    v[j] = t;
    x[j] = t;
    dinv[j] = LDinv[j];
  });
  sfor<0, NV>(SLAM(ii) {
    constexpr int i = SK(ii);
    sfor<0, i>(SLAM(jj) {
      constexpr int j = SK(jj);
      if constexpr ((XT::pmask[i] >> j) & 1) LDr[i][j] = LD[i * NV + j];
    });
  });
  // x[j] -= LD[i][j] x[i] for j in anc(i), i descending, where x[i] != 0
  sfor<0, NV>(SLAM(ii) {
    constexpr int i = NV - 1 - SK(ii);
    const bool nz = x[i] != 0;
    sfor<0, i>(SLAM(jj) {
      constexpr int j = SK(jj);
      if constexpr ((XT::pmask[i] >> j) & 1) {
        const real u = x[j] - LDr[i][j] * x[i];
        x[j] = nz ? u : x[j];
      }
    });
  });
  sfor<0, NV>(SLAM(ii) { x[SK(ii)] *= dinv[SK(ii)]; });
  // x[i] -= LD[i][j] x[j] for j in anc(i) descending, i ascending
  sfor<0, NV>(SLAM(ii) {
    constexpr int i = SK(ii);
    sfor<0, i>(SLAM(jj) {
      constexpr int j = i - 1 - SK(jj);
      if constexpr ((XT::pmask[i] >> j) & 1) x[i] -= LDr[i][j] * x[j];
    });
  });
  real vv = v[0], xv = x[0];
  sfor<1, NV>(SLAM(ii) {
    vv = T.tid == SK(ii) ? v[SK(ii)] : vv;
    xv = T.tid == SK(ii) ? x[SK(ii)] : xv;
  });
  if (T.tid < NV) {
    T.w[L.qfrc_smooth + T.tid] = vv;
    T.w[L.qacc_smooth + T.tid] = xv;
  }
  TSYNC();
  return true;
}

__device__ __forceinline__ real lane_sum(real s0, real v, int n) {
  for (int i = 0; i < n; i++) s0 += bcast(v, i);
  return s0;
}
// the same ordered sum over the lanes of a (wave-uniform) mask only: lanes
// outside it hold -0.0, and x + (-0.0) == x for every x, so skipping them is exact
__device__ __forceinline__ real lane_sum_mask(real s0, real v, unsigned long long mask) {
  for (unsigned long long mm = mask; mm; mm &= mm - 1) s0 += bcast(v, __builtin_ctzll(mm));
  return s0;
}

// constraint cost of residuals `jar`; force/state per row, qfrc_constraint per dof.
// With `chg`: *chg (uniform) = some row's state differs from the one it held
// on entry (one-wave teams; wider teams report a change unconditionally)
__device__ inline real constraint_update(const auto& m, const auto& L, const auto& C, const Team& T,
                                           const real* jar, int* chg = nullptr) {
  const int nv = m.nv, ne = T.iw[L.nefc];
  real* D = T.w + L.efc_D;
  real* force = T.w + L.efc_force;
  real* J = T.w + L.efc_J;
  real* qc = T.w + L.qfrc_con;
  int* state = T.iw + L.efc_state;
  real* term = T.c + C.cterm;
  bool ch = false;
  FOR_T(i, ne) {
    real jr = jar[i];
    if (chg) ch |= state[i] != (jr < 0 ? 1 : 0);
    if (jr < 0) {
      real Di = D[i];
      force[i] = -Di * jr;
      state[i] = 1;
      term[i] = 0.5 * Di * jr * jr;
    } else {
      force[i] = 0;
      state[i] = 0;
    }
  }
  if (chg) *chg = T.nt <= 64 ? (__ballot(ch) != 0ull) : 1;
  TSYNC();
  FOR_T(j, nv) {
    real s = 0;
    int i = 0;
    for (; i + 8 <= ne; i += 8) {  // eight rows' loads in flight, additions in row order
      real jj[8], ff[8];
#pragma unroll
      for (int q = 0; q < 8; q++) {
        jj[q] = J[(i + q) * nv + j];
        ff[q] = force[i + q];
      }
#pragma unroll
      for (int q = 0; q < 8; q++) s += jj[q] * ff[q];
    }
    for (; i < ne; i++) s += J[i * nv + j] * force[i];
    qc[j] = s;
  }
  if (ne <= TEAM_SIZE && T.nt == TEAM_SIZE) {
    // the active rows' terms added in row order on broadcasts (uniform)
    const int r = T.tid;
    const real jr = r < ne ? jar[r] : (real)0;
    const bool act = r < ne && jr < 0;
    const real tv = act ? 0.5 * D[r] * jr * jr : -0.0;
    const real cost = lane_sum_mask(0.0, tv, __ballot(act));
    TSYNC();
    return cost;
  }
  if (T.tid == 0) {
    real cost = 0;
    for (int i = 0; i < ne; i++)
      if (state[i]) cost += term[i];
    T.c[C.bc] = cost;
  }
  TSYNC();
  return T.c[C.bc];
}

// compile-time lane map of the Hessian build for NVC dofs: lane t owns up to
// HB consecutive entries of one lower-triangle row (row r, columns c0 ..
// c0 + cnt - 1); every row takes ceil((r + 1) / HB) lanes
constexpr int HB = 8;
template <int NVC>
struct HessLanes {
  int n = 0;
  constexpr HessLanes() {
    for (int rr = 0; rr < NVC; rr++) n += rr / HB + 1;
  }
};
template <int NVC>
constexpr bool hess_lanes_ok() {
  if constexpr (NVC > 0) return HessLanes<NVC>{}.n <= 64;
  else return false;
}

__device__ inline void hessian_factor(const auto& m, const auto& L, const auto& C, const Team& T,
                                      real* H) {
  constexpr int NVC = nv_const<std::remove_cvref_t<decltype(m)>>();
  const int nv = NVC > 0 ? NVC : m.nv, ne = T.iw[L.nefc];
  real* J = T.w + L.efc_J;
  real* D = T.w + L.efc_D;
  real* qM = T.w + L.qM;
  int* state = T.iw + L.efc_state;
  // one lane per lower-triangle entry (r, c); the active rows walked in
  // ascending order (as a ballot when nefc <= 64), inactive rows skipped as
  // the oracle skips them
  const int ntri = nv * (nv + 1) / 2;
  // the active set as ballots of 64 rows (up to HMASK of them, before the
  // entry loop, with every lane active)
  constexpr int HMASK = 4;
  const bool bal = ne <= 64 * HMASK && T.nt == 64;
  unsigned long long am[HMASK];
#pragma unroll
  for (int q = 0; q < HMASK; q++) {
    const int i = 64 * q + T.tid;
    am[q] = bal && 64 * q < ne ? __ballot(i < ne && state[i] != 0) : 0ull;
  }
  // (fp64 only: the fp32 FD sweep's instance measured slower, 4.31 -> 4.41 ms a
  // chunk, while the fp64 rollout's chunk went 1.509 -> 1.395 ms)
  if constexpr (hess_lanes_ok<NVC>() && ILQG_HESS_ROWS && sizeof(real) == 8) {
    if (bal) {
      // lane t: entries (r, c0 .. c0 + cnt - 1) of one row; per active row i
      // (ascending, the oracle's order) J(i, r) D(i) is formed once and each
      // entry adds (J(i, r) D(i)) J(i, c) -- the per-entry form's operations
      constexpr int NL = HessLanes<NVC>{}.n;
      const int t = T.tid;
      const bool own = t < NL;
      // lane t's block: rows take rr / HB + 1 lanes each, in row order
      int r = 0, c0 = 0, cnt = 0;
      {
        int acc = 0;
        sfor<0, NVC>(SLAM(rq) {
          constexpr int rr = SK(rq), nb = rr / HB + 1;
          if (t >= acc && t < acc + nb) {
            r = rr;
            c0 = (t - acc) * HB;
            cnt = rr + 1 - c0 < HB ? rr + 1 - c0 : HB;
          }
          acc += nb;
        });
      }
      real h[HB];
#pragma unroll
      for (int q = 0; q < HB; q++) h[q] = 0;
#pragma unroll
      for (int w = 0; w < HMASK; w++) {
        for (unsigned long long mm = am[w]; mm; mm &= mm - 1) {
          const int i = 64 * w + __builtin_ctzll(mm);
          const real* Ji = J + i * nv;
          const real ad = Ji[r] * D[i];
          real b[HB];
#pragma unroll
          for (int q = 0; q < HB; q++) b[q] = Ji[c0 + (q < cnt ? q : 0)];
#pragma unroll
          for (int q = 0; q < HB; q++)
            if (q < cnt) h[q] += ad * b[q];
        }
      }
      if (own) {
#pragma unroll
        for (int q = 0; q < HB; q++)
          if (q < cnt) H[r * nv + c0 + q] = qM[r * nv + c0 + q] + h[q];
      }
      goto built;
    }
  }
  FOR_T(e, ntri) {
    int r = (int)((sqrtf(8.0f * (float)e + 1.0f) - 1.0f) * 0.5f);
    while (r * (r + 1) / 2 > e) r--;
    while ((r + 1) * (r + 2) / 2 <= e) r++;
    const int c = e - r * (r + 1) / 2;
    real h = 0;
    if (bal) {
      // eight active rows' loads in flight at once, the terms added in row order
#pragma unroll
      for (int w = 0; w < HMASK; w++) {
        for (unsigned long long mm = am[w]; mm;) {
          int id[8];
          real a[8], d[8], b[8];
#pragma unroll
          for (int q = 0; q < 8; q++) {
            id[q] = mm ? 64 * w + __builtin_ctzll(mm) : -1;
            mm &= mm - 1;
          }
#pragma unroll
          for (int q = 0; q < 8; q++) {
            const int i = id[q] < 0 ? id[0] : id[q];
            a[q] = J[i * nv + r];
            d[q] = D[i];
            b[q] = J[i * nv + c];
          }
#pragma unroll
          for (int q = 0; q < 8; q++)
            if (id[q] >= 0) h += a[q] * d[q] * b[q];
        }
      }
    } else {
      for (int i = 0; i < ne; i++)
        if (state[i]) h += J[i * nv + r] * D[i] * J[i * nv + c];
    }
    H[r * nv + c] = qM[r * nv + c] + h;
  }
built:
  TSYNC();
  STAMP(31);
  if (nv <= RMAX) {
    cholesky_rows(nv, T.tid, H);
    return;
  }
#if ILQG_CHOL32
  if (nv <= 32 && T.nt == TEAM_SIZE) {
    cholesky_rows32<nv_const<std::remove_cvref_t<decltype(m)>>()>(nv, T.tid, H);
    return;
  }
#endif
  if (nv <= SERIAL_NV) {
    if (T.tid == 0) {
      for (int j = 0; j < nv; j++) {
        real t = H[j * nv + j];
        if (j) t -= tdot(H + j * nv, H + j * nv, j);
        if (t < MINVAL) t = MINVAL;
        H[j * nv + j] = sqrt(t);
        t = 1 / H[j * nv + j];
        for (int i = j + 1; i < nv; i++) H[i * nv + j] = (H[i * nv + j] - tdot(H + i * nv, H + j * nv, j)) * t;
      }
    }
    TSYNC();
    return;
  }
  if (nv <= TEAM_SIZE && T.nt == TEAM_SIZE) {
    // lane i owns row i: per column j every row's dot product with row j at
    // once (the diagonal's is lane j's), the pivot broadcast from lane j
    const int i = T.tid;
    const bool own = i < nv;
    for (int j = 0; j < nv; j++) {
      const bool part = own && i >= j;
      const real s = part ? tdotw(H + i * nv, H + j * nv, j) : (real)0;
      real t = 0;
      if (i == j) {
        t = H[j * nv + j];
        if (j) t -= s;
        if (t < MINVAL) t = MINVAL;
        t = sqrt(t);
      }
      const real d = bcast(t, j);
      const real tinv = 1 / d;
      if (i == j) H[j * nv + j] = d;
      if (part && i > j) H[i * nv + j] = (H[i * nv + j] - s) * tinv;
      TSYNC();
    }
    return;
  }
  for (int j = 0; j < nv; j++) {
    if (T.tid == 0) {
      real t = H[j * nv + j];
      if (j) t -= tdot(H + j * nv, H + j * nv, j);
      if (t < MINVAL) t = MINVAL;
      H[j * nv + j] = sqrt(t);
      T.c[C.bc + 1] = 1 / H[j * nv + j];
    }
    TSYNC();
    const real tinv = T.c[C.bc + 1];
    FOR_T(i, nv) {
      if (i > j) H[i * nv + j] = (H[i * nv + j] - tdot(H + i * nv, H + j * nv, j)) * tinv;
    }
    TSYNC();
  }
}

// ---- the exact line search's iterations (oracle linesearch), rows uniform --
// After the lane form's eval(0) (one constraint row per lane), a solve with
// NE <= LS_NE rows copies rows 0..NE-1 (jr, jv, D, D jv^2) into wave-uniform
// registers once, and each iteration then forms every row's term on every
// lane and adds the active ones in row order -- the oracle's expressions and
// order, inactive rows adding -0.0 (the exact identity) -- with no cross-lane
// operation on the chain d1 -> step -> x -> term -> d1.  The active set is
// still taken lane-parallel (one ballot), and d2 and its reciprocal are formed
// again only when it changes.  At tolerance 0 (the FD solves,
// mjderivative.cpp:241-242) most line searches run all LS_ITER iterations.
#ifndef ILQG_LS_NE
#define ILQG_LS_NE 8
#endif
constexpr int LS_NE = ILQG_LS_NE;
// the compile-time-model Newton solver's line search entirely on uniform rows
// (linesearch_u, rows padded to 4 or 8): the rollout's solves (model
// tolerance, ~1.4 iterations per line search) spend most of theirs in eval(0)
#ifndef ILQG_LS_U
#define ILQG_LS_U 0
#endif
constexpr bool LS_U = ILQG_LS_U != 0;
// Speculative bisection (FD translation units): at tolerance 0 nine in ten
// line-search iterations are bisection steps (the Newton candidate falls
// outside the bracket; measured on the oracle over the bench's FD sweep), and
// a run of them is a walk down a binary tree whose nodes are fixed by the
// bracket alone: node alpha = 0.5 (lo + hi), then lo or hi := alpha by the
// sign of d1 there.  Once an iteration bisects, lane t evaluates node t of the
// next LS_TREE_K levels (63 nodes) at once -- its alpha by the same midpoint
// sequence, d1 and d2 by the same row sums, its own Newton candidate
// alpha - d1 / d2 and the bisection test against its bracket -- and the wave
// then walks the tree from the root with the three ballots: a node where
// |d1| < gtol (or the LS_ITER-th iteration) ends the search, a node whose
// Newton candidate lies inside its bracket hands its state (alpha, d1, d2,
// lo, hi) back to the serial loop, else the walk descends.  Every value the
// walk uses is the one the serial iteration computes, so the result is the
// same; up to six iterations cost one pass.  Returns true when the search ended.
#ifndef ILQG_LS_TREE
#define ILQG_LS_TREE 1
#endif
constexpr bool LS_TREE = ILQG_LS_TREE != 0;
constexpr int LS_TREE_K = 6;
// rows up to which the tree runs (the uniform-row limit: at tolerance 0 the
// hopper's bisection steps fall on 4-row (31 %) and 8-row (48 %) solves)
#ifndef ILQG_LS_TREE_NE
#define ILQG_LS_TREE_NE 8
#endif
constexpr int LS_TREE_NE = ILQG_LS_TREE_NE;
template <int NE>
__device__ inline bool ls_bisect_tree(const real (&ujr)[NE], const real (&ujv)[NE], const real (&uD)[NE],
                                      const real (&uc2)[NE], real g1, real g2, real gtol, real& alpha, real& d1,
                                      real& d2c, real& lo, real& hi, int& it) {
  const int t = (int)__lane_id();
  const unsigned p1 = (unsigned)(t < 63 ? t : 62) + 1u;  // heap index + 1: 1 b1 b2 .. b_depth
  const int dt = 31 - __builtin_clz(p1);
  real l_ = lo, h_ = hi, a_ = 0.5 * (lo + hi);
  sfor<1, LS_TREE_K>(SLAM(kk) {
    constexpr int lev = SK(kk);
    const bool go = lev <= dt;
    const bool right = go && ((p1 >> (go ? dt - lev : 0)) & 1u);  // d1 < 0 at the parent: lo := its alpha
    l_ = (go && right) ? a_ : l_;
    h_ = (go && !right) ? a_ : h_;
    const real mid = 0.5 * (l_ + h_);
    a_ = go ? mid : a_;
  });
  real s = g1 + g2 * a_, d2 = g2;
  sfor<0, NE>(SLAM(jj) {
    constexpr int j = SK(jj);
    const real x = ujr[j] + a_ * ujv[j];
    const real tt = uD[j] * x * ujv[j];
    const bool ac = x < 0;
    s += ac ? tt : (real)-0.0;
    d2 += ac ? uc2[j] : (real)-0.0;
  });
  const bool neg = s < 0;
  const real lo2 = neg ? a_ : l_, hi2 = neg ? h_ : a_;
  const real cand = a_ - s / d2;
  const unsigned long long mstop = __ballot(fabs(s) < gtol), mneg = __ballot(neg),
                           mbis = __ballot(hi2 >= 0 && !(cand > lo2 && cand < hi2));
  // the walk is scalar: the iteration count and node index stay in SGPRs
  // (readfirstlane: the compiler cannot prove them uniform and would run the
  // walk under exec masks)
  int n = 0;
  it = __builtin_amdgcn_readfirstlane(it);
  for (int lev = 0; lev < LS_TREE_K; lev++) {
    it++;
    if (((mstop >> n) & 1ull) || it >= LS_ITER) {
      alpha = bcast(a_, n);
      return true;
    }
    if (!((mbis >> n) & 1ull) || lev == LS_TREE_K - 1) {
      alpha = bcast(a_, n);
      d1 = bcast(s, n);
      d2c = bcast(d2, n);
      lo = bcast(lo2, n);
      hi = bcast(hi2, n);
      return false;
    }
    n = __builtin_amdgcn_readfirstlane(2 * n + 1 + (int)((mneg >> n) & 1ull));
  }
  return false;  // not reached
}

// the iterations on rows already in wave-uniform registers (ujr, ujv, uD, uc2)
template <int NE>
__device__ inline real ls_iterate_u(const real (&ujr)[NE], const real (&ujv)[NE], const real (&uD)[NE],
                                    const real (&uc2)[NE], real g1, real g2, real jr, real jv, bool row, real d1,
                                    real d2c, real rd2, unsigned long long pmask, real gtol, int& iters) {
  real alpha = 0, lo = 0, hi = -1;
  int it = 0;
  while (it < LS_ITER) {
    it = __builtin_amdgcn_readfirstlane(it);
    real anew = alpha - div_ref_lane<0>(d1, d2c, rd2);
    const bool bis = __ballot(hi >= 0 && !(anew > lo && anew < hi)) != 0;  // uniform
    if constexpr (LS_TREE && NE <= LS_TREE_NE) {
      if (bis) {
        if (ls_bisect_tree<NE>(ujr, ujv, uD, uc2, g1, g2, gtol, alpha, d1, d2c, lo, hi, it)) break;
        rd2 = rcp_ref(d2c);
        pmask = __ballot(row && jr + alpha * jv < 0);
        continue;
      }
    }
    if (bis) anew = 0.5 * (lo + hi);
    alpha = anew;
    const unsigned long long am = __ballot(row && jr + alpha * jv < 0);
    real s = g1 + g2 * alpha;
    bool act[NE];
    sfor<0, NE>(SLAM(jj) {
      constexpr int j = SK(jj);
      const real x = ujr[j] + alpha * ujv[j];
      const real t = uD[j] * x * ujv[j];
      act[j] = x < 0;
      s += act[j] ? t : (real)-0.0;
    });
    d1 = s;
    it++;
    if (am != pmask) {
      real d2 = g2;
      sfor<0, NE>(SLAM(jj) { d2 += act[SK(jj)] ? uc2[SK(jj)] : (real)-0.0; });
      d2c = d2;
      rd2 = rcp_ref(d2c);
      pmask = am;
    }
    if (__ballot(fabs(d1) < gtol) != 0) break;  // uniform
    if (d1 < 0) lo = alpha; else hi = alpha;
  }
  iters = it;
  return alpha;
}
template <int NE>
__device__ inline real ls_iterate_rows(real g1, real g2, real jr, real jv, real Di, real c2, bool row, real d1,
                                       real d2c, real rd2, unsigned long long pmask, real gtol, int& iters) {
  real ujr[NE], ujv[NE], uD[NE], uc2[NE];
  sfor<0, NE>(SLAM(jj) {
    constexpr int j = SK(jj);
    ujr[j] = bcast(jr, j);
    ujv[j] = bcast(jv, j);
    uD[j] = bcast(Di, j);
    uc2[j] = bcast(c2, j);
  });
  return ls_iterate_u<NE>(ujr, ujv, uD, uc2, g1, g2, jr, jv, row, d1, d2c, rd2, pmask, gtol, iters);
}

// the whole exact line search (eval(0) included) on wave-uniform rows, for a
// solve with at most NE rows (lanes >= ne hold jr = jv = Di = 0, which never
// activate: x = 0 + alpha 0 is not < 0): eval(0)'s two ordered sums formed on
// every lane from the broadcast rows instead of two lane walks -- the lane
// form's expressions and order (linesearch_rows below), inactive rows adding
// the exact identity -0.0
template <int NE>
__device__ inline real linesearch_u(int ne, real g1, real g2, real jr, real jv, real Di, bool row) {
  real ujr[NE], ujv[NE], uD[NE], uc2[NE];
  sfor<0, NE>(SLAM(jj) {
    constexpr int j = SK(jj);
    ujr[j] = bcast(jr, j);
    ujv[j] = bcast(jv, j);
    uD[j] = bcast(Di, j);
  });
  real d1 = g1 + g2 * 0.0, d2c = g2;
  bool a0[NE];
  sfor<0, NE>(SLAM(jj) {
    constexpr int j = SK(jj);
    uc2[j] = uD[j] * ujv[j] * ujv[j];
    const real x0 = ujr[j] + 0.0 * ujv[j];
    const real c10 = uD[j] * x0 * ujv[j];
    a0[j] = x0 < 0;
    d1 += a0[j] ? c10 : (real)-0.0;
  });
  if (__ballot(d1 >= 0) != 0) return 0;  // uniform
  sfor<0, NE>(SLAM(jj) { d2c += a0[SK(jj)] ? uc2[SK(jj)] : (real)-0.0; });
  const unsigned long long am = __ballot(row && jr + 0.0 * jv < 0);
  const real rd2 = rcp_ref(d2c);
  int iters = 0;
  const real alpha = ls_iterate_u<NE>(ujr, ujv, uD, uc2, g1, g2, jr, jv, row, d1, d2c, rd2, am,
                                      LS_TOL * fabs(d1), iters);
  (void)ne;
  (void)iters;
  return alpha;
}

// the line search from the lane form's state after eval(0): returns alpha
__device__ inline real ls_iterate(int ne, real g1, real g2, real jr, real jv, real Di, real c2, bool row, real d1,
                                  real d2c, real rd2, unsigned long long pmask, int& iters) {
  const real gtol = LS_TOL * fabs(d1);
  switch (ne) {
#define ILQG_LS_CASE(n)                                                                     \
  case n:                                                                                   \
    if constexpr (n <= LS_NE) return ls_iterate_rows<n>(g1, g2, jr, jv, Di, c2, row, d1, d2c, rd2, pmask, gtol, iters); \
    break;
    ILQG_LS_CASE(1) ILQG_LS_CASE(2) ILQG_LS_CASE(3) ILQG_LS_CASE(4)
    ILQG_LS_CASE(5) ILQG_LS_CASE(6) ILQG_LS_CASE(7) ILQG_LS_CASE(8)
#undef ILQG_LS_CASE
    default:
      break;
  }
  // more rows: the terms stay on their lanes, summed in lane order over the
  // active ones
  real alpha = 0, lo = 0, hi = -1, d2 = d2c;
  int it = 0;
  while (it < LS_ITER) {
    real anew = alpha - div_ref_lane<0>(d1, d2, rd2);
    if (hi >= 0 && !(anew > lo && anew < hi)) anew = 0.5 * (lo + hi);
    alpha = anew;
    const real x = jr + alpha * jv;
    const bool on = row && x < 0;
    const real c1 = Di * x * jv;
    const unsigned long long am = __ballot(on);
    d1 = lane_sum_mask(g1 + g2 * alpha, c1, am);
    if (am != pmask) {
      d2c = lane_sum_mask(g2, c2, am);
      rd2 = rcp_ref(d2c);
      pmask = am;
    }
    d2 = d2c;
    it++;
    if (fabs(d1) < gtol) break;
    if (d1 < 0) lo = alpha; else hi = alpha;
  }
  iters = it;
  return alpha;
}

__device__ inline void solver_newton(const auto& m, const auto& L, const auto& C, const Team& T,
                                     int maxiter, real tol) {
  constexpr int NVC = nv_const<std::remove_cvref_t<decltype(m)>>();
  const int nv = NVC > 0 ? NVC : m.nv, ne = T.iw[L.nefc];
  const real scale = 1 / (m.stat_meaninertia * (nv > 1 ? nv : 1));
  real* s = T.w + L.s_newton;
  real *Ma = s, *grad = s + nv, *search = s + 2 * nv, *Mv = s + 3 * nv, *H = s + 4 * nv;
  real* jar = s + 4 * nv + nv * nv;
  real* Jv = jar + ne;
  real* qM = T.w + L.qM;
  real* qacc = T.w + L.qacc;
  real* J = T.w + L.efc_J;
  real* aref = T.w + L.efc_aref;
  real* qfs = T.w + L.qfrc_smooth;
  real* qas = T.w + L.qacc_smooth;
  real* qc = T.w + L.qfrc_con;
  real* Dv = T.w + L.efc_D;
  real* bc = T.c + C.bc;
  FOR_T(i, nv) Ma[i] = tdotw(qM + i * nv, qacc, nv);
  FOR_T(i, ne) jar[i] = tdotw(J + i * nv, qacc, nv) - aref[i];
  TSYNC();
  real ccost = constraint_update(m, L, C, T, jar);
  if (T.tid == 0) {
    real g = 0;
    for (int j = 0; j < nv; j++) g += (Ma[j] - qfs[j]) * (qacc[j] - qas[j]);
    bc[2] = 0.5 * g + ccost;
  }
  FOR_T(j, nv) grad[j] = (Ma[j] - qfs[j]) - qc[j];
  TSYNC();
  real cost = bc[2];
  hessian_factor(m, L, C, T, H);
  STAMP(19);
  int iter = 0;
#ifdef ILQG_STAMPS
  CNT_ADD(9, 1ull);
#endif
  while (iter < maxiter) {
    // search = -H^-1 grad ; line search ; all on lane 0 except the parallel products
    if (nv <= RMAX) {
      chol_solve_rows(nv, T.tid, H, grad, search);
    } else if (ILQG_CHOLS == 1 && nv <= 32 && T.nt == TEAM_SIZE) {
      chol_solve_rows32(nv, T.tid, H, grad, search);
    } else if (ILQG_CHOLS == 2 && nv <= 32 && T.nt == TEAM_SIZE) {
      chol_solve_u2<nv_const<std::remove_cvref_t<decltype(m)>>()>(nv, T.tid, H, grad, search);
    } else if (nv <= TEAM_SIZE) {
      chol_solve_wave(nv, T.tid, H, grad, search);
    } else {
      if (T.tid == 0) {
        for (int i = 0; i < nv; i++) search[i] = grad[i];
        for (int i = 0; i < nv; i++) {
          if (i) search[i] -= tdot(H + i * nv, search, i);
          search[i] /= H[i * nv + i];
        }
        for (int i = nv - 1; i >= 0; i--) {
          for (int j = i + 1; j < nv; j++) search[i] -= H[j * nv + i] * search[j];
          search[i] /= H[i * nv + i];
        }
        for (int j = 0; j < nv; j++) search[j] = -search[j];
      }
      TSYNC();
    }
    STAMP(14);
    FOR_T(i, nv) Mv[i] = tdotw(qM + i * nv, search, nv);
    FOR_T(i, ne) Jv[i] = tdotw(J + i * nv, search, nv);
    TSYNC();
    STAMP(15);
    if (ne <= TEAM_SIZE && T.nt == TEAM_SIZE) {
      // the same exact line search on every lane (uniform), the row sums in row
      // order over the active rows' lanes (fwd_constraint_fast's form)
      real alpha = 0;
      const real snorm = sqrt(tdot(search, search, nv));
      if (!(snorm < MINVAL)) {
        const int r = T.tid;
        const bool row = r < ne;
        const real jr = row ? jar[r] : (real)0, jv = row ? Jv[r] : (real)0, Di = row ? Dv[r] : (real)0;
        real g1 = 0, g2 = 0, d1, d2;
        for (int j = 0; j < nv; j++) g1 += search[j] * (Ma[j] - qfs[j]);
        for (int j = 0; j < nv; j++) g2 += search[j] * Mv[j];
        unsigned long long pmask = 0;
        bool have = false;
        real d2c = 0, rd2 = 0;
        const real c2 = Di * jv * jv;
        auto eval = [&](real a) {
          const real x = jr + a * jv;
          const bool on = row && x < 0;
          const real c1 = Di * x * jv;
          const unsigned long long am = __ballot(on);
          d1 = lane_sum_mask(g1 + g2 * a, c1, am);
          if (!have || am != pmask) {
            d2c = lane_sum_mask(g2, c2, am);
            rd2 = rcp_ref(d2c);
            pmask = am;
            have = true;
          }
          d2 = d2c;
        };
        eval(0.0);
        if (!(d1 >= 0)) {
          int iters = 0;
          alpha = ls_iterate(ne, g1, g2, jr, jv, Di, c2, row, d1, d2c, rd2, pmask, iters);
        }
      }
      if (T.tid == 0) bc[3] = alpha;
    } else if (T.tid == 0) {
      real alpha = 0;
      real snorm = sqrt(tdot(search, search, nv));
      if (!(snorm < MINVAL)) {
        real g1 = 0, g2 = 0, d1, d2, lo = 0, hi = -1;
        for (int j = 0; j < nv; j++) g1 += search[j] * (Ma[j] - qfs[j]);
        for (int j = 0; j < nv; j++) g2 += search[j] * Mv[j];
        auto eval = [&](real a) {
          d1 = g1 + g2 * a;
          d2 = g2;
          for (int i = 0; i < ne; i++) {
            real jv = Jv[i];
            real x = jar[i] + a * jv;
            if (x < 0) {
              real Di = Dv[i];
              d1 += Di * x * jv;
              d2 += Di * jv * jv;
            }
          }
        };
        eval(0.0);
        if (!(d1 >= 0)) {  // oracle: return 0 iff d1 >= 0 (a NaN proceeds)
          real gtol = LS_TOL * fabs(d1);
          for (int it = 0; it < LS_ITER; it++) {
            real anew = alpha - d1 / d2;
            if (hi >= 0 && !(anew > lo && anew < hi)) anew = 0.5 * (lo + hi);
            alpha = anew;
            eval(alpha);
            if (fabs(d1) < gtol) break;
            if (d1 < 0) lo = alpha; else hi = alpha;
          }
        }
      }
      bc[3] = alpha;
    }
    TSYNC();
    STAMP(16);
    const real alpha = bc[3];
    if (alpha == 0) break;
    FOR_T(j, nv) {
      qacc[j] += alpha * search[j];
      Ma[j] += alpha * Mv[j];
    }
    FOR_T(i, ne) jar[i] += alpha * Jv[i];
    TSYNC();
    iter++;
#ifdef ILQG_STAMPS
    CNT_ADD(8, 1ull);
#endif
    STAMP(17);
    real oldcost = cost;
    int chg = 1;
    ccost = constraint_update(m, L, C, T, jar, &chg);
    FOR_T(j, nv) grad[j] = (Ma[j] - qfs[j]) - qc[j];
    TSYNC();
    // the same scalars on every lane (uniform): no LDS round trip
    const real c2 = 0.5 * gauss_w(Ma, qfs, qacc, qas, nv) + ccost;
    const real improvement = scale * (oldcost - c2);
    const real gradient = scale * sqrt(tdotw(grad, grad, nv));
    STAMP(18);
    cost = c2;
    if (improvement < tol || gradient < tol) break;
    // the factor is a function of (qM, J, D, efc_state) alone: rebuilt only
    // when some row's state changed since it was computed (the same bits)
    if (chg) hessian_factor(m, L, C, T, H);
    STAMP(19);
  }
}


// ---------------------------------------------------------------------------
// Newton solver, wave-parallel form for nefc <= 64 (one constraint row per
// lane).  Every ordered reduction over rows (constraint cost, line-search
// derivatives) keeps the oracle's row order: each lane forms its row's term,
// then the terms are added in lane order through v_readlane.  A row that the
// oracle skips contributes -0.0, the exact identity of IEEE addition.  The
// Hessian factor is reused while the active set is unchanged: it is a
// function of (qM, J, D, active set) only, so the reused factor is the one
// the oracle recomputes, bit for bit.

// constraint_update for row registers: returns the cost (uniform) and the
// active-row mask; with `full` also force/state and qfrc_constraint = J' force
__device__ inline real cu_fast(const auto& m, const auto& L, const Team& T, real jr, real Di, bool full,
                                 unsigned long long& mask, bool want_cost = true) {
  const int nv = m.nv, ne = T.iw[L.nefc];
  const int r = T.tid;
  const bool row = r < ne;
  const bool act = row && jr < 0;
  if (full) {
    real* force = T.w + L.efc_force;
    int* state = T.iw + L.efc_state;
    if (row) {
      force[r] = act ? -Di * jr : 0.0;
      state[r] = act ? 1 : 0;
    }
    TSYNC();
    real* J = T.w + L.efc_J;
    real* qc = T.w + L.qfrc_con;
    // rows with zero force add J * 0 = +-0 to a sum that is never -0 (it starts
    // at +0): skipping them is exact
    const unsigned long long am = __ballot(act);
    FOR_T(j, nv) {
      real s = 0;
      for (unsigned long long mm = am; mm; mm &= mm - 1) {
        const int i = __builtin_ctzll(mm);
        s += J[i * nv + j] * force[i];
      }
      qc[j] = s;
    }
    TSYNC();
  }
  mask = __ballot(act);
  if (!want_cost) return 0.0;
  const real tv = act ? 0.5 * Di * jr * jr : -0.0;
  return lane_sum_mask(0.0, tv, mask);
}

// 0.5 * sum_j (Ma_j - qfs_j)(qacc_j - qas_j), every lane (uniform)
__device__ inline real gauss_u(int nv, const real* Ma, const real* qfs, const real* qacc, const real* qas) {
  real g = 0;
  for (int j = 0; j < nv; j++) g += (Ma[j] - qfs[j]) * (qacc[j] - qas[j]);
  return 0.5 * g;
}

// amask: the active rows (efc_state != 0) as a ballot, walked in ascending order
__device__ inline void hessian_build_fast(const auto& m, const auto& L, const Team& T, real* H,
                                          unsigned long long amask) {
  const int nv = m.nv;
  real* J = T.w + L.efc_J;
  real* D = T.w + L.efc_D;
  real* qM = T.w + L.qM;
  FOR_T(e, nv * nv) {
    int r = e / nv, c = e % nv;
    if (c <= r) {
      real h = 0;
      for (unsigned long long mm = amask; mm; mm &= mm - 1) {
        const int i = __builtin_ctzll(mm);
        h += J[i * nv + r] * D[i] * J[i * nv + c];
      }
      H[e] = qM[e] + h;
    }
  }
  TSYNC();
}

// The helper wave of a two-wave rollout team, beside the primary's
// acceleration stage: everything of the Newton start that depends only on the
// warm start -- jar and M*warm, its constraint cost, the full constraint update
// (forces, states, qfrc_constraint) and the Hessian factor of its active set.
// The primary then needs only the smooth start's cost to choose; from the warm
// start (the common case) it goes straight to the first iteration.  Same
// expressions as fwd_constraint_fast, on the other wave.
__device__ inline void newton_warm_prep(const auto& m, const auto& L, const auto& C, const Team& T) {
  const int nv = m.nv, ne = T.iw[L.nefc];
  real* s = T.w + L.s_newton;
  real *Ma = s, *H = s + 4 * nv;
  real* jar = s + 4 * nv + nv * nv;
  real* qM = T.w + L.qM;
  real* warm = T.w + L.warm;
  real* J = T.w + L.efc_J;
  real* aref = T.w + L.efc_aref;
  const int r = T.tid;
  const bool row = r < ne;
  const real Di = row ? T.w[L.efc_D + r] : 0.0;
  const real jw = row ? tdot(J + r * nv, warm, nv) - aref[r] : 0.0;
  if (row) jar[r] = jw;
  FOR_T(i, nv) Ma[i] = tdot(qM + i * nv, warm, nv);
  TSYNC();
  unsigned long long mw;
  const real cu_w = cu_fast(m, L, T, jw, Di, true, mw);
  hessian_build_fast(m, L, T, H, mw);
  cholesky_rows(nv, T.tid, H);
  if (T.tid == 0) {
    T.c[C.bc + 4] = cu_w;
    T.c[C.bc + 5] = __longlong_as_double((long long)mw);
  }
  TSYNC();
}

// ---- Newton solver in wave-uniform registers (compile-time nv <= RMAX) ----
// The primal Newton solver of oracle/mjsub.c (fwd_constraint + solver_newton)
// with every nv-vector (qacc, M qacc, gradient, search direction, M search,
// J' force) and the Hessian's Cholesky factor held IN REGISTERS ON EVERY LANE
// (each lane computes the same values), while constraint row r keeps its
// jacobian row, D and residual on lane r.  The serial recursions (the
// factorization, both substitutions, the cost and gradient sums) then run as
// straight-line VALU code on values already in registers: no LDS round trip,
// no wave barrier and no cross-lane broadcast on their chains.  The row-parallel
// products (M search, J search, the Hessian entries) run one output per lane
// and are gathered once.  Every scalar is the oracle's expression with the
// oracle's summation order, so the results are bit-identical to the lane-
// parallel form (fwd_constraint_fast below) it replaces for these models.

// v[j] = p[j] on every lane (uniform LDS reads)
template <int N>
__device__ __forceinline__ void ldu(real (&v)[N], const real* p) {
  sfor<0, N>(SLAM(jj) { v[SK(jj)] = p[SK(jj)]; });
}
// s = 0 + a[0] b[0] + a[1] b[1] + ... (the oracle's dotn)
template <int N>
__device__ __forceinline__ real dotu(const real (&a)[N], const real (&b)[N]) {
  real r = 0;
  sfor<0, N>(SLAM(jj) { r += a[SK(jj)] * b[SK(jj)]; });
  return r;
}
// a wave-uniform value (a readlane result, held in SGPRs) moved to a VGPR:
// the solver keeps dozens of uniform values live, and left in SGPRs they
// overflow the scalar file (spilled to VGPR lanes, each reload a v_readlane
// on the chain)
__device__ __forceinline__ real vreg(real x) {
  asm("" : "+v"(x));
  return x;
}
// out[j] = value of x on lane j (x: one entry per lane)
template <int N>
__device__ __forceinline__ void gatheru(real (&out)[N], real x) {
  sfor<0, N>(SLAM(jj) { out[SK(jj)] = vreg(bcast(x, SK(jj))); });
}
// out[j] = 0 + p[j](lane i0) + p[j](lane i1) + ... over the set lanes of mask,
// ascending (uniform mask): N ordered sums sharing one walk of the mask
template <int N>
__device__ __forceinline__ void lane_sums_mask(real (&out)[N], const real (&p)[N], unsigned long long mask) {
  sfor<0, N>(SLAM(jj) { out[SK(jj)] = 0; });
  for (unsigned long long mm = mask; mm; mm &= mm - 1) {
    const int i = __builtin_ctzll(mm);
    sfor<0, N>(SLAM(jj) { out[SK(jj)] += bcast(p[SK(jj)], i); });
  }
}
// a / b, uniform operands, divisor reciprocal r = rcp_ref(b) (dsmall.h)
__device__ __forceinline__ real divu(real a, real b, real r) { return div_ref_lane<0>(a, b, r); }

// H = M + J' diag(D * active) J (oracle hessian_factor), entries one per lane
// (lane e = r NV + c, c <= r; J and D read from LDS), gathered, then the
// dense Cholesky in registers; rd[j] = rcp_ref of the factor's diagonal
template <int NV>
__device__ inline void hessian_factor_u(const real* qM, const real* J, const real* D, unsigned long long amask,
                                        int tid, real (&Hf)[NV][NV], real (&rd)[NV]) {
  const int r = tid / NV, c = tid % NV;
  real h = 0;
  if (tid < NV * NV && c <= r) {
    for (unsigned long long mm = amask; mm; mm &= mm - 1) {
      const int i = __builtin_ctzll(mm);
      h += J[i * NV + r] * D[i] * J[i * NV + c];
    }
    h = qM[tid] + h;
  }
  sfor<0, NV>(SLAM(rr) {
    sfor<0, SK(rr) + 1>(SLAM(cc) { Hf[SK(rr)][SK(cc)] = vreg(bcast(h, SK(rr) * NV + SK(cc))); });
  });
  sfor<0, NV>(SLAM(jc) {
    constexpr int j = SK(jc);
    real t = Hf[j][j];
    if constexpr (j > 0) {
      real q = 0;
      sfor<0, j>(SLAM(qq) { q += Hf[j][SK(qq)] * Hf[j][SK(qq)]; });
      t -= q;
    }
    if (t < MINVAL) t = MINVAL;
    Hf[j][j] = sqrt(t);
    const real ti = 1 / Hf[j][j];
    sfor<j + 1, NV>(SLAM(ii) {
      constexpr int i = SK(ii);
      real q = 0;
      sfor<0, j>(SLAM(qq) { q += Hf[i][SK(qq)] * Hf[j][SK(qq)]; });
      Hf[i][j] = (Hf[i][j] - q) * ti;
    });
  });
  sfor<0, NV>(SLAM(jj) { rd[SK(jj)] = rcp_ref(Hf[SK(jj)][SK(jj)]); });
}
// the factor computed elsewhere (newton_warm_prep's LDS H, row-major nv x nv)
template <int NV>
__device__ inline void factor_load_u(const real* H, real (&Hf)[NV][NV], real (&rd)[NV]) {
  sfor<0, NV>(SLAM(rr) {
    sfor<0, SK(rr) + 1>(SLAM(cc) { Hf[SK(rr)][SK(cc)] = H[SK(rr) * NV + SK(cc)]; });
  });
  sfor<0, NV>(SLAM(jj) { rd[SK(jj)] = rcp_ref(Hf[SK(jj)][SK(jj)]); });
}
// a / b with b's refined reciprocal r (dsmall.h div_tail) and the fallback
// deferred: `bad` collects the lanes where the divisor would have been scaled
// (the caller redoes the whole computation with IEEE division then), so no
// branch sits on the dependency chain
__device__ __forceinline__ double div_defer(double a, double b, double r, bool& bad) {
  bool ok;
  const double q = div_tail(a, b, r, ok);
  bad |= !ok;
  return q;
}
__device__ __forceinline__ float div_defer(float a, float b, float, bool&) { return a / b; }
template <bool EXACT>
__device__ __forceinline__ real divx(real a, real b, real r, bool& bad) {
  if constexpr (EXACT) return a / b;
  else return div_defer(a, b, r, bad);
}

// search = -(L L')^-1 g (oracle chol_solve and the sign flip)
template <int NV, bool EXACT>
__device__ inline bool chol_solve_u_impl(const real (&Hf)[NV][NV], const real (&rd)[NV], const real (&g)[NV],
                                         real (&sv)[NV]) {
  bool bad = false;
  real x[NV], acc[NV];
  sfor<0, NV>(SLAM(ii) { acc[SK(ii)] = 0; });
  // forward: x[i] = (g[i] - dotn(L_i, x, i)) / L_ii, the dot products grown as
  // the x[j] are final (ascending j from +0: dotn's order); the scheduling
  // barriers keep each product right behind the x[j] it needs (in-order issue:
  // the compiler otherwise sinks them to the next division's operand)
  sfor<0, NV>(SLAM(ii) {
    constexpr int i = SK(ii);
    real t = g[i];
    if constexpr (i > 0) t -= acc[i];
    x[i] = divx<EXACT>(t, Hf[i][i], rd[i], bad);
    sfor<i + 1, NV>(SLAM(kk) { acc[SK(kk)] += Hf[SK(kk)][i] * x[i]; });
    __builtin_amdgcn_sched_barrier(0);
  });
  // backward: x[i] -= L[j][i] x[j] for j = i+1.. ascending, then / L_ii
  real pr[NV][NV];  // pr[i][j] = L[j][i] x[j], formed as x[j] is final
  sfor<0, NV>(SLAM(ii) {
    constexpr int i = NV - 1 - SK(ii);
    real t = x[i];
    sfor<i + 1, NV>(SLAM(jj) { t -= pr[i][SK(jj)]; });
    x[i] = divx<EXACT>(t, Hf[i][i], rd[i], bad);
    sfor<0, i>(SLAM(kk) { pr[SK(kk)][i] = Hf[i][SK(kk)] * x[i]; });
    __builtin_amdgcn_sched_barrier(0);
  });
  sfor<0, NV>(SLAM(jj) { sv[SK(jj)] = -x[SK(jj)]; });
  return bad;
}
template <int NV>
__device__ inline void chol_solve_u(const real (&Hf)[NV][NV], const real (&rd)[NV], const real (&g)[NV],
                                    real (&sv)[NV]) {
  const bool bad = chol_solve_u_impl<NV, false>(Hf, rd, g, sv);
  if (__builtin_expect(__ballot(bad) != 0, 0)) (void)chol_solve_u_impl<NV, true>(Hf, rd, g, sv);
}
// 0.5 sum_j (Ma_j - qfs_j)(qacc_j - qas_j) (oracle gauss_cost)
template <int N>
__device__ __forceinline__ real gauss_uu(const real (&Ma)[N], const real (&qfs)[N], const real (&qa)[N],
                                         const real (&qas)[N]) {
  real g = 0;
  sfor<0, N>(SLAM(jj) { g += (Ma[SK(jj)] - qfs[SK(jj)]) * (qa[SK(jj)] - qas[SK(jj)]); });
  return 0.5 * g;
}

// the exact line search (oracle linesearch) from lane-row terms: eval(0) in
// the lane form, then ls_iterate; returns alpha (uniform)
__device__ inline real linesearch_rows(int ne, real g1, real g2, real jr, real jv, real Di, bool row, const Team& T) {
  const real c2 = Di * jv * jv;
  const real x0 = jr + 0.0 * jv;  // the oracle's LS_EVAL(0.0)
  const real c10 = Di * x0 * jv;
  const unsigned long long am = __ballot(row && x0 < 0);
  const real d1 = lane_sum_mask(g1 + g2 * 0.0, c10, am);
  if (d1 >= 0) return 0;
  const real d2c = lane_sum_mask(g2, c2, am);
  const real rd2 = rcp_ref(d2c);
  int iters = 0;
#ifdef ILQG_STAMPS
  const unsigned long long tls_ = __builtin_amdgcn_s_memtime();
#endif
  const real alpha = ls_iterate(ne, g1, g2, jr, jv, Di, c2, row, d1, d2c, rd2, am, iters);
#ifdef ILQG_STAMPS
  CNT_ADD(5, __builtin_amdgcn_s_memtime() - tls_);
  CNT_ADD(0, 1ull);
  CNT_ADD(1, (unsigned long long)iters);
  CNT_ADD(2, (unsigned long long)(iters == LS_ITER));
  CNT_ADD(3, (unsigned long long)ne);
  CNT_ADD(4, (unsigned long long)(ne <= LS_NE));
#endif
  (void)T;
  return alpha;
}

// fwd_constraint + solver_newton for a compile-time nv <= RMAX and nefc <= 64
// (dual: the rollout's primary wave, whose helper ran newton_warm_prep).
// Workspace contract: the outputs are qacc, the warm start and the rows'
// jar; unlike fwd_constraint_fast / fwd_constraint, this solver keeps the
// constraint forces and states in registers and does NOT write efc_force,
// efc_state, efc_b or qfrc_constraint back to LDS -- those fields are stale
// after a compile-time-model solve (nothing reads them after the solve today;
// a future consumer such as a contact-force cost or sensor must add the
// write-back).
// ILQG_SPEC_H (three-wave rollout, step_dual_split): the Newton Hessian factor
// of the active set a full step (alpha = 1) would give is built by wave 2,
// idle through phase 5, while the primary runs the line search; when the
// step's active set changed and equals that set, the primary loads the factor
// instead of building it (the factor is a function of qM, J, D and the set
// alone: the same bits).  The oracle over the bench's rollouts: 64-77 % of the
// rebuilds are such sets (tools/ls_study/nt_run.py).  Hand-off words:
// T.ci[C.ibc + 1] the primary's iteration token sid * 128 + k (jr, jv of the
// iteration in the Newton scratch), sid * 128 + 127 at the end of its solve;
// T.ci[C.ibc + 2] the token whose factor wave 2 left at s_newton + 4 nv (the
// warm start's factor slot, free once loaded), its active set in T.c[C.bc + 6].
#ifndef ILQG_SPEC_H
#define ILQG_SPEC_H 1
#endif
constexpr int SPEC_DONE = 127;
#ifndef ILQG_EULER_EARLY
#define ILQG_EULER_EARLY 1
#endif
// ILQG_SPEC_SMOOTH (opt-in): wave 2 also builds the smooth start's factor at
// the phase's start (used when the solve starts from qacc_smooth).  Measured
// slower: the factor can start only when phase 5 does (qacc_smooth is phase 4's
// output), and the primary then waits for it (profiles/r06_ab_spec_smooth.txt)
#ifndef ILQG_SPEC_SMOOTH
#define ILQG_SPEC_SMOOTH 0
#endif
template <int NV>
__device__ inline void fwd_constraint_u(const auto& m, const auto& L, const auto& C, const Team& T, int maxiter,
                                        real tol, bool dual, int spec_sid = 0) {
#ifdef ILQG_STAMPS
  const unsigned long long tnt_ = __builtin_amdgcn_s_memtime();
#endif
  const int ne = T.iw[L.nefc];
  const real scale = 1 / (m.stat_meaninertia * (NV > 1 ? NV : 1));
  real* sn = T.w + L.s_newton;
  real* jar_l = sn + 4 * NV + NV * NV;
  const real* qM = T.w + L.qM;
  const real* J = T.w + L.efc_J;
  const int r = T.tid;
  const bool row = r < ne;
  const real Di = row ? T.w[L.efc_D + r] : 0.0;
  const real aref = row ? T.w[L.efc_aref + r] : 0.0;
  real Jr[NV], Mr[NV];  // lane r: jacobian row r; lane i < NV: row i of M
  sfor<0, NV>(SLAM(jj) {
    constexpr int j = SK(jj);
    Jr[j] = row ? J[r * NV + j] : 0.0;
    Mr[j] = r < NV ? qM[r * NV + j] : 0.0;
  });
  real qas[NV], qfs[NV], warm[NV];
  ldu(qas, T.w + L.qacc_smooth);
  ldu(qfs, T.w + L.qfrc_smooth);
  ldu(warm, T.w + L.warm);
  // warm-start selection (oracle fwd_constraint)
  const real jb = row ? dotu(Jr, qas) - aref : 0.0;
  const bool acts = row && jb < 0;
  const unsigned long long ms = __ballot(acts);
  const real cost_smooth = lane_sum_mask(0.0, acts ? 0.5 * Di * jb * jb : -0.0, ms);
  real jw, cost_warm, Ma[NV];
  unsigned long long mw;
  const bool specH = ILQG_SPEC_H && spec_sid > 0 && maxiter < SPEC_DONE;
  if (dual) {
    // the helper's newton_warm_prep is in LDS (the three-wave schedule ran it
    // in the previous phase: no barrier here then)
    if (!specH) __syncthreads();
    jw = row ? jar_l[r] : 0.0;
    mw = (unsigned long long)__double_as_longlong((double)T.c[C.bc + 5]);
    ldu(Ma, sn);
    cost_warm = gauss_uu(Ma, qfs, warm, qas) + T.c[C.bc + 4];
  } else {
    jw = row ? dotu(Jr, warm) - aref : 0.0;
    gatheru(Ma, dotu(Mr, warm));
    const bool actw = row && jw < 0;
    mw = __ballot(actw);
    cost_warm = gauss_uu(Ma, qfs, warm, qas) + lane_sum_mask(0.0, actw ? 0.5 * Di * jw * jw : -0.0, mw);
  }
  const bool use_smooth = __ballot(cost_warm > cost_smooth) != 0;  // uniform
  // solver start (oracle solver_newton)
  real qacc[NV], qc[NV], grad[NV], Hf[NV][NV], rd[NV];
  real jr, cost;
  unsigned long long mask;
  sfor<0, NV>(SLAM(jj) { qacc[SK(jj)] = use_smooth ? qas[SK(jj)] : warm[SK(jj)]; });
  if (use_smooth) {
    jr = jb;
    gatheru(Ma, dotu(Mr, qas));
    mask = ms;
    cost = gauss_uu(Ma, qfs, qacc, qas) + cost_smooth;
  } else {
    jr = jw;
    mask = mw;
    cost = cost_warm;
  }
  if (!use_smooth && dual) {
    // forces, J' force and the factor of the warm start's active set: the helper's
    ldu(qc, T.w + L.qfrc_con);
    factor_load_u<NV>(sn + 4 * NV, Hf, rd);
  } else {
    real p[NV];
    const real f = (row && jr < 0) ? -Di * jr : 0.0;
    sfor<0, NV>(SLAM(jj) { p[SK(jj)] = Jr[SK(jj)] * f; });
    lane_sums_mask(qc, p, mask);
    bool got = false;
    if (ILQG_SPEC_SMOOTH && specH && use_smooth) {
      // the smooth start's factor: wave 2 built it at the phase's start (token sid * 128)
      wave_wait(T.ci + C.ibc + 2, spec_sid * 128);
      if ((unsigned long long)__double_as_longlong((double)T.c[C.bc + 7]) == mask) {
        factor_load_u<NV>(T.c + C.buf6, Hf, rd);
        got = true;
      }
    }
    if (!got) hessian_factor_u<NV>(qM, J, T.w + L.efc_D, mask, r, Hf, rd);
  }
  sfor<0, NV>(SLAM(jj) { grad[SK(jj)] = (Ma[SK(jj)] - qfs[SK(jj)]) - qc[SK(jj)]; });
  unsigned long long hmask = mask;
  int iter = 0;
  CNT_ADD(9, 1ull);
  STAMP(10);
  int* f_it = T.ci + C.ibc + 1;
  int* f_h = T.ci + C.ibc + 2;
  while (iter < maxiter) {
    real sv[NV], Mv[NV];
    chol_solve_u<NV>(Hf, rd, grad, sv);
    STAMP(14);
    gatheru(Mv, dotu(Mr, sv));
    const real jv = row ? dotu(Jr, sv) : 0.0;
    // the full step's active set, and the iteration's rows for wave 2
    unsigned long long m1 = 0;
    if (specH) {
      m1 = __ballot(row && jr + jv < 0);
      if (row) {
        jar_l[r] = jr;
        jar_l[ne + r] = jv;
      }
      wave_signal(f_it, spec_sid * 128 + iter + 1);
    }
    STAMP(15);
    real alpha = 0;
    if (!(sqrt(dotu(sv, sv)) < MINVAL)) {
      real g1 = 0, g2 = 0;
      sfor<0, NV>(SLAM(jj) { g1 += sv[SK(jj)] * (Ma[SK(jj)] - qfs[SK(jj)]); });
      sfor<0, NV>(SLAM(jj) { g2 += sv[SK(jj)] * Mv[SK(jj)]; });
      if constexpr (LS_U) {
        alpha = ne <= 4 ? linesearch_u<4>(ne, g1, g2, jr, jv, Di, row)
                : ne <= 8 ? linesearch_u<8>(ne, g1, g2, jr, jv, Di, row)
                          : linesearch_rows(ne, g1, g2, jr, jv, Di, row, T);
      } else {
        alpha = linesearch_rows(ne, g1, g2, jr, jv, Di, row, T);
      }
    }
    STAMP(16);
    if (__ballot(alpha == 0) != 0) break;  // uniform
    sfor<0, NV>(SLAM(jj) {
      qacc[SK(jj)] += alpha * sv[SK(jj)];
      Ma[SK(jj)] += alpha * Mv[SK(jj)];
    });
    jr += alpha * jv;
    iter++;
    CNT_ADD(8, 1ull);
    STAMP(17);
    const real oldcost = cost;
    const bool act = row && jr < 0;
    mask = __ballot(act);
    cost = gauss_uu(Ma, qfs, qacc, qas) + lane_sum_mask(0.0, act ? 0.5 * Di * jr * jr : -0.0, mask);
    {
      real p[NV];
      const real f = act ? -Di * jr : 0.0;
      sfor<0, NV>(SLAM(jj) { p[SK(jj)] = Jr[SK(jj)] * f; });
      lane_sums_mask(qc, p, mask);
    }
    sfor<0, NV>(SLAM(jj) { grad[SK(jj)] = (Ma[SK(jj)] - qfs[SK(jj)]) - qc[SK(jj)]; });
    const real improvement = scale * (oldcost - cost);
    const real gradient = scale * sqrt(dotu(grad, grad));
    STAMP(18);
    if (__ballot(improvement < tol || gradient < tol) != 0) break;
    // the factor is a function of (qM, J, D, active set) alone: rebuilt only
    // when the active set changed since it was computed (the same bits)
    if (mask != hmask) {
      bool got = false;
      if (specH && mask == m1) {
        // wave 2 built this set's factor (this iteration's token)
        wave_wait(f_h, spec_sid * 128 + iter);
        if ((unsigned long long)__double_as_longlong((double)T.c[C.bc + 6]) == mask) {
          factor_load_u<NV>(sn + 4 * NV, Hf, rd);
          got = true;
        }
      }
      if (!got) hessian_factor_u<NV>(qM, J, T.w + L.efc_D, mask, r, Hf, rd);
      hmask = mask;
    }
    STAMP(19);
  }
  if (specH) wave_signal(f_it, spec_sid * 128 + SPEC_DONE);
  if (row) jar_l[r] = jr;
  real* qa_l = T.w + L.qacc;
  real* wm_l = T.w + L.warm;
  real qv = qacc[0];
  sfor<1, NV>(SLAM(jj) { qv = r == SK(jj) ? qacc[SK(jj)] : qv; });
  if (r < NV) {
    qa_l[r] = qv;
    wm_l[r] = qv;
  }
  TSYNC();
#ifdef ILQG_STAMPS
  CNT_ADD(6, __builtin_amdgcn_s_memtime() - tnt_);
#endif
}

#ifndef ILQG_WARM_U
#define ILQG_WARM_U 1
#endif
// newton_warm_prep for compile-time nv <= RMAX in fwd_constraint_u's register
// forms (its non-dual branch's warm-start values: J w - aref per row, M w,
// the warm start's constraint cost and J' force, the factor of its Hessian),
// published where fwd_constraint_u's dual branch reads them: jar and M w in
// the Newton scratch, J' force in qfrc_constraint, the factor's lower triangle
// at s_newton + 4 nv, the cost and the active mask in the team scalars
template <int NV>
__device__ inline void newton_warm_prep_u(const auto& m, const auto& L, const auto& C, const Team& T) {
  const int ne = T.iw[L.nefc];
  real* sn = T.w + L.s_newton;
  real* jar_l = sn + 4 * NV + NV * NV;
  const real* qM = T.w + L.qM;
  const real* J = T.w + L.efc_J;
  const int r = T.tid;
  const bool row = r < ne;
  const real Di = row ? T.w[L.efc_D + r] : 0.0;
  const real aref = row ? T.w[L.efc_aref + r] : 0.0;
  real Jr[NV], Mr[NV], warm[NV];
  sfor<0, NV>(SLAM(jj) {
    constexpr int j = SK(jj);
    Jr[j] = row ? J[r * NV + j] : 0.0;
    Mr[j] = r < NV ? qM[r * NV + j] : 0.0;
  });
  ldu(warm, T.w + L.warm);
  const real jw = row ? dotu(Jr, warm) - aref : 0.0;
  const real maw = dotu(Mr, warm);
  const bool actw = row && jw < 0;
  const unsigned long long mw = __ballot(actw);
  const real cu_w = lane_sum_mask(0.0, actw ? 0.5 * Di * jw * jw : -0.0, mw);
  real qc[NV], p[NV];
  const real f = actw ? -Di * jw : 0.0;
  sfor<0, NV>(SLAM(jj) { p[SK(jj)] = Jr[SK(jj)] * f; });
  lane_sums_mask(qc, p, mw);
  real Hf[NV][NV], rd[NV];
  hessian_factor_u<NV>(qM, J, T.w + L.efc_D, mw, r, Hf, rd);
  if (row) jar_l[r] = jw;
  if (r < NV) sn[r] = maw;
  real qv = qc[0];
  sfor<1, NV>(SLAM(jj) { qv = r == SK(jj) ? qc[SK(jj)] : qv; });
  if (r < NV) T.w[L.qfrc_con + r] = qv;
  if (r < NV * NV) {
    const int i = r / NV, j = r % NV;
    real hv = 0;
    sfor<0, NV>(SLAM(ii) {
      sfor<0, SK(ii) + 1>(SLAM(cc) { hv = r == SK(ii) * NV + SK(cc) ? Hf[SK(ii)][SK(cc)] : hv; });
    });
    if (j <= i) sn[4 * NV + r] = hv;
  }
  if (r == 0) {
    T.c[C.bc + 4] = cu_w;
    T.c[C.bc + 5] = __longlong_as_double((long long)mw);
  }
  TSYNC();
}

// wave 2's side of ILQG_SPEC_H (see fwd_constraint_u): for each iteration the
// primary announces, the factor of the active set its rows give at alpha = 1,
// into the warm start's factor slot, announced with that iteration's token;
// ends when the primary's solve does
template <int NV>
__device__ inline void newton_spec_helper(const auto& L, const auto& C, const Team& T, int sid) {
  const int ne = T.iw[L.nefc];
  real* sn = T.w + L.s_newton;
  const real* jar_l = sn + 4 * NV + NV * NV;
  const int r = T.tid;
  const bool row = r < ne;
  const int* f_it = T.ci + C.ibc + 1;
  int* f_h = T.ci + C.ibc + 2;
  // store the factor Hf (lower triangle, row-major nv x nv) at dst, its set in *ms_dst
  auto publish = [&](real* dst, real* ms_dst, const real (&Hf)[NV][NV], unsigned long long set) {
    if (r < NV * NV) {
      const int i = r / NV, j = r % NV;
      real hv = 0;
      sfor<0, NV>(SLAM(ii) {
        sfor<0, SK(ii) + 1>(SLAM(cc) { hv = r == SK(ii) * NV + SK(cc) ? Hf[SK(ii)][SK(cc)] : hv; });
      });
      if (j <= i) dst[r] = hv;
    }
    if (r == 0) *ms_dst = __longlong_as_double((long long)set);
  };
  if (ILQG_SPEC_SMOOTH) {
    // the smooth start's factor (fwd_constraint_u: jb = J qacc_smooth - aref,
    // the active set of jb < 0), in case the solve starts there; qacc_smooth is
    // the primary's phase-4 output, the rows wave 1's
    real Jr[NV], qas[NV];
    sfor<0, NV>(SLAM(jj) { Jr[SK(jj)] = row ? T.w[L.efc_J + r * NV + SK(jj)] : 0.0; });
    ldu(qas, T.w + L.qacc_smooth);
    const real aref = row ? T.w[L.efc_aref + r] : 0.0;
    const real jb = row ? dotu(Jr, qas) - aref : 0.0;
    const unsigned long long ms = __ballot(row && jb < 0);
    real Hf[NV][NV], rd[NV];
    hessian_factor_u<NV>(T.w + L.qM, T.w + L.efc_J, T.w + L.efc_D, ms, r, Hf, rd);
    (void)rd;
    publish(T.c + C.buf6, T.c + C.bc + 7, Hf, ms);
    wave_signal(f_h, sid * 128);
  }
  int seen = sid * 128;
  for (int guard = 0; guard < (1 << 22); guard++) {
    const int tok = __builtin_amdgcn_readfirstlane(
        __hip_atomic_load(f_it, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
    if (tok >= sid * 128 + SPEC_DONE) break;
    if (tok <= seen) {
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    seen = tok;
    const real jr = row ? jar_l[r] : 0.0, jv = row ? jar_l[ne + r] : 0.0;
    const unsigned long long m1 = __ballot(row && jr + jv < 0);
    real Hf[NV][NV], rd[NV];
    hessian_factor_u<NV>(T.w + L.qM, T.w + L.efc_J, T.w + L.efc_D, m1, r, Hf, rd);
    (void)rd;
    publish(sn + 4 * NV, T.c + C.bc + 6, Hf, m1);
    wave_signal(f_h, tok);
  }
}

// dual: the primary wave of a two-wave team whose helper runs newton_warm_prep
// concurrently; exactly one __syncthreads (after the smooth start's cost)
__device__ inline void fwd_constraint_fast(const auto& m, const auto& L, const auto& C, const auto& X,
                                           const Team& T, int maxiter, real tol, bool dual = false,
                                           int spec_sid = 0) {
  using MT = std::remove_cvref_t<decltype(m)>;
  if constexpr (StaticModel<MT>) {
    if constexpr (MT::nv <= RMAX) {
      fwd_constraint_u<MT::nv>(m, L, C, T, maxiter, tol, dual, spec_sid);
      return;
    }
  }
#ifdef ILQG_STAMPS
  const unsigned long long tnt_ = __builtin_amdgcn_s_memtime();
#endif
  const int nv = m.nv, ne = T.iw[L.nefc];
  const real scale = 1 / (m.stat_meaninertia * (nv > 1 ? nv : 1));
  real* s = T.w + L.s_newton;
  real *Ma = s, *grad = s + nv, *search = s + 2 * nv, *Mv = s + 3 * nv, *H = s + 4 * nv;
  real* jar = s + 4 * nv + nv * nv;
  real* Jv = jar + ne;
  real* qM = T.w + L.qM;
  real* qacc = T.w + L.qacc;
  real* warm = T.w + L.warm;
  real* J = T.w + L.efc_J;
  real* aref = T.w + L.efc_aref;
  real* b = T.w + L.efc_b;
  real* qfs = T.w + L.qfrc_smooth;
  real* qas = T.w + L.qacc_smooth;
  real* qc = T.w + L.qfrc_con;
  const int r = T.tid;
  const bool row = r < ne;
  const real Di = row ? T.w[L.efc_D + r] : 0.0;
  unsigned long long mask, hmask;
  // warm-start selection (oracle fwd_constraint): smooth vs warmstart cost
  real jb = 0, jw = 0, cost_warm, cost_smooth;
  unsigned long long mask_w = 0;
  if (dual) {
    if (row) {
      jb = tdot(J + r * nv, qas, nv) - aref[r];
      b[r] = jb;
    }
    cost_smooth = cu_fast(m, L, T, jb, Di, false, mask);
    __syncthreads();  // the helper's warm-start part (newton_warm_prep) is in LDS
    if (row) jw = jar[r];
    mask_w = (unsigned long long)__double_as_longlong(T.c[C.bc + 5]);
    cost_warm = gauss_u(nv, Ma, qfs, warm, qas) + T.c[C.bc + 4];
  } else {
    if (row) {
      jb = tdot(J + r * nv, qas, nv) - aref[r];
      jw = tdot(J + r * nv, warm, nv) - aref[r];
      b[r] = jb;
    }
    FOR_T(i, nv) Ma[i] = tdot(qM + i * nv, warm, nv);
    TSYNC();
    cost_smooth = cu_fast(m, L, T, jb, Di, false, mask);
    cost_warm = gauss_u(nv, Ma, qfs, warm, qas) + cu_fast(m, L, T, jw, Di, false, mask);
  }
  const bool use_smooth = cost_warm > cost_smooth;
  // solver start (oracle solver_newton): Ma, jar at qacc, full constraint update
  real jr = use_smooth ? jb : jw;
  FOR_T(i, nv) qacc[i] = use_smooth ? qas[i] : warm[i];
  TSYNC();
  if (use_smooth) {
    FOR_T(i, nv) Ma[i] = tdot(qM + i * nv, qacc, nv);
    TSYNC();
  }
  // from the warm start the full update's cost is cost_warm's expression on the
  // same values: only its side effects (force, state, qfrc_constraint) are new
  real cost;
  if (use_smooth) {
    cost = gauss_u(nv, Ma, qfs, qacc, qas) + cu_fast(m, L, T, jr, Di, true, mask);
  } else if (dual) {
    mask = mask_w;  // forces, states, qfrc_constraint and the factor: the helper's
    cost = cost_warm;
  } else {
    (void)cu_fast(m, L, T, jr, Di, true, mask, false);
    cost = cost_warm;
  }
  FOR_T(j, nv) grad[j] = (Ma[j] - qfs[j]) - qc[j];
  if (use_smooth || !dual) {
    hessian_build_fast(m, L, T, H, mask);
    cholesky_rows(nv, T.tid, H);
  } else {
    TSYNC();
  }
  hmask = mask;
  int iter = 0;
#ifdef ILQG_STAMPS
  CNT_ADD(9, 1ull);
#endif
  while (iter < maxiter) {
    chol_solve_rows(nv, T.tid, H, grad, search);
    STAMP(14);
    FOR_T(i, nv) Mv[i] = tdot(qM + i * nv, search, nv);
    const real jv = row ? tdot(J + r * nv, search, nv) : 0.0;
    TSYNC();
    STAMP(15);
    // exact line search (oracle linesearch), uniform on every lane
    real alpha = 0;
    {
      real snorm = sqrt(tdot(search, search, nv));
      if (!(snorm < MINVAL)) {
        real g1 = 0, g2 = 0, d1, d2;
        for (int j = 0; j < nv; j++) g1 += search[j] * (Ma[j] - qfs[j]);
        for (int j = 0; j < nv; j++) g2 += search[j] * Mv[j];
        // active rows only (the others add -0.0); d2 depends on the active set
        // alone, so it is summed again only when the set changes
        unsigned long long pmask = 0;
        bool have = false;
        real d2c = 0, rd2 = 0;
        const real c2 = Di * jv * jv;
        auto eval = [&](real a) {
          const real x = jr + a * jv;
          const bool on = row && x < 0;
          const real c1 = Di * x * jv;
          const unsigned long long am = __ballot(on);
          d1 = lane_sum_mask(g1 + g2 * a, c1, am);
          if (!have || am != pmask) {
            d2c = lane_sum_mask(g2, c2, am);
            rd2 = rcp_ref(d2c);  // d1 / d2 below: the divisor's part, once per active set
            pmask = am;
            have = true;
          }
          d2 = d2c;
        };
        eval(0.0);
        if (!(d1 >= 0)) {
          int iters = 0;
#ifdef ILQG_STAMPS
          const unsigned long long tls_ = __builtin_amdgcn_s_memtime();
#endif
          alpha = ls_iterate(ne, g1, g2, jr, jv, Di, c2, row, d1, d2c, rd2, pmask, iters);
#ifdef ILQG_STAMPS
          CNT_ADD(5, __builtin_amdgcn_s_memtime() - tls_);
          CNT_ADD(0, 1ull);
          CNT_ADD(1, (unsigned long long)iters);
          CNT_ADD(2, (unsigned long long)(iters == LS_ITER));
          CNT_ADD(3, (unsigned long long)ne);
          CNT_ADD(4, (unsigned long long)(ne <= LS_NE));
#endif
        }
      }
    }
    STAMP(16);
    if (alpha == 0) break;
    FOR_T(j, nv) {
      qacc[j] += alpha * search[j];
      Ma[j] += alpha * Mv[j];
    }
    jr += alpha * jv;
    TSYNC();
    iter++;
#ifdef ILQG_STAMPS
    CNT_ADD(8, 1ull);
#endif
    STAMP(17);
    const real oldcost = cost;
    cost = gauss_u(nv, Ma, qfs, qacc, qas) + cu_fast(m, L, T, jr, Di, true, mask);
    FOR_T(j, nv) grad[j] = (Ma[j] - qfs[j]) - qc[j];
    TSYNC();
    const real improvement = scale * (oldcost - cost);
    const real gradient = scale * sqrt(tdot(grad, grad, nv));
    STAMP(18);
    if (improvement < tol || gradient < tol) break;
    if (mask != hmask) {
      hessian_build_fast(m, L, T, H, mask);
      cholesky_rows(nv, T.tid, H);
      hmask = mask;
    }
    STAMP(19);
  }
  if (row) jar[r] = jr;
  FOR_T(i, nv) warm[i] = qacc[i];
  TSYNC();
#ifdef ILQG_STAMPS
  CNT_ADD(6, __builtin_amdgcn_s_memtime() - tnt_);
#endif
}

__device__ inline void fwd_constraint(const auto& m, const auto& L, const auto& C, const auto& X, const Team& T,
                                      int maxiter, real tol) {
  const int nv = m.nv, ne = T.iw[L.nefc];
  real* qacc = T.w + L.qacc;
  real* warm = T.w + L.warm;
  real* qas = T.w + L.qacc_smooth;
  real* qc = T.w + L.qfrc_con;
  if (!ne) {
    FOR_T(i, nv) { real v = qas[i]; qacc[i] = v; warm[i] = v; qc[i] = 0; }
    TSYNC();
    return;
  }
  if (ne <= TEAM_SIZE && nv <= RMAX) {
    fwd_constraint_fast(m, L, C, X, T, maxiter, tol);
    return;
  }
  {
    real* s = T.w + L.s_newton;
    real* Ma = s;
    real* jar = s + 4 * nv + nv * nv;
    real* J = T.w + L.efc_J;
    real* aref = T.w + L.efc_aref;
    real* b = T.w + L.efc_b;
    real* qM = T.w + L.qM;
    real* qfs = T.w + L.qfrc_smooth;
    FOR_T(i, ne) {
      b[i] = tdotw(J + i * nv, qas, nv) - aref[i];
      jar[i] = tdotw(J + i * nv, warm, nv) - aref[i];
    }
    FOR_T(i, nv) Ma[i] = tdotw(qM + i * nv, warm, nv);
    TSYNC();
    real cost_smooth = constraint_update(m, L, C, T, b);
    real cw = constraint_update(m, L, C, T, jar);
    if (T.tid == 0) {
      real g = 0;
      for (int j = 0; j < nv; j++) g += (Ma[j] - qfs[j]) * (warm[j] - qas[j]);
      real cost_warm = 0.5 * g + cw;
      T.ci[C.ibc] = cost_warm > cost_smooth ? 1 : 0;
    }
    TSYNC();
    const int use_smooth = T.ci[C.ibc];
    FOR_T(i, nv) qacc[i] = use_smooth ? qas[i] : warm[i];
    TSYNC();
  }
  solver_newton(m, L, C, T, maxiter, tol);
  FOR_T(i, nv) warm[i] = qacc[i];
  TSYNC();
}

__device__ inline void forward_skip(const auto& m, const auto& L, const auto& C, const auto& X,
                                    const Team& T, int skipstage, int maxiter, real tol) {
  STAMP(-1);
  TSYNC();
  STAMP(20);
  TSYNC();
  STAMP(21);
  if (skipstage < STAGE_POS) fwd_position(m, L, C, X, T);
  if (skipstage < STAGE_VEL) fwd_velocity(m, L, C, T);
  STAMP(6);
  fwd_acceleration(m, L, X, T);
  STAMP(7);
  fwd_constraint(m, L, C, X, T, maxiter, tol);
  STAMP(8);
}

// forward_skip split at the warm start: the position and velocity stages never
// read qacc_warmstart, the acceleration stage's constraint solve does
__device__ inline void forward_posvel(const auto& m, const auto& L, const auto& C, const auto& X, const Team& T,
                                      int skipstage) {
  STAMP(-1);
  TSYNC();
  if (skipstage < STAGE_POS) fwd_position(m, L, C, X, T);
  if (skipstage < STAGE_VEL) fwd_velocity(m, L, C, T);
  STAMP(6);
}
__device__ inline void forward_acc(const auto& m, const auto& L, const auto& C, const auto& X, const Team& T,
                                   int maxiter, real tol) {
  STAMP(-1);
  fwd_acceleration(m, L, X, T);
  STAMP(7);
  fwd_constraint(m, L, C, X, T, maxiter, tol);
  STAMP(8);
}

__device__ inline void integrate_pos(const auto& m, const Team& T, real* qpos, const real* qvel, real dt) {
  FOR_T(j, m.njnt) {
    int pa = m.jnt_qposadr[j], va = m.jnt_dofadr[j];
    int type = m.jnt_type[j];
    if (type == JNT_FREE || type == JNT_BALL) {
      if (type == JNT_FREE) {
        for (int i = 0; i < 3; i++) qpos[pa + i] += dt * qvel[va + i];
        pa += 3;
        va += 3;
      }
      real q[4], v[3];
      ldm<4>(q, qpos + pa);
      ldm<3>(v, qvel + va);
      quat_integrate(q, v, dt);
      for (int k = 0; k < 4; k++) qpos[pa + k] = q[k];
    } else {
      qpos[pa] += dt * qvel[va];
    }
  }
  TSYNC();
}

__device__ inline void reset_data(const auto& m, const auto& L, const Team& T) {
  real* qpos = T.w + L.qpos;
  FOR_T(i, m.nq) qpos[i] = m.qpos0[i];
  FOR_T(i, m.nv) {
    T.w[L.qvel + i] = 0;
    T.w[L.warm + i] = 0;
    T.w[L.qfrc_applied + i] = 0;
  }
  FOR_T(i, m.nu) T.w[L.ctrl + i] = 0;
  FOR_T(i, 6 * m.nbody) T.w[L.xfrc_applied + i] = 0;
  if (T.tid == 0) T.w[L.time] = 0;
  TSYNC();
}

// mj_checkPos/Vel/Acc test: any NaN/huge entry (a wave ballot, no serial scan)
__device__ inline int any_bad(const Team& T, const auto& C, const real* x, int n) {
  unsigned long long bad = 0;
  for (int i0 = 0; i0 < n; i0 += TEAM_SIZE) {
    const int i = i0 + T.tid;
    bad |= __ballot(i < n && is_bad(x[i]));
  }
  return bad != 0ull;
}

// Euler with implicit joint damping (MuJoCo mj_Euler): qacc_e = (M + h D)^-1 M qacc.
// Split so a helper wave can factor M + h D (a function of qM only) while the
// primary wave is still in the velocity stage; the factor is the same numbers.
__device__ inline bool euler_damped(const auto& m, const Team& T) {
  const int nv = m.nv;
  unsigned long long dmask = 0;
  for (int i0 = 0; i0 < nv; i0 += TEAM_SIZE) dmask |= __ballot(i0 + T.tid < nv && m.dof_damping[i0 + T.tid] > 0);
  return dmask != 0ull;
}
__device__ inline void euler_prefactor(const auto& m, const auto& L, const auto& C, const auto& X, const Team& T) {
  const int nv = m.nv;
  real* s = T.w + L.s_euler;
  real *qH = s + nv, *qHLD = s + nv + nv * nv, *qHinv = s + nv + 2 * nv * nv;
  real* qM = T.w + L.qM;
  if (!euler_damped(m, T)) return;
  FOR_T(e, nv * nv) {
    int i = e / nv, j = e % nv;
    real v = qM[e];
    if (i == j) v += m.opt_timestep * m.dof_damping[i];
    qH[e] = v;
  }
  TSYNC();
  factor_ld(m, X, T, qH, qHLD, qHinv, T.c + C.ftmp);
}
__device__ inline void euler_finish(const auto& m, const auto& L, const auto& C, const auto& X, const Team& T,
                                    bool factored) {
  const int nv = m.nv;
  real* s = T.w + L.s_euler;
  real *qacc = s, *qHLD = s + nv + nv * nv, *qHinv = s + nv + 2 * nv * nv;
  real* qM = T.w + L.qM;
  real* dq = T.w + L.qacc;
  real* qvel = T.w + L.qvel;
  if (!euler_damped(m, T)) {
    FOR_T(i, nv) qacc[i] = dq[i];
    TSYNC();
  } else {
    FOR_T(i, nv) qacc[i] = tdot(qM + i * nv, dq, nv);
    TSYNC();
    if (!factored) euler_prefactor(m, L, C, X, T);
    solve_ld(m, X, T, qHLD, qHinv, qacc);
  }
  const real h = m.opt_timestep;
  FOR_T(i, nv) qvel[i] += qacc[i] * h;
  TSYNC();
  integrate_pos(m, T, T.w + L.qpos, qvel, h);
  if (T.tid == 0) T.w[L.time] += h;
  TSYNC();
}
__device__ inline void euler(const auto& m, const auto& L, const auto& C, const auto& X, const Team& T) {
  euler_finish(m, L, C, X, T, false);
}

// compile-time models with slide/hinge joints only (nq == nv <= RMAX) whose
// ancestor masks are constants
#ifndef ILQG_EULER_U
#define ILQG_EULER_U 1
#endif
template <class MT>
constexpr bool euler_regs_ok() {
  if constexpr (StaticModel<MT> && ILQG_EULER_U) {
    if constexpr (MT::nv <= RMAX && MT::nq == MT::nv) {
      for (int j = 0; j < MT::njnt; j++)
        if (MT::jnt_type[j] != JNT_SLIDE && MT::jnt_type[j] != JNT_HINGE) return false;
      return true;
    }
  }
  return false;
}
// euler_finish for those models when M + h D is damped and already factored
// (the rollout's helper wave): the whole chain qacc -> M qacc -> (L'DL)^-1 ->
// qvel -> qpos on wave-uniform registers, one LDS read phase and one write.
// M qacc is one row per lane (tdot's order), gathered; the tree solve is
// solve_ld_rows' sequence with compile-time ancestor sets (a skipped update
// where x[i] == 0 becomes a select of the unchanged value); qvel += qacc h and
// qpos += h qvel per joint as integrate_pos.  Returns false (nothing done)
// when the general path must run.
template <class MT>
__device__ inline bool euler_finish_u(const auto& m, const auto& L, const auto& X, const Team& T) {
  constexpr int NV = MT::nv;
  using XT = std::remove_cvref_t<decltype(X)>;
  (void)X;
  if (!euler_damped(m, T)) return false;
  const real* s = T.w + L.s_euler;
  const real *qHLD = s + NV + NV * NV, *qHinv = s + NV + 2 * NV * NV;
  const real* qM = T.w + L.qM;
  real qa[NV], x[NV], qv[NV], qp[NV], dinv[NV], LDr[NV][NV];
  ldu(qa, T.w + L.qacc);
  ldu(qv, T.w + L.qvel);
  ldu(qp, T.w + L.qpos);
  ldu(dinv, qHinv);
  sfor<0, NV>(SLAM(ii) {
    constexpr int i = SK(ii);
    sfor<0, i>(SLAM(jj) {
      constexpr int j = SK(jj);
      if constexpr ((XT::pmask[i] >> j) & 1) LDr[i][j] = qHLD[i * NV + j];
    });
  });
  const int r = T.tid < NV ? T.tid : 0;
  real Mr[NV];
  sfor<0, NV>(SLAM(jj) { Mr[SK(jj)] = qM[r * NV + SK(jj)]; });
  gatheru(x, dotu(Mr, qa));
  // x[j] -= LD[i][j] x[i] for j in anc(i), i descending, where x[i] != 0
  sfor<0, NV>(SLAM(ii) {
    constexpr int i = NV - 1 - SK(ii);
    const bool nz = x[i] != 0;
    sfor<0, i>(SLAM(jj) {
      constexpr int j = SK(jj);
      if constexpr ((XT::pmask[i] >> j) & 1) {
        const real u = x[j] - LDr[i][j] * x[i];
        x[j] = nz ? u : x[j];
      }
    });
  });
  sfor<0, NV>(SLAM(ii) { x[SK(ii)] *= dinv[SK(ii)]; });
  // x[i] -= LD[i][j] x[j] for j in anc(i) descending, i ascending
  sfor<0, NV>(SLAM(ii) {
    constexpr int i = SK(ii);
    sfor<0, i>(SLAM(jj) {
      constexpr int j = i - 1 - SK(jj);
      if constexpr ((XT::pmask[i] >> j) & 1) x[i] -= LDr[i][j] * x[j];
    });
  });
  const real h = m.opt_timestep;
  sfor<0, NV>(SLAM(ii) { qv[SK(ii)] += x[SK(ii)] * h; });
  sfor<0, MT::njnt>(SLAM(jj) {
    constexpr int j = SK(jj);
    constexpr int pa = MT::jnt_qposadr[j], va = MT::jnt_dofadr[j];
    qp[pa] += h * qv[va];
  });
  real* sw = T.w + L.s_euler;
  real* qvel = T.w + L.qvel;
  real* qpos = T.w + L.qpos;
  real xv = x[0], vv = qv[0], pv = qp[0];
  sfor<1, NV>(SLAM(ii) {
    xv = T.tid == SK(ii) ? x[SK(ii)] : xv;
    vv = T.tid == SK(ii) ? qv[SK(ii)] : vv;
    pv = T.tid == SK(ii) ? qp[SK(ii)] : pv;
  });
  if (T.tid < NV) {
    sw[T.tid] = xv;
    qvel[T.tid] = vv;
    qpos[T.tid] = pv;
  }
  if (T.tid == 0) T.w[L.time] += h;
  TSYNC();
  return true;
}

__device__ inline void rk4(const auto& m, const auto& L, const auto& C, const auto& X, const Team& T,
                           int maxiter, real tol) {
  const real A[9] = {0.5, 0, 0, 0, 0.5, 0, 0, 0, 1};
  const real Bw[4] = {1.0 / 6, 1.0 / 3, 1.0 / 3, 1.0 / 6};
  const int nv = m.nv, nq = m.nq, N = 4;
  const real h = m.opt_timestep;
  real* qpos = T.w + L.qpos;
  real* qvel = T.w + L.qvel;
  real* qaccw = T.w + L.qacc;
  const real time = T.w[L.time];
  real Cc[3], Tt[3];
  real* s = T.w + L.s_rk4;
  real *dX = s, *X0 = s + 2 * nv, *F = s + 2 * nv + 4 * (nq + nv);
  for (int i = 1; i < N; i++) {
    Cc[i - 1] = 0;
    for (int j = 0; j < i; j++) Cc[i - 1] += A[(i - 1) * (N - 1) + j];
    Tt[i - 1] = time + Cc[i - 1] * h;
  }
  FOR_T(k, nq) X0[k] = qpos[k];
  FOR_T(k, nv) { X0[nq + k] = qvel[k]; F[k] = qaccw[k]; }
  TSYNC();
  for (int i = 1; i < N; i++) {
    real* Xi = X0 + i * (nq + nv);
    FOR_T(k, nv) {
      real a0 = 0, a1 = 0;
      for (int j = 0; j < i; j++) {
        real a = A[(i - 1) * (N - 1) + j];
        a0 += X0[j * (nq + nv) + nq + k] * a;
        a1 += F[j * nv + k] * a;
      }
      dX[k] = a0;
      dX[nv + k] = a1;
    }
    FOR_T(k, nq + nv) Xi[k] = X0[k];
    TSYNC();
    integrate_pos(m, T, Xi, dX, h);
    FOR_T(k, nv) Xi[nq + k] += dX[nv + k] * h;
    TSYNC();
    FOR_T(k, nq) qpos[k] = Xi[k];
    FOR_T(k, nv) qvel[k] = Xi[nq + k];
    if (T.tid == 0) T.w[L.time] = Tt[i - 1];
    TSYNC();
    forward_skip(m, L, C, X, T, STAGE_NONE, maxiter, tol);
    FOR_T(k, nv) F[i * nv + k] = qaccw[k];
    TSYNC();
  }
  FOR_T(k, nv) {
    real a0 = 0, a1 = 0;
    for (int j = 0; j < N; j++) {
      a0 += X0[j * (nq + nv) + nq + k] * Bw[j];
      a1 += F[j * nv + k] * Bw[j];
    }
    dX[k] = a0;
    dX[nv + k] = a1;
  }
  TSYNC();
  FOR_T(k, nq) qpos[k] = X0[k];
  FOR_T(k, nv) qvel[k] = X0[nq + k] + dX[nv + k] * h;
  if (T.tid == 0) T.w[L.time] = time;
  TSYNC();
  integrate_pos(m, T, qpos, dX, h);
  if (T.tid == 0) T.w[L.time] += h;
  TSYNC();
}

// mj_step with the model's own solver settings
__device__ inline void step(const auto& m, const auto& L, const auto& C, const auto& X,
                            const Team& T) {
  if (any_bad(T, C, T.w + L.qpos, m.nq)) reset_data(m, L, T);
  if (any_bad(T, C, T.w + L.qvel, m.nv)) reset_data(m, L, T);
  forward_skip(m, L, C, X, T, STAGE_NONE, m.opt_iterations, m.opt_tolerance);
  if (any_bad(T, C, T.w + L.qacc, m.nv)) {
    reset_data(m, L, T);
    forward_skip(m, L, C, X, T, STAGE_NONE, m.opt_iterations, m.opt_tolerance);
  }
  STAMP(-1);
  if (m.opt_integrator == 1)
    rk4(m, L, C, X, T, m.opt_iterations, m.opt_tolerance);
  else
    euler(m, L, C, X, T);
  STAMP(9);
}

// the L'DL factor of M and, for Euler with damping, the factor of M + h D
// (euler_prefactor's matrix) in one pass of the register-row factorization:
// lanes 0..31 factor M, lanes 32..63 factor M + h D.  Same numbers as
// factor_ld() followed by euler_prefactor().
__device__ inline void factor_m_and_euler(const auto& m, const auto& L, const auto& C, const auto& X,
                                          const Team& T, bool eul) {
  const int nv = m.nv;
  real* qM = T.w + L.qM;
  if (!(eul && euler_damped(m, T))) {
    factor_ld(m, X, T, qM, T.w + L.qLD, T.w + L.qLDinv, T.c + C.ftmp);
    return;
  }
  if (!(nv <= RMAX && has_pmask(X))) {
    factor_ld(m, X, T, qM, T.w + L.qLD, T.w + L.qLDinv, T.c + C.ftmp);
    euler_prefactor(m, L, C, X, T);
    return;
  }
  real* s = T.w + L.s_euler;
  real *qH = s + nv, *qHLD = s + nv + nv * nv, *qHinv = s + nv + 2 * nv * nv;
  using MT = std::remove_cvref_t<decltype(m)>;
  if constexpr (fld_lanes_ok<MT>()) {
    // lane 0 factors M, lane 1 M + h D (its diagonal formed in registers as
    // euler_prefactor forms it; the matrix itself is read by nothing else)
    constexpr int NV = MT::nv;
    real add[NV];
    sfor<0, NV>(SLAM(ii) { add[SK(ii)] = m.opt_timestep * m.dof_damping[SK(ii)]; });
#ifdef ILQG_ASM_MARK
    asm volatile(";;MARK_F2_BEGIN" ::: "memory");
#endif
    factor_ld_lanes<std::remove_cvref_t<decltype(X)>, NV>(T.tid, qM, add, true, T.w + L.qLD, T.w + L.qLDinv,
                                                          (int)(qHLD - (T.w + L.qLD)), (int)(qHinv - (T.w + L.qLDinv)));
#ifdef ILQG_ASM_MARK
    asm volatile(";;MARK_F2_END" ::: "memory");
#endif
    return;
  }
  FOR_T(e, nv * nv) {
    int i = e / nv, j = e % nv;
    real v = qM[e];
    if (i == j) v += m.opt_timestep * m.dof_damping[i];
    qH[e] = v;
  }
  TSYNC();
#ifdef ILQG_ASM_MARK
  asm volatile(";;MARK_F2_BEGIN" ::: "memory");
#endif
  factor_ld_rows2(nv, X.pmask, T.tid, qM, T.w + L.qLD, T.w + L.qLDinv, qH, qHLD, qHinv);
#ifdef ILQG_ASM_MARK
  asm volatile(";;MARK_F2_END" ::: "memory");
#endif
}

// The primary's phase 4 under ILQG_SPLIT3 in one pass of registers: lane 0
// factors M and, with that factor still in its registers, solves qacc_smooth =
// M^-1 qfrc_smooth; lane 1 factors M + h D (Euler with damping).  The same
// operations as factor_m_and_euler (factor_ld_lanes' loop) followed by
// fwd_acceleration_u (the tree solve of solve_ld_rows' sequence), without the
// factor's round trip through LDS between them.  Returns false, having done
// nothing, when a body carries xfrc_applied (the general path runs).
#ifndef ILQG_FACC
#define ILQG_FACC 1
#endif
template <class MT>
__device__ inline bool factor_acc_u(const auto& m, const auto& L, const auto& X, const Team& T, bool eul) {
  constexpr int NV = MT::nv, NB = MT::nbody;
  using XT = std::remove_cvref_t<decltype(X)>;
  (void)X;
  const real* xf = T.w + L.xfrc_applied;
  static_assert(6 * NB <= TEAM_SIZE, "one ballot over xfrc_applied");
  if (__ballot(T.tid >= 6 && T.tid < 6 * NB && xf[T.tid] != 0) != 0ull) return false;
  const bool two = eul && euler_damped(m, T);
  const bool l1 = two && T.tid == 1;
  const real *qp = T.w + L.qfrc_passive, *qb = T.w + L.qfrc_bias, *qap = T.w + L.qfrc_applied;
  const real* qa = T.w + L.qfrc_act;
  const real* qM = T.w + L.qM;
  real v[NV], a[NV][NV];
  sfor<0, NV>(SLAM(jj) {
    constexpr int j = SK(jj);
    real t = qp[j] - qb[j];
    t += qap[j];
    t += qa[j];
    v[j] = t;
  });
  sfor<0, NV>(SLAM(ii) {
    constexpr int i = SK(ii);
    sfor<0, i + 1>(SLAM(jj) { a[i][SK(jj)] = qM[i * NV + SK(jj)]; });
    const real s_ = a[i][i] + m.opt_timestep * m.dof_damping[i];
    a[i][i] = l1 ? s_ : a[i][i];
  });
  // the factor (factor_ld_lanes' loop)
  sfor<0, NV>(SLAM(kk) {
    constexpr int k = NV - 1 - SK(kk);
    real dk = a[k][k];
    if (dk < MINVAL) dk = MINVAL;
    a[k][k] = dk;
    sfor<0, k>(SLAM(ii) {
      constexpr int i = k - 1 - SK(ii);
      if constexpr ((XT::pmask[k] >> i) & 1) {
        const real tmp = a[k][i] / dk;
        sfor<0, i + 1>(SLAM(jj) {
          constexpr int j = i - SK(jj);
          if constexpr (j == i || ((XT::pmask[i] >> j) & 1)) a[i][j] -= tmp * a[k][j];
        });
        a[k][i] = tmp;
      }
    });
  });
  real dinv[NV];
  sfor<0, NV>(SLAM(ii) { dinv[SK(ii)] = 1 / a[SK(ii)][SK(ii)]; });
  // qacc_smooth = (L'DL)^-1 qfrc_smooth (fwd_acceleration_u's sequence), lane 0's factor
  real x[NV];
  sfor<0, NV>(SLAM(jj) { x[SK(jj)] = v[SK(jj)]; });
  sfor<0, NV>(SLAM(ii) {
    constexpr int i = NV - 1 - SK(ii);
    const bool nz = x[i] != 0;
    sfor<0, i>(SLAM(jj) {
      constexpr int j = SK(jj);
      if constexpr ((XT::pmask[i] >> j) & 1) {
        const real u = x[j] - a[i][j] * x[i];
        x[j] = nz ? u : x[j];
      }
    });
  });
  sfor<0, NV>(SLAM(ii) { x[SK(ii)] *= dinv[SK(ii)]; });
  sfor<0, NV>(SLAM(ii) {
    constexpr int i = SK(ii);
    sfor<0, i>(SLAM(jj) {
      constexpr int j = i - 1 - SK(jj);
      if constexpr ((XT::pmask[i] >> j) & 1) x[i] -= a[i][j] * x[j];
    });
  });
  // lane 0: the factor of M and both accelerations; lane 1: the factor of M + h D
  if (T.tid == 0 || l1) {
    real* s_ = T.w + L.s_euler;
    real* LD = l1 ? s_ + NV + NV * NV : T.w + L.qLD;
    real* Dinv = l1 ? s_ + NV + 2 * NV * NV : T.w + L.qLDinv;
    sfor<0, NV>(SLAM(ii) {
      constexpr int i = SK(ii);
      sfor<0, NV>(SLAM(jj) {
        constexpr int j = SK(jj);
        if constexpr (j <= i) LD[i * NV + j] = a[i][j];
        else LD[i * NV + j] = (real)0;
      });
      Dinv[i] = dinv[i];
    });
  }
  if (T.tid == 0) {
    sfor<0, NV>(SLAM(ii) {
      T.w[L.qfrc_smooth + SK(ii)] = v[SK(ii)];
      T.w[L.qacc_smooth + SK(ii)] = x[SK(ii)];
    });
  }
  TSYNC();
  return true;
}

// factor_m_and_euler split for the three-wave step: the factor of M, announced
// on `fm` (step id sid) as soon as it is formed (phase 4; the primary's
// acceleration stage waits for it), and the factor of M + h D, which only
// the integrator reads (phase 5, beside the primary's Newton solve).
// factor_ld_rows twice is factor_ld_rows2's operations.  Returns whether the
// second factor is still to be formed (euler_factor_rows).
__device__ inline bool factor_m_signal(const auto& m, const auto& L, const auto& C, const auto& X, const Team& T,
                                       bool eul, int* fm, int sid) {
  const int nv = m.nv;
  if (!(nv <= RMAX && has_pmask(X))) {
    factor_m_and_euler(m, L, C, X, T, eul);
    wave_signal(fm, sid);
    return false;
  }
  factor_ld_rows(nv, X.pmask, T.tid, T.w + L.qM, T.w + L.qLD, T.w + L.qLDinv);
  wave_signal(fm, sid);
  return eul && euler_damped(m, T);
}
__device__ inline void euler_factor_rows(const auto& m, const auto& L, const auto& X, const Team& T) {
  const int nv = m.nv;
  const real* qM = T.w + L.qM;
  real* s = T.w + L.s_euler;
  real *qH = s + nv, *qHLD = s + nv + nv * nv, *qHinv = s + nv + 2 * nv * nv;
  FOR_T(e, nv * nv) {
    int i = e / nv, j = e % nv;
    real v = qM[e];
    if (i == j) v += m.opt_timestep * m.dof_damping[i];
    qH[e] = v;
  }
  TSYNC();
  factor_ld_rows(nv, X.pmask, T.tid, qH, qHLD, qHinv);
}

// the acceleration stage in phase 4 (beside the helpers), the factor of M
// handed over by wave 2 and the factor of M + h D moved to phase 5: bit-exact
// but measured slower (two factorizations in series on wave 2 cost more than
// factor_ld_rows2's one pass), so off
#ifndef ILQG_ACC_P4
#define ILQG_ACC_P4 0
#endif
#ifndef ILQG_COLL_SPLIT
#define ILQG_COLL_SPLIT 1
#endif
#ifndef ILQG_SPLIT3
#define ILQG_SPLIT3 1
#endif
// pairs (compile-time aux) with a plane geom: bit p
template <class MT, class XT>
constexpr unsigned long long plane_pair_mask() {
  unsigned long long mk = 0;
  for (int p = 0; p < XT::npair && p < 64; p++)
    if (MT::geom_type[XT::pair[2 * p]] == GEOM_PLANE || MT::geom_type[XT::pair[2 * p + 1]] == GEOM_PLANE)
      mk |= 1ull << p;
  return mk;
}
template <class MT, class XT>
constexpr bool coll_split_ok() {
  if constexpr (StaticModel<MT> && ILQG_COLL_SPLIT) {
    if constexpr (XT::npair > 0 && XT::npair <= 64) {
      constexpr unsigned long long pm = plane_pair_mask<MT, XT>();
      constexpr unsigned long long all = XT::npair == 64 ? ~0ull : (1ull << XT::npair) - 1;
      return pm != 0 && pm != all;
    }
  }
  return false;
}

// step_dual for the split layout (L.split: RNE / com-velocity / Euler scratch
// outside the union) and register-row models, on a THREE-wave team (wave 0
// the dependency chain, waves 1 and 2 helpers).  Work moves to where a helper
// has slack, without changing any value:
//   phase 1 (beside the kinematics), wave 1: control law + record, the limit
//     rows of make_constraint (qpos only), passive forces, transmission and
//     actuator forces (ctrl only);
//   phase 2 (beside com_pos), wave 1: collision;
//   phase 3 (beside crb), wave 1: contact jacobians and row allocation;
//   phase 4 (beside com velocities + RNE), wave 1: the contact rows'
//     jacobians and parameters, constraint reference accelerations and the
//     warm-start half of the Newton start; wave 2: the factors of M and of
//     M + h D in one register-row pass;
//   phase 5: the primary's acceleration stage and constraint solve find the
//     Newton warm start ready.
// the rollout teams' phase barriers order LDS only: inside a step the waves
// hand each other nothing through global memory (the trajectory record's
// stores and the next record's loads are the only global traffic), so those
// stay in flight across the barriers instead of being drained at each one
// (__syncthreads waits for vmcnt(0)); ILQG_PHASE_LDS=0 restores it (A/B)
#ifndef ILQG_PHASE_LDS
#define ILQG_PHASE_LDS 1
#endif
__device__ __forceinline__ void phase_sync() {
#if ILQG_PHASE_LDS
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
#else
  __syncthreads();
#endif
}

__device__ inline void step_dual_split(const auto& m, const auto& L, const auto& C, const auto& X, const Team& T,
                                       int wave, int sid, auto&& pre, auto&& late) {
  const bool A = wave == 0, B = wave == 1;
  int* fq = T.ci + C.ibc + 6;  // quaternions final (primary -> frames helper)
  int* ff = T.ci + C.ibc + 7;  // frame rotations final (helper -> primary)
  const bool eul = m.opt_integrator != 1;
  STAMP(-1);
  STAMPB(-1);
  STAMPC(-1);
  const bool bad = any_bad(T, C, T.w + L.qpos, m.nq) || any_bad(T, C, T.w + L.qvel, m.nv);
  if (bad) {
    if (B) {
      pre();
      late();
    }
    phase_sync();
    if (A) reset_data(m, L, T);
    phase_sync();  // the helpers' phase-1 work reads the reset state
  }
  int* nlim_sh = T.ci + C.ibc + 5;  // the limit rows' count, from wave 2 to wave 1
  constexpr bool ksplit = kin_split_ok<std::remove_cvref_t<decltype(m)>>();
  if (A) {
    if constexpr (ksplit) kinematics_primary(m, L, C, T, fq, ff, sid);
    else kinematics(m, L, C, T);
    STAMP(0);
  } else if (!B) {
    // wave 2: the qpos/qvel-only rows and forces, then the frame rotations
    const int nl = limit_rows_pre(m, L, C, T);
    if (T.tid == 0) *nlim_sh = nl;
    passive_forces(m, L, T);
    if constexpr (ksplit) kinematics_frames(m, L, T, fq, ff, sid);
    STAMPC(48);
  } else {
    if (!bad) pre();
    STAMPB(41);
    transmission(m, L, T);
    TSYNC();
    actuator_force(m, L, T);
    STAMPB(42);
  }
  phase_sync();
  const int nlim = *nlim_sh;
  STAMP(24);
  STAMPB(32);
  STAMPC(49);
  if (A) {
    using MT = std::remove_cvref_t<decltype(m)>;
    if constexpr (StaticModel<MT> && ILQG_COM_U) com_pos_u<MT>(m, L, T);
    else com_pos(m, L, T);
    STAMP(1);
  } else {
    using MT = std::remove_cvref_t<decltype(m)>;
    using XT = std::remove_cvref_t<decltype(X)>;
    if constexpr (coll_split_ok<MT, XT>()) {
      // the narrow phase split by pair kind over the two helpers (no divergent
      // mix of kernels on one wave): wave 1 the pairs with a plane, wave 2 the
      // rest; wave 2 hands its counts and candidates to wave 1, which compacts
      int* fc = T.ci + C.ibc + 4;
      constexpr unsigned long long pm = plane_pair_mask<MT, XT>();
      const bool mine = T.tid < XT::npair && (((pm >> T.tid) & 1ull) != 0) == B;
      if (mine) collision_pair(m, L, C, X, T, T.tid);
      if (!B) {
        wave_signal(fc, sid);
        STAMPC(50);
      } else {
        wave_wait(fc, sid);
        collision_finish(m, L, C, X, T);
        STAMPB(33);
      }
    } else if (B) {
      collision(m, L, C, X, T);
      STAMPB(33);
    }
  }
  phase_sync();
  STAMP(25);
  STAMPB(34);
  STAMPC(51);
  bool rows_done = false;
  // ILQG_SPLIT3 (the register-row models): the velocity stage, which reads only
  // com_pos's outputs (cdof, cinert) and the state, runs on wave 2 beside crb;
  // wave 1 forms the constraint rows and their reference accelerations here
  // too.  Phase 4 is then the primary's factors of M and M + h D and its
  // acceleration stage beside wave 1's Newton warm start.
  using MT3 = std::remove_cvref_t<decltype(m)>;
  constexpr bool split3 = ILQG_SPLIT3 && !ILQG_ACC_P4 && StaticModel<MT3> && ILQG_VEL_H && vel_regs_ok<MT3>() &&
                          euler_regs_ok<MT3>();
  if (A) {
    using MT = std::remove_cvref_t<decltype(m)>;
    if constexpr (StaticModel<MT> && ILQG_COM_U) crb_u<MT>(m, L, C, X, T);
    else crb(m, L, C, X, T);
    STAMP(2);
  } else if (B) {
    mc_contact_jac(m, L, X, T);
    TSYNC();
    const bool par = mc_alloc(m, L, C, T);
    TSYNC();
    if (!par || nlim < 0) {
      // the serial allocation (njmax truncation): every row here, as make_constraint
      mc_rows(m, L, C, T, 0, T.iw[L.nefc]);
      TSYNC();
      rows_done = true;
    }
    if constexpr (split3) {
      if (!rows_done) {
        mc_rows(m, L, C, T, nlim, T.iw[L.nefc]);
        TSYNC();
        rows_done = true;
      }
      STAMPB(35);
      constraint_ref(m, L, T);
      TSYNC();
      STAMPB(37);
    } else {
      STAMPB(35);
    }
  } else {
    if constexpr (split3) {
      fwd_velocity_h<MT3>(m, L, T);
      STAMPC(57);
    }
  }
  phase_sync();
  STAMP(26);
  STAMPB(36);
  STAMPC(52);
  const int ne5 = T.iw[L.nefc];
  const bool spec = ne5 > 0 && ne5 <= TEAM_SIZE && m.nv <= RMAX;
  // ILQG_SPEC_H: wave 2 builds the primary's Newton factors ahead (fwd_constraint_u)
  using MT5 = std::remove_cvref_t<decltype(m)>;
  constexpr bool spec_h_ok = [] {
    if constexpr (StaticModel<MT5>) return ILQG_SPEC_H && split3 && MT5::nv <= RMAX && MT5::opt_iterations < SPEC_DONE;
    else return false;
  }();
  const bool spec_h = spec_h_ok && spec;
  // the acceleration stage beside the helpers' phase-4 work (the factor of M
  // handed over by wave 2 as soon as it is formed), or in phase 5
  using MT4 = std::remove_cvref_t<decltype(m)>;
  constexpr bool acc4 = ILQG_ACC_P4 && vel_regs_ok<MT4>() && euler_regs_ok<MT4>();
  int* fm = T.ci + C.ibc + 3;  // the factor of M final (wave 2 -> primary)
  bool acc_done = false;
  bool euler_late = false;  // wave 2: the factor of M + h D left for phase 5
  if (A) {
    using MT = std::remove_cvref_t<decltype(m)>;
    if constexpr (split3) {
      if constexpr (ILQG_FACC) acc_done = factor_acc_u<MT>(m, L, X, T, eul);
      if (!acc_done) {
        factor_m_and_euler(m, L, C, X, T, eul);
        STAMP(3);
        acc_done = fwd_acceleration_u<MT>(m, L, X, T);
      }
      STAMP(7);
    } else {
      if constexpr (vel_regs_ok<MT>() && ILQG_VEL_H) fwd_velocity_h<MT>(m, L, T);
      else if constexpr (vel_regs_ok<MT>()) fwd_velocity_u<MT>(m, L, T);
      else fwd_velocity(m, L, C, T, 1);
      STAMP(6);
      if constexpr (acc4) {
        wave_wait(fm, sid);
        acc_done = fwd_acceleration_u<MT>(m, L, X, T);
        STAMP(7);
      }
    }
  } else if (B) {
    if constexpr (!split3) {
      if (!rows_done) {
        mc_rows(m, L, C, T, nlim, T.iw[L.nefc]);
        TSYNC();
      }
      constraint_ref(m, L, T);
      TSYNC();
      STAMPB(37);
    }
    if (spec) {
      using MT = std::remove_cvref_t<decltype(m)>;
      bool done_u = false;
      if constexpr (StaticModel<MT>) {
        if constexpr (ILQG_WARM_U && MT::nv <= RMAX) {
          newton_warm_prep_u<MT::nv>(m, L, C, T);
          done_u = true;
        }
      }
      if (!done_u) newton_warm_prep(m, L, C, T);
    }
    STAMPB(30);
  } else {
    if constexpr (acc4) euler_late = factor_m_signal(m, L, C, X, T, eul, fm, sid);
    else if constexpr (!split3) factor_m_and_euler(m, L, C, X, T, eul);
    STAMPC(53);
  }
  phase_sync();
  STAMP(27);
  STAMPB(39);
  STAMPC(54);
  if (A) {
    using MT = std::remove_cvref_t<decltype(m)>;
    if constexpr (!acc4 && !split3 && vel_regs_ok<MT>() && euler_regs_ok<MT>())
      acc_done = fwd_acceleration_u<MT>(m, L, X, T);
    if (!acc_done) fwd_acceleration(m, L, X, T, true);
    if constexpr (!split3) STAMP(7);
    if (spec) {
      fwd_constraint_fast(m, L, C, X, T, m.opt_iterations, m.opt_tolerance, true, spec_h ? sid : 0);
    } else {
      phase_sync();
      fwd_constraint(m, L, C, X, T, m.opt_iterations, m.opt_tolerance);
    }
    STAMP(8);
  } else {
    // the primary's barrier inside its Newton start (none in the ILQG_SPEC_H
    // schedule: wave 1's warm start is from phase 4)
    if (!spec_h) phase_sync();
    // `late` (the caller's work after `pre` that no phase reads: parking the
    // prefetched record) runs here, where wave 1 has slack, so its loads have
    // landed long before
    if (B && !bad) late();
    // wave 2: the factor of M + h D, read by the integrator in phase 6
    if (!B && euler_late) euler_factor_rows(m, L, X, T);
    // wave 2: the Newton factors of the full steps' active sets (ILQG_SPEC_H)
    if constexpr (spec_h_ok) {
      if (!B && spec_h) newton_spec_helper<MT5::nv>(L, C, T, sid);
    }
    STAMPB(38);
  }
  phase_sync();
  STAMP(29);
  STAMPB(43);
  STAMPC(55);
  if (A) {
    bool reset = false;
    if (any_bad(T, C, T.w + L.qacc, m.nv)) {
      reset = true;
      reset_data(m, L, T);
      forward_skip(m, L, C, X, T, STAGE_NONE, m.opt_iterations, m.opt_tolerance);
    }
    if (!eul) {
      rk4(m, L, C, X, T, m.opt_iterations, m.opt_tolerance);
    } else {
      bool done = false;
      using MT = std::remove_cvref_t<decltype(m)>;
      if constexpr (euler_regs_ok<MT>())
        if (!reset) done = euler_finish_u<MT>(m, L, X, T);
      if (!done) euler_finish(m, L, C, X, T, !reset);
    }
    STAMP(9);
  }
  phase_sync();
  STAMP(28);
  STAMPB(40);
  STAMPC(56);
}

// mj_step by a two-wave team (rollout kernels): wave 0 runs the dependency
// chain, wave 1 takes the branches off it -- collision beside com_pos,
// make_constraint beside crb + factor_ld(M), passive forces + constraint
// reference + the Euler factor of M + h D beside com velocities + RNE.  Every
// quantity is still computed by the same code, so results are unchanged;
// both waves pass the same __syncthreads sequence.
__device__ inline void step_dual(const auto& m, const auto& L, const auto& C, const auto& X, const Team& T,
                                 int wave, auto&& pre, auto&& late) {
  const bool A = wave == 0;
  const bool eul = m.opt_integrator != 1;
  STAMP(-1);
  STAMPB(-1);
  // `pre` (the caller's per-step work that reads the state before the step:
  // control law, trajectory record) runs on the helper wave beside the
  // kinematics.  mj_checkPos/Vel resets the state, so on a bad state it runs
  // first, as in the one-wave order; both waves test the same LDS state.
  const bool bad = any_bad(T, C, T.w + L.qpos, m.nq) || any_bad(T, C, T.w + L.qvel, m.nv);
  if (bad) {
    if (!A) pre();
    phase_sync();
    if (A) reset_data(m, L, T);
  }
  if (A) {
    kinematics(m, L, C, T);
    STAMP(0);
  } else if (!bad) {
    pre();
    STAMPB(41);
  }
  phase_sync();
  STAMP(24);
  STAMPB(32);
  if (A) {
    com_pos(m, L, T);
    STAMP(1);
  } else {
    collision(m, L, C, X, T);
    STAMPB(33);
  }
  phase_sync();
  STAMP(25);
  STAMPB(34);
  if (A) {
    transmission(m, L, T);
    crb(m, L, C, X, T);
    STAMP(2);
  } else {
    make_constraint(m, L, C, X, T);
    STAMPB(35);
  }
  phase_sync();
  STAMP(26);
  STAMPB(36);
  // the L'DL factor of M runs on the helper beside the com velocities and RNE
  // (nothing on the primary reads it before the acceleration stage)
  if (A) {
    fwd_velocity(m, L, C, T, 1);
    STAMP(6);
  } else {
    fwd_velocity(m, L, C, T, 2);
    STAMPB(37);
    factor_ld(m, X, T, T.w + L.qM, T.w + L.qLD, T.w + L.qLDinv, T.c + C.ftmp);
    STAMPB(42);
  }
  phase_sync();
  STAMP(27);
  STAMPB(39);
  // the Euler factor of M + h D on the helper beside the constraint solve
  // ... and the warm-start half of the Newton start before it (one extra
  // barrier inside the phase, on both waves)
  const int ne5 = T.iw[L.nefc];
  const bool spec = ne5 > 0 && ne5 <= TEAM_SIZE && m.nv <= RMAX;
  // ILQG_EULER_EARLY: without the warm-start hand-off (the generic solver:
  // nv > 8 or > 64 rows, the humanoid) nothing needs the barrier inside this
  // phase, and the helper starts the Euler factor of M + h D (112k cycles a
  // humanoid step) beside the primary's acceleration stage instead of after it
  const bool mid_sync = spec || !ILQG_EULER_EARLY;
  if (A) {
    fwd_acceleration(m, L, X, T);
    STAMP(7);
    if (spec) {
      fwd_constraint_fast(m, L, C, X, T, m.opt_iterations, m.opt_tolerance, true);
    } else {
      if (mid_sync) phase_sync();
      fwd_constraint(m, L, C, X, T, m.opt_iterations, m.opt_tolerance);
    }
    STAMP(8);
  } else {
    if (spec) {
      using MT = std::remove_cvref_t<decltype(m)>;
      bool done_u = false;
      if constexpr (StaticModel<MT>) {
        if constexpr (ILQG_WARM_U && MT::nv <= RMAX) {
          newton_warm_prep_u<MT::nv>(m, L, C, T);
          done_u = true;
        }
      }
      if (!done_u) newton_warm_prep(m, L, C, T);
    }
    STAMPB(30);
    if (mid_sync) phase_sync();
    if (eul) euler_prefactor(m, L, C, X, T);
    // `late` (the caller's work no phase reads: the next point's record into
    // its second buffer) where the helper waits for the constraint solve
    late();
    STAMPB(38);
  }
  phase_sync();
  STAMP(29);
  STAMPB(43);
  if (A) {
    // (after the barrier: a reset recomputes the forward pass on this wave
    // alone, and its factorisations share scratch with the helper's)
    bool reset = false;
    if (any_bad(T, C, T.w + L.qacc, m.nv)) {
      reset = true;
      reset_data(m, L, T);
      forward_skip(m, L, C, X, T, STAGE_NONE, m.opt_iterations, m.opt_tolerance);
    }
    if (!eul) rk4(m, L, C, X, T, m.opt_iterations, m.opt_tolerance);
    else euler_finish(m, L, C, X, T, !reset);
    STAMP(9);
  }
  phase_sync();
  STAMP(28);
  STAMPB(40);
}

