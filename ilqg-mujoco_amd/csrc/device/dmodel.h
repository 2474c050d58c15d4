// Device-side model and per-evaluation workspace layout.
//
// The compiled model lives in ONE device allocation; DevModel carries the
// sizes by value (kernel argument -> SGPRs) and pointers into that allocation
// (wave-uniform, so model reads become scalar loads).
//
// Each physics evaluation ("lane") owns a slice of a workspace laid out
// structure-of-arrays ACROSS lanes: element e of lane l lives at
// ws[e * stride + l], so a wave's 64 lanes touching the same field hit 64
// consecutive doubles (512 B, fully coalesced).
#pragma once

#include <cstddef>

#include "ilqg_model_fields.h"

namespace ilqg {

struct DevModel {
#define ILQG_DM_I(nm) int nm;
#define ILQG_DM_F(nm) double nm;
#define ILQG_DM_FA(nm, cnt) const double* nm;
#define ILQG_DM_IA(nm, cnt) const int* nm;
  ILQG_MODEL_I32_SCALARS(ILQG_DM_I)
  ILQG_MODEL_F64_SCALARS(ILQG_DM_F)
  ILQG_MODEL_F64_ARRAYS(ILQG_DM_FA)
  ILQG_MODEL_I32_ARRAYS(ILQG_DM_IA)
#undef ILQG_DM_I
#undef ILQG_DM_F
#undef ILQG_DM_FA
#undef ILQG_DM_IA
  int maxcon, maxefc;
  const unsigned char* img;  // base of the compact model image (device memory)
  int img_bytes;             // image size, a multiple of 8
  int static_id;             // compiled model-specific kernels (static_models.h), 0 = generic
};

// contact record inside the workspace (doubles, then ints)
enum {
  CON_DIST = 0, CON_POS = 1, CON_FRAME = 4, CON_INCLM = 13, CON_FRIC = 14,
  CON_SOLREF = 19, CON_SOLIMP = 21, CON_ND = 26
};
enum { CONI_DIM = 0, CONI_G1 = 1, CONI_G2 = 2, CONI_EFCADR = 3, CON_NI = 4 };

struct WsLayout {
  int qpos, qvel, ctrl, qacc, warm, qfrc_applied, xfrc_applied, time;
  int xpos, xquat, xmat, xipos, ximat, xanchor, xaxis, gxpos, gxmat, scom, cdof, cinert, crb;
  int qM, qLD, qLDinv, amom;
  int con;
  int efc_J, efc_pos, efc_margin, efc_D, efc_KBIP, efc_aref, efc_vel, efc_force, efc_b;
  int cvel, cdof_dot, qfrc_passive, qfrc_bias, afrc, qfrc_act, qfrc_smooth, qacc_smooth, qfrc_con;
  int s_rne, s_con, s_newton, s_euler, s_rk4, s_fd;
  int pcon, jc;  // cooperative layout only: per-pair contacts, contact-frame jacobians
  int kstr;      // stride of efc_KBIP rows (4 lane layout, 3 cooperative)
  int split;     // two-wave rollout layout: RNE / com-velocity scratch outside the union
  int nd;
  int coni, efc_type, efc_id, efc_state, ncon, nefc;
  int ni;
};

// npair < 0: the lane-per-evaluation layout (dphys.h).  npair >= 0: the
// cooperative layout (dcoop.h), where scratch that is dead after
// make_constraint (contacts, per-pair candidates, contact-frame jacobians)
// shares storage with scratch first written afterwards (RNE, com velocities,
// Newton, Euler, efc_b/efc_vel): less LDS per team, more teams per CU.
// split (rollout kernels): the RNE and com-velocity scratch live outside the
// union, so the helper wave may still read contacts and contact-frame
// jacobians while the primary runs the velocity stage (step_dual)
template <class M>
constexpr WsLayout make_layout(const M& m, int npair = -1, bool split = false) {
  WsLayout L{};
  int o = 0;
  const int nq = m.nq, nv = m.nv, nu = m.nu, nb = m.nbody, nj = m.njnt, ng = m.ngeom;
  const int nc = m.maxcon > 0 ? m.maxcon : 1, ne = m.maxefc > 0 ? m.maxefc : 1;
  const bool coop = npair >= 0;
  auto take = [&](int n) { int r = o; o += n; return r; };
  L.qpos = take(nq); L.qvel = take(nv); L.ctrl = take(nu); L.qacc = take(nv); L.warm = take(nv);
  L.qfrc_applied = take(nv); L.xfrc_applied = take(6 * nb); L.time = take(1);
  L.xpos = take(3 * nb); L.xquat = take(4 * nb); L.xmat = take(9 * nb); L.xipos = take(3 * nb);
  L.ximat = take(9 * nb); L.xanchor = take(3 * nj); L.xaxis = take(3 * nj); L.gxpos = take(3 * ng);
  L.gxmat = take(9 * ng); L.scom = take(3 * nb); L.cdof = take(6 * nv); L.cinert = take(10 * nb);
  L.crb = take(10 * nb); L.qM = take(nv * nv); L.qLD = take(nv * nv); L.qLDinv = take(nv);
  L.amom = take(nu * nv);
  L.kstr = coop ? 3 : 4;
  if (!coop) L.con = take(CON_ND * nc);
  L.efc_J = take(ne * nv); L.efc_pos = take(ne); L.efc_margin = take(ne); L.efc_D = take(ne);
  L.efc_KBIP = take(L.kstr * ne);
  if (!coop) {
    L.efc_aref = take(ne);
    L.efc_vel = take(ne);
    L.efc_force = take(ne);
    L.efc_b = take(ne);
  }
  L.cvel = take(6 * nb); L.cdof_dot = take(6 * nv); L.qfrc_passive = take(nv); L.qfrc_bias = take(nv);
  L.afrc = take(nu); L.qfrc_act = take(nv); L.qfrc_smooth = take(nv); L.qacc_smooth = take(nv);
  L.qfrc_con = take(nv);
  if (!coop) {
    L.s_rne = take(12 * nb);
    L.s_con = take(10 * nv);
    L.s_newton = take(4 * nv + nv * nv + 2 * ne);
    L.s_euler = take(2 * nv + 2 * nv * nv);
  }
  L.s_rk4 = take(2 * nv + 4 * (nq + nv) + 4 * nv);
  L.s_fd = take(2 * nv);
  if (coop && split) {
    L.split = 1;
    L.s_rne = take(12 * nb);
    L.s_con = take(10 * nv);
    L.s_euler = take(2 * nv + 2 * nv * nv);  // factored beside the contact rows' reads
  }
  if (coop) {
    const int u = o;
    int a = u;  // position-stage view
    L.con = a; a += CON_ND * nc;
    // per-pair candidates (dead once collision has compacted them into con)
    // and contact-frame jacobians (first written by make_constraint) share storage
    L.pcon = a;
    L.jc = a;
    a += 14 * (npair > 0 ? npair : 1) > 3 * nv * nc ? 14 * (npair > 0 ? npair : 1) : 3 * nv * nc;
    int b = u;  // velocity / constraint / integration view
    if (!split) {
      L.s_rne = b; b += 12 * nb;
      L.s_con = b; b += 10 * nv;
    }
    L.s_newton = b; b += 4 * nv + nv * nv + 2 * ne;
    if (!split) {
      L.s_euler = b; b += 2 * nv + 2 * nv * nv;
    }
    L.efc_b = b; b += ne;
    L.efc_vel = b; b += ne;
    // reference accelerations (velocity stage) and forces (constraint solve):
    // first written after make_constraint, like the rest of this view
    L.efc_aref = b; b += ne;
    L.efc_force = b; b += ne;
    o = a > b ? a : b;
  }
  L.nd = o;
  int oi = 0;
  L.coni = oi; oi += CON_NI * nc;
  L.efc_type = oi; oi += ne;
  L.efc_id = oi; oi += ne;
  L.efc_state = oi; oi += ne;
  L.ncon = oi; oi += 1;
  L.nefc = oi; oi += 1;
  L.ni = oi;
  return L;
}

namespace coop {
// extra per-team scratch (doubles / ints), appended after the WsLayout block
struct CoopLayout {
  int qloc, buf6, ftmp, pcon, jc, cterm, rtmp, bc;  // doubles
  int cdesc, rec;  // cost descriptor copy; prefetched rollout record (x*, u*, K, k)
  int nd;
  int pcnt, rsub, jcnt, ibc;  // ints
  int ni;
  int imgd;  // doubles of LDS holding the staged model image
};

template <class M>
constexpr CoopLayout make_coop_layout(const M& m, int npair) {
  CoopLayout C{};
  int o = 0, oi = 0;
  const int nc = m.maxcon > 0 ? m.maxcon : 1, ne = m.maxefc > 0 ? m.maxefc : 1;
  C.qloc = o; o += 4 * m.njnt;
  C.buf6 = o; o += 6 * m.nv;
  C.ftmp = o; o += m.nv;
  C.pcon = 0;  // in the cooperative WsLayout (union scratch)
  C.jc = 0;
  C.cterm = o; o += ne;
  C.rtmp = o; o += 6 * m.nbody;
  C.bc = o; o += 8;
  C.cdesc = o; o += 3 * (m.nq + m.nv + m.nu);
  C.rec = o; o += m.nq + m.nv + 2 * m.nu + 2 * m.nv * m.nu;
  C.nd = o;
  C.pcnt = oi; oi += (npair > 0 ? npair : 1);
  C.rsub = oi; oi += ne;
  C.jcnt = oi; oi += 2 * m.njnt;
  C.ibc = oi; oi += 8;
  C.ni = oi;
  C.imgd = (m.img_bytes + 7) / 8;
  return C;
}

// static data the host derives once per model
struct CoopAux {
  const int* isanc;  // nv*nv: isanc[i*nv+j] = 1 if dof j is dof i or an ancestor of it
  const int* pair;   // 2*npair: geom pairs passing the static collision filters, oracle order
  int npair;
  const unsigned long long* pmask;  // nv: proper-ancestor bitmask of each dof (null if nv > 64)
  // pmask != null, as a flag: a null test of pmask after stage_model points it
  // into LDS makes this ROCm's backend emit an illegal is-shared compare
  // (V_CMP_NE_U32_e32 0, src_shared_base) in the -DILQG_STAMPS build
  int haspm;
};
// has_pmask(X): the generic aux's flag, or the static models' compile-time table
template <class XT>
__host__ __device__ __forceinline__ bool has_pmask(const XT& X) {
  if constexpr (requires { X.haspm; }) return X.haspm != 0;
  else return static_cast<bool>(X.pmask);
}

}  // namespace coop
}  // namespace ilqg
