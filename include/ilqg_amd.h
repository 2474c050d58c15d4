/*
 * ilqg_amd -- MI355X-native iLQR hot path (FD derivative sweep, Riccati
 * backward pass, forward rollout) behind a plain C ABI.
 *
 * Every entry point takes plain pointers and sizes and returns an int status
 * (ILQG_OK == 0).  Host buffers are row-major float64.  Each entry point names
 * the reference interface it replaces (paths under /root/reference).
 *
 * Trajectory record (the per-point state contract of cpMjData, src/util.cpp:4-14),
 * per seed s and point p = 0..N (p = N is the initial state, p = 0 the terminal
 * one, inc/ilqr.h:52):
 *   time[s][p], qpos[s][p][nq], qvel[s][p][nv], warm[s][p][nv] (qacc_warmstart),
 *   ctrl[s][p][nu]
 * qfrc_applied / xfrc_applied are per-seed constants (the reference never
 * changes them along a trajectory).
 *
 * FD record per point (src/mjderivative.cpp:88,107,120,138,174,202), D =
 * nv*(2nv+nu) + 2nv + nu doubles, written exactly as the reference writes it:
 *   [i + j*nv]            d qacc_j / d qpos_i
 *   [nv^2 + i + j*nv]     d qacc_j / d qvel_i
 *   [2nv^2 + i + j*nu]    d qacc_j / d ctrl_i
 *   [2nv^2+nv*nu + i]     d cost / d qpos_i   (then qvel, then ctrl)
 * Gains: K[s][p] is nu x 2nv column-major (Eigen layout, inc/ilqr.h:130),
 * k[s][p] is nu.
 */
#ifndef ILQG_AMD_H
#define ILQG_AMD_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ILQG_OK 0
#define ILQG_ERR_ARG 1
#define ILQG_ERR_MODEL 2
#define ILQG_ERR_HIP 3
#define ILQG_ERR_UNSUPPORTED 4
#define ILQG_ERR_NODEVICE 5

typedef struct ilqg_model ilqg_model;
typedef struct ilqg_solver ilqg_solver;

/* Diagonal-quadratic + linear step cost over (qpos, qvel, ctrl), evaluated on
   the device inside the sweep and the rollout.  Replaces the host callback
   stepCostFn_t (inc/mjderivative.h:5) on the batched path:
     c = sum_i wq_i (qpos_i - tq_i)^2 + lq_i qpos_i  + (same for qvel, ctrl)
   accumulated in (q, v, u) order, index ascending.  inc/inverted_pendulum/
   cost.h:7-17 is wq = {1,10}, wv = {1,10}, wu = {1}.  NULL arrays mean 0. */
typedef struct ilqg_cost {
  const double *wq, *tq, *lq;
  const double *wv, *tv, *lv;
  const double *wu, *tu, *lu;
} ilqg_cost;

typedef struct ilqg_solver_opts {
  int horizon;          /* N; N+1 trajectory points (inc/ilqr.h:14 template N) */
  int nseed;            /* independent trajectories (MPC seeds) on this device */
  int nalpha;           /* rollout candidates per seed; alphas[0] == 1 is the reference rollout */
  const double* alphas; /* feed-forward scales: u = K(x - x*) + alpha*k + u* */
  int select_mode;      /* 0: keep alphas[0] (reference semantics); 1: lowest trajectory cost */
  double mu;            /* Levenberg-Marquardt constant, 1000 in inc/ilqr.h:65 */
  int device;           /* HIP device ordinal */
} ilqg_solver_opts;

const char* ilqg_last_error(void);
int ilqg_version(void);
int ilqg_device_count(int* count);

/* ---- model: replaces mj_loadXML / mj_deleteModel (cmd/basic.cpp:123) ----
   Model-size limit: every device path runs one physics evaluation per
   workgroup with its workspace (mjData equivalent) in LDS, so the workspace
   must fit one CU's 160 KB (the bundled humanoid, nv = 27 with 12 contact
   slots, uses 147 KB).  A larger model is refused at load with
   ILQG_ERR_UNSUPPORTED; the reference's CPU path has no such limit. */
int ilqg_model_load_xml(const char* path, ilqg_model** out);
int ilqg_model_load_xml_string(const char* xml, ilqg_model** out);
void ilqg_model_free(ilqg_model* m);
/* sizes[10] = nq nv nu nbody njnt ngeom maxcon maxefc nconmax njmax */
int ilqg_model_sizes(const ilqg_model* m, int* sizes);
int ilqg_model_timestep(const ilqg_model* m, double* dt);
int ilqg_model_qpos0(const ilqg_model* m, double* qpos0);
/* compiled-model record (include/ilqg_model_blob.h); needed = bytes required */
int ilqg_model_blob(const ilqg_model* m, void* buf, size_t cap, size_t* needed);
/* specialisation key: the integer data (sizes, topology, static collision
   pairs, device-image layout) that model-specific kernels compile in
   (tools/gen_static_models.py); n = entries written (or required if key is
   NULL).  static_id: the compiled specialisation this model runs on, 0 = the
   generic kernels.  Results are identical either way. */
int ilqg_model_static_key(const ilqg_model* m, int* key, int cap, int* n);
int ilqg_model_static_id(const ilqg_model* m, int* id);

/* ---- batched single-point physics (device) ----
   n independent states; host buffers (n x nq etc.).  step: mj_step
   (inc/ilqr.h:86,128, src/update.cpp:8-11) -- advances time/qpos/qvel/warm in
   place; forward: mj_forward -> qacc (n x nv), warm updated in place. */
int ilqg_step_batch(const ilqg_model* m, int n, int nstep, double* time, double* qpos, double* qvel,
                    double* warm, const double* ctrl, const double* qfrc_applied,
                    const double* xfrc_applied);
int ilqg_forward_batch(const ilqg_model* m, int n, const double* qpos, const double* qvel,
                       double* warm, const double* ctrl, const double* qfrc_applied,
                       const double* xfrc_applied, double* qacc);
/* calcMJDerivatives (src/mjderivative.cpp:212-255) at n independent points;
   deriv is n x D.  cost may be NULL (cost-gradient entries then 0). */
int ilqg_fd_batch(const ilqg_model* m, int n, const double* qpos, const double* qvel,
                  const double* warm, const double* ctrl, const double* qfrc_applied,
                  const double* xfrc_applied, const ilqg_cost* cost, double* deriv);

/* ---- the iLQR solver context (ILQR<nv,nu,N>, inc/ilqr.h:14-188) ---- */
int ilqg_solver_create(const ilqg_model* m, const ilqg_solver_opts* opts, const ilqg_cost* cost,
                       ilqg_solver** out);
void ilqg_solver_free(ilqg_solver* s);
/* ILQR ctor (inc/ilqr.h:69-97): per seed, d = dmain; initial passive rollout
   with constant ctrl fills the trajectory; then setDInit(dmain).  dmain
   arrays are nseed x {1, nq, nv, nv, nu}; applied forces may be NULL (zero). */
int ilqg_solver_init(ilqg_solver* s, const double* time, const double* qpos, const double* qvel,
                     const double* warm, const double* ctrl, const double* qfrc_applied,
                     const double* xfrc_applied);
/* setDInit (inc/ilqr.h:110-113) per seed */
int ilqg_solver_set_dinit(ilqg_solver* s, const double* time, const double* qpos, const double* qvel,
                          const double* warm, const double* ctrl);
int ilqg_solver_set_traj(ilqg_solver* s, const double* time, const double* qpos, const double* qvel,
                         const double* warm, const double* ctrl);
int ilqg_solver_get_traj(ilqg_solver* s, double* time, double* qpos, double* qvel, double* warm,
                         double* ctrl);
int ilqg_solver_set_gains(ilqg_solver* s, const double* K, const double* k);
int ilqg_solver_get_gains(ilqg_solver* s, double* K, double* k);
int ilqg_solver_get_deriv(ilqg_solver* s, double* deriv);     /* nseed x (N+1) x D */
/* one FD record (D doubles) of seed `seed` at point `point` (0 = terminal) */
int ilqg_solver_get_deriv_point(ilqg_solver* s, int seed, int point, double* deriv);
/* overwrite the FD records before ilqg_backward, e.g. with cost-gradient
   entries from a host cost callback (stepCostFn_t, inc/mjderivative.h:5) */
int ilqg_solver_set_deriv(ilqg_solver* s, const double* deriv);
int ilqg_solver_get_value(ilqg_solver* s, double* V, double* v); /* nseed x nx x nx (col-major), nseed x nx */
/* per-seed trajectory cost of every candidate (nseed x nalpha) and the selected index */
int ilqg_solver_get_costs(ilqg_solver* s, double* cost, int* selected);

/* hot path, enqueued on the solver's stream (asynchronous) */
int ilqg_forward(ilqg_solver* s);   /* forwardPass over all candidates + selection (inc/ilqr.h:116-130) */
int ilqg_fd_sweep(ilqg_solver* s);  /* calcMJDerivatives at every point of every seed */
int ilqg_backward(ilqg_solver* s);  /* initV + Riccati n = 1..N (inc/ilqr.h:100-107,133-176) */
/* calcMJDerivatives at points p0 .. p0+np-1 of every seed (one rank's share
   of a point-sharded sweep, src/mjderivative.cpp:212-255 per point; records
   identical to ilqg_fd_sweep's).  With the records of the other points
   written into the buffer ilqg_solver_device_deriv exposes (an all-gather),
   ilqg_backward then runs the recursion over all of them. */
int ilqg_fd_sweep_range(ilqg_solver* s, int p0, int np);
/* One seed's iteration point-sharded over `world` ranks, pipelined
   (BASELINE.json configs[4]: one humanoid seed on 8 GPUs).  Every rank runs
   the whole rollout (forwardPass, inc/ilqr.h:116-130, in the pipelined
   iterate's chunks) and, behind each chunk, calcMJDerivatives
   (src/mjderivative.cpp:212-255) at the points it owns (point_owners), then
   selection / setDInit (inc/ilqr.h:110-113); the solver's stream is left
   behind every sweep launch.  The caller then gathers the other ranks'
   records into ilqg_solver_device_deriv's buffer and calls ilqg_backward.
   ILQG_ERR_UNSUPPORTED unless the solver pipelines its iterate (one candidate
   per seed, the unfused sweep: fp32 FD or the MFMA recursion).  world = 1 is
   ilqg_iterate without the backward pass. */
int ilqg_forward_sharded(ilqg_solver* s, int rank, int world);
/* owner[p] (p = 0 .. npoint-1, 0 = terminal) = the rank that differentiates
   point p under ilqg_forward_sharded: the pipelined rollout's chunks of
   `chunk` points (launch order: descending from npoint - 1) dealt round-robin,
   the last two chunks' points in contiguous blocks over every rank.  Pure host
   logic (no device).  solver_point_owners: the same for a solver's chunking. */
int ilqg_point_owners(int npoint, int chunk, int world, int* owner);
int ilqg_solver_point_owners(ilqg_solver* s, int world, int* owner);
int ilqg_iterate(ilqg_solver* s);   /* forwardPass; setDInit(dArray[N]); backwardPass (inc/ilqr.h:179-186) */
/* waits for every launch; returns ILQG_ERR_HIP once if a fused sweep's
   hand-off wait timed out since the last call (the report is cleared by it) */
int ilqg_synchronize(ilqg_solver* s);
/* test hook: preset the fault report word that ilqg_synchronize reads */
int ilqg_solver_debug_set_fault(ilqg_solver* s, unsigned value);
/* test hook: run the fused sweep's ticket planner on the durations the last
   sweep recorded and copy out the schedule (slot -> FD item) and the
   durations; nitems = the sweep's FD item count (0: no fused sweep) */
int ilqg_solver_debug_plan(ilqg_solver* s, unsigned* order, unsigned* dur, int* nitems);
/* test hook: the next fused sweep's ticket map (planned, or the identity) gets
   order[slot] = item before it is validated (calls accumulate until then).  Every map is checked on the
   device (items in range, none repeated, every column behind its centre); an
   invalid one is replaced by the identity, the sweep runs normally, and
   ilqg_synchronize returns ILQG_ERR_HIP once ("invalid ticket schedule") */
int ilqg_solver_debug_plant_schedule(ilqg_solver* s, unsigned slot, unsigned item);
void* ilqg_solver_stream(ilqg_solver* s); /* hipStream_t */
/* enqueue subsequent hot-path launches on an external stream (hipStream_t,
   e.g. torch's current stream) instead of the solver's own; NULL restores it */
int ilqg_solver_set_stream(ilqg_solver* s, void* stream);
/* per-kernel HIP-event timing of the hot path, recorded on the launch stream:
   index 0 rollout, 1 select, 2 fd_centre, 3 fd_cols (or the fused sweep run
   alone), 4 backward, 5 fd_backward (the fused sweep with the backward pass
   streamed behind it: ilqg_iterate on cooperative models) */
#define ILQG_NKERNEL 6
int ilqg_solver_set_timing(ilqg_solver* s, int enable);
/* synchronises; returns summed device ms and launch counts per kernel, then resets */
int ilqg_solver_get_timing(ilqg_solver* s, double* ms, int* launches);
/* How the Riccati recursion reads the FD records (Differentiator::
   updateDerivatives, inc/differentiator.h:85-93).  REFERENCE (default): as the
   reference does -- Eigen column-major maps of the row-major deriv blocks
   (differentiator.h:57-59), i.e. A's lower blocks are
   dt J^T and B's lower block is a permutation of dt J_u when nu > 1.
   CORRECTED: the true linearisation, A lower = [dt J_q, I + dt J_v], B lower =
   dt J_u (SURVEY.md Appendix A Q1 "provide a corrected mode").  The FD records
   themselves (ilqg_solver_get_deriv) are the reference's either way. */
#define ILQG_LAYOUT_REFERENCE 0
#define ILQG_LAYOUT_CORRECTED 1
int ilqg_solver_set_layout(ilqg_solver* s, int layout);
/* initV override (virtual ILQR::initV, inc/ilqr.h:100-107,142): the next
   backward pass (ilqg_backward or ilqg_iterate) starts its recursion from
   these V0 (nseed x nx x nx, column-major) and v0 (nseed x nx) instead of the
   terminal point's v = dgdx, V = v'v.  One-shot: later passes use initV. */
int ilqg_solver_set_value(ilqg_solver* s, const double* V, const double* v);
/* Levenberg-Marquardt constant mu (the public ILQR::mu, inc/ilqr.h:65, read
   by every backward step at inc/ilqr.h:166): used by every backward pass
   enqueued after the call (opts.mu at creation until then).  NaN is refused. */
int ilqg_solver_set_mu(ilqg_solver* s, double mu);
/* Riccati recursion (inc/ilqr.h:133-176) engine.  EXACT (default): the
   oracle's loops, bit-identical K, k, V, v (streamed behind the FD sweep on
   cooperative models).  MFMA: every matrix product (B'V, Quu = -2B'VB - 2R,
   Qux = B'VA, A + BK, (A+BK)'V(A+BK), K'RK) on the fp64 matrix cores
   (v_mfma_f64_16x16x4_f64), four wavefronts per seed -- the north star's
   "MFMA on the Quu/Qux block products" for large nu x nx (humanoid 21 x 54);
   results agree with EXACT to rounding (product sums in the matrix core's
   order).  BASELINE.json configs[4]. */
#define ILQG_RICCATI_EXACT 0
#define ILQG_RICCATI_MFMA 1
int ilqg_solver_set_riccati(ilqg_solver* s, int mode);
/* FD sweep precision (calcMJDerivatives, src/mjderivative.cpp:212-255).  F64
   (default): the reference's fp64 arithmetic and eps = 1e-6, bit-identical to
   the oracle.  F32: BASELINE.json configs[4]'s "fp32 FD with fp64 Riccati" --
   the physics of every FD evaluation in fp32 (workspace, state and arithmetic;
   the model stays fp64), eps = ILQG_FD32_EPS (1e-6 is below fp32 resolution,
   SURVEY.md §7(g)), fp64 records for the fp64 (exact or MFMA) recursion.
   Agrees with the fp64 oracle at the same eps to the tolerance stated in
   tests/test_gpu_parity.py (fp32 rounding amplified by 1/(2 eps)). */
#define ILQG_FD_F64 0
#define ILQG_FD_F32 1
#define ILQG_FD32_EPS 1e-3
int ilqg_solver_set_fd_precision(ilqg_solver* s, int prec);
/* Seed groups: ilqg_iterate runs the seeds as ngroups (1..4, <= nseed)
   contiguous ranges, software-pipelined -- each group's rollout on a stream
   CU-masked to XCDs of its own, its fused FD sweep + recursion on a stream
   masked to the rest, and group g's rollout of an iteration behind group
   g - 1's, so one group's sweep runs beside the next group's (latency-bound)
   rollout.  Every seed's launches and results are the ungrouped iterate's (bit
   for bit); only the overlap between independent seeds changes.  Work enqueued
   on the solver's stream after ilqg_iterate waits for every group; the groups
   wait for work on that stream only when it came through this API (ilqg_forward,
   ilqg_fd_sweep, ilqg_backward, set_stream, join_stream ...) -- work of your
   own enqueued there (a collective reading the costs) must be followed by
   ilqg_solver_join_stream before the next ilqg_iterate.  The seeds of MahanFathi/iLQG-MuJoCo's
   driver are independent (one ILQR per MPC problem, inc/ilqr.h:52-71), so
   the reference has no counterpart call.  ILQG_ERR_UNSUPPORTED unless the fused
   sweep is in use (fp64 FD, exact recursion, cooperative model); 1 restores
   the ungrouped iterate.  get_groups: the count and the CUs of each group's
   rollout mask (0: unmasked). */
int ilqg_solver_set_groups(ilqg_solver* s, int ngroups);
int ilqg_solver_get_groups(ilqg_solver* s, int* ngroups, int* rollout_cus);
/* the next ilqg_iterate's seed groups wait for everything enqueued on the
   solver's stream up to now (work of the caller's own, e.g. the RCCL cost
   all-gather, which reads the buffers the next rollout writes); without
   groups every launch is on that stream anyway and this is a no-op */
int ilqg_solver_join_stream(ilqg_solver* s);
/* sha256 prefix (16 hex digits) of the sources this library was built from
   (csrc/**, Makefile; the same digest as ilqg_amd.source_sha()): the host
   refuses a library whose digest differs from the sources beside it */
const char* ilqg_source_sha(void);
/* device pointer to the per-seed selected-candidate cost (nseed doubles), for
   an in-stream collective (RCCL all-gather) without a host round trip */
int ilqg_solver_device_costs(ilqg_solver* s, double** dptr);
/* device pointer to the resident FD records, [nseed][N+1][stride] doubles
   (stride >= D: each record padded to whole 128-byte lines) */
int ilqg_solver_device_deriv(ilqg_solver* s, double** dptr, int* stride);
/* device pointer to the resident nominal trajectory (field 0 time, 1 qpos,
   2 qvel, 3 warm, 4 ctrl; seed-major [nseed][N+1][...], point N = the first
   applied control): the multi-GPU MPC broadcast of the winning seed's first
   control reads it in place */
int ilqg_solver_device_traj(ilqg_solver* s, int field, double** dptr);
/* test hook: q[i] = a[i] / b[i] (host arrays, n <= 2^24) through the device's
   split fp64 division (divisor reciprocal computed ahead, dsmall.h rcp_ref /
   div_ref), both the every-lane and the one-lane form; q2 may be NULL.  The
   physics kernels use it for the Cholesky solve and the line search, so it
   must equal IEEE division bit for bit */
int ilqg_selftest_div(const double* a, const double* b, double* q, double* q2, int n);
#ifdef __cplusplus
}
#endif
#endif
