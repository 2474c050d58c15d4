/*
 * MuJoCo 2.0 C API subset used by the reference's iLQR code, served by the
 * MI355X path (libilqg_mujoco.so over libilqg_amd.so).
 *
 * This is the product side of the legacy drop-in boundary:
 * source files written against MuJoCo 2.0 -- inc/mjderivative.h, inc/util.h,
 * inc/update.h and the inverted-pendulum controller sources -- compile against
 * it unchanged.
 * The struct tags are MuJoCo's (_mjModel/_mjData) so C++ symbols taking
 * mjModel* and mjData* mangle exactly as against the real MuJoCo, e.g.
 * _Z17calcMJDerivativesP8_mjModelP7_mjDataPdPFdPKS1_E.
 *
 * Physics (mj_step, mj_forward, calcMJDerivatives) runs on the GPU through the
 * C ABI in include/ilqg_amd.h; there is no CPU physics behind this header.
 * mjModel fields carry MuJoCo's names and meaning for the supported model
 * subset; mjData holds the state the reference reads and writes.
 */
#ifndef ILQG_LEGACY_MUJOCO_H
#define ILQG_LEGACY_MUJOCO_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef double mjtNum;
typedef unsigned char mjtByte;

#define mjMINVAL 1E-15
#define mjPI 3.14159265358979323846
#define mjMIN(a, b) (((a) < (b)) ? (a) : (b))
#define mjMAX(a, b) (((a) > (b)) ? (a) : (b))

typedef enum _mjtJoint { mjJNT_FREE = 0, mjJNT_BALL, mjJNT_SLIDE, mjJNT_HINGE } mjtJoint;
typedef enum _mjtGeom { mjGEOM_PLANE = 0, mjGEOM_HFIELD, mjGEOM_SPHERE, mjGEOM_CAPSULE } mjtGeom;
typedef enum _mjtStage { mjSTAGE_NONE = 0, mjSTAGE_POS, mjSTAGE_VEL, mjSTAGE_ACC } mjtStage;
typedef enum _mjtIntegrator { mjINT_EULER = 0, mjINT_RK4 } mjtIntegrator;

struct _mjOption {
  mjtNum timestep;
  mjtNum impratio;
  mjtNum tolerance;
  mjtNum gravity[3];
  int integrator;
  int cone;
  int solver;
  int iterations;
  int disableflags;
  int enableflags;
};
typedef struct _mjOption mjOption;

struct _mjStatistic {
  mjtNum meaninertia;
};
typedef struct _mjStatistic mjStatistic;

struct _mjModel {
  /* sizes */
  int nq, nv, nu, nbody, njnt, ngeom, nconmax, njmax, nstack;
  mjOption opt;
  mjStatistic stat;
  /* arrays (MuJoCo names; row-major as in MuJoCo) */
  mjtNum *qpos0, *qpos_spring;
  mjtNum *body_pos, *body_quat, *body_ipos, *body_iquat, *body_mass, *body_subtreemass, *body_inertia,
      *body_invweight0;
  mjtNum *jnt_solref, *jnt_solimp, *jnt_pos, *jnt_axis, *jnt_stiffness, *jnt_range, *jnt_margin;
  mjtNum *dof_armature, *dof_damping, *dof_invweight0;
  mjtNum *geom_solmix, *geom_solref, *geom_solimp, *geom_size, *geom_rbound, *geom_pos, *geom_quat,
      *geom_friction, *geom_margin, *geom_gap;
  mjtNum *actuator_gear, *actuator_ctrlrange, *actuator_forcerange, *actuator_gainprm;
  int *body_parentid, *body_rootid, *body_weldid, *body_jntnum, *body_jntadr, *body_dofnum, *body_dofadr,
      *body_geomnum, *body_geomadr;
  int *jnt_type, *jnt_qposadr, *jnt_dofadr, *jnt_bodyid, *jnt_limited;
  int *dof_bodyid, *dof_jntid, *dof_parentid;
  int *geom_type, *geom_contype, *geom_conaffinity, *geom_condim, *geom_bodyid;
  int *actuator_trnid, *actuator_ctrllimited, *actuator_forcelimited;
  /* library-private */
  void* ilqg_model; /* ilqg_model* of include/ilqg_amd.h */
  void* ilqg_arena;
};
typedef struct _mjModel mjModel;

struct _mjData {
  /* stack (mj_stackAlloc / mjMARKSTACK / mjFREESTACK) */
  int nstack;
  int pstack;
  int maxuse_stack;
  mjtNum* stack;
  /* state and control; qvel directly follows qpos in memory (inc/ilqr.h:90) */
  mjtNum time;
  mjtNum* qpos;
  mjtNum* qvel;
  mjtNum* qacc_warmstart;
  mjtNum* ctrl;
  mjtNum* qfrc_applied;
  mjtNum* xfrc_applied;
  /* outputs */
  mjtNum* qacc;
  /* library-private */
  void* ilqg_arena;
};
typedef struct _mjData mjData;

#define mjMARKSTACK int _mark = d->pstack;
#define mjFREESTACK d->pstack = _mark;

/* activation: no license is needed; kept for source compatibility (cmd/basic.cpp:116) */
int mj_activate(const char* filename);
void mj_deactivate(void);

/* model: MJCF subset compiled by the library's own compiler (mj_loadXML, cmd/basic.cpp:123) */
mjModel* mj_loadXML(const char* filename, const void* vfs, char* error, int error_sz);
void mj_deleteModel(mjModel* m);

/* data */
mjData* mj_makeData(const mjModel* m);
void mj_deleteData(mjData* d);
void mj_resetData(const mjModel* m, mjData* d);
mjtNum* mj_stackAlloc(mjData* d, int size);

/* physics on the GPU.  mj_step advances time/qpos/qvel/qacc_warmstart in
   place; mj_forward writes qacc and qacc_warmstart.  mj_forwardSkip computes
   every stage (equal to MuJoCo's result whenever the skipped stages are up to
   date, which is how src/mjderivative.cpp uses it). */
void mj_step(const mjModel* m, mjData* d);
void mj_forward(const mjModel* m, mjData* d);
void mj_forwardSkip(const mjModel* m, mjData* d, int skipstage, int skipsensor);

/* utilities */
void mju_copy(mjtNum* res, const mjtNum* data, int n);
void mju_zero(mjtNum* res, int n);
void* mju_malloc(size_t size);
void mju_free(void* ptr);
void mju_error(const char* msg);
void mju_error_s(const char* msg, const char* text);
void mju_quatIntegrate(mjtNum* quat, const mjtNum* vel, mjtNum scale);

#ifdef __cplusplus
}
#endif
#endif
