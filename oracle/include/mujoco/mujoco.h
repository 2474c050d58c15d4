/*
 * ORACLE / TEST INFRASTRUCTURE ONLY.  Never linked into the product library.
 *
 * MuJoCo-2.0-compatible C API subset used by the reference's FD driver
 * (/root/reference/src/mjderivative.cpp, src/util.cpp, src/update.cpp) and by
 * the oracle's own CPU restatement of the iLQR hot path.  The physics behind it
 * (oracle/mjsub.c) is a plain-C restatement of MuJoCo 2.0's documented
 * pipeline for the features used by res/{inverted_pendulum,hopper,humanoid}.xml
 * (SURVEY.md Appendix B).  MuJoCo 2.0 itself is absent from this container, so
 * fidelity to the real engine is "parity unpinned" (SURVEY.md §8c).
 *
 * The struct tags _mjModel/_mjData are kept so that the reference's
 * calcMJDerivatives mangles to the same symbol as against real MuJoCo
 * (SURVEY.md §8b).
 */
#pragma once

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#ifdef ORA_MJTNUM
typedef ORA_MJTNUM mjtNum; /* instrumented flop-counting build (oracle/flops) */
#else
typedef double mjtNum;
#define ORA_FLOP_TRANS() ((void)0)
#endif
typedef unsigned char mjtByte;

#define mjPI            3.14159265358979323846
#define mjMINVAL        1E-15
#define mjMAXVAL        1E+10
#define mjMINIMP        0.0001
#define mjMAXIMP        0.9999
#define mjNREF          2
#define mjNIMP          5

#define mjMIN(a, b)     (((a) < (b)) ? (a) : (b))
#define mjMAX(a, b)     (((a) > (b)) ? (a) : (b))

/* stack helpers, exactly as MuJoCo 2.0 defines them */
#define mjMARKSTACK     int _mark = d->pstack;
#define mjFREESTACK     d->pstack = _mark;

typedef enum _mjtJoint { mjJNT_FREE = 0, mjJNT_BALL, mjJNT_SLIDE, mjJNT_HINGE } mjtJoint;
typedef enum _mjtGeom {
  mjGEOM_PLANE = 0, mjGEOM_HFIELD, mjGEOM_SPHERE, mjGEOM_CAPSULE,
  mjGEOM_ELLIPSOID, mjGEOM_CYLINDER, mjGEOM_BOX, mjGEOM_MESH
} mjtGeom;
typedef enum _mjtStage { mjSTAGE_NONE = 0, mjSTAGE_POS, mjSTAGE_VEL, mjSTAGE_ACC } mjtStage;
typedef enum _mjtIntegrator { mjINT_EULER = 0, mjINT_RK4 } mjtIntegrator;
typedef enum _mjtCone { mjCONE_PYRAMIDAL = 0, mjCONE_ELLIPTIC } mjtCone;
typedef enum _mjtSolver { mjSOL_PGS = 0, mjSOL_CG, mjSOL_NEWTON } mjtSolver;
typedef enum _mjtConstraint {
  mjCNSTR_EQUALITY = 0, mjCNSTR_FRICTION_DOF, mjCNSTR_FRICTION_TENDON,
  mjCNSTR_LIMIT_JOINT, mjCNSTR_LIMIT_TENDON, mjCNSTR_CONTACT_FRICTIONLESS,
  mjCNSTR_CONTACT_PYRAMIDAL, mjCNSTR_CONTACT_ELLIPTIC
} mjtConstraint;

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
  int nq, nv, nu, na, nbody, njnt, ngeom;
  int nconmax, njmax, nstack;
  int nbuffer;                  /* bytes of the mjData arena (MuJoCo 2.0 semantics) */

  mjOption opt;
  mjStatistic stat;

  mjtNum* qpos0;                /* nq */
  mjtNum* qpos_spring;          /* nq */

  int* body_parentid;           /* nbody */
  int* body_rootid;
  int* body_weldid;
  int* body_jntnum;
  int* body_jntadr;
  int* body_dofnum;
  int* body_dofadr;
  int* body_geomnum;
  int* body_geomadr;
  mjtNum* body_pos;             /* nbody x 3 */
  mjtNum* body_quat;            /* nbody x 4 */
  mjtNum* body_ipos;            /* nbody x 3 */
  mjtNum* body_iquat;           /* nbody x 4 */
  mjtNum* body_mass;            /* nbody */
  mjtNum* body_subtreemass;     /* nbody */
  mjtNum* body_inertia;         /* nbody x 3 */
  mjtNum* body_invweight0;      /* nbody x 2 */

  int* jnt_type;                /* njnt */
  int* jnt_qposadr;
  int* jnt_dofadr;
  int* jnt_bodyid;
  int* jnt_limited;
  mjtNum* jnt_solref;           /* njnt x 2 */
  mjtNum* jnt_solimp;           /* njnt x 5 */
  mjtNum* jnt_pos;              /* njnt x 3 */
  mjtNum* jnt_axis;             /* njnt x 3 */
  mjtNum* jnt_stiffness;        /* njnt */
  mjtNum* jnt_range;            /* njnt x 2 */
  mjtNum* jnt_margin;           /* njnt */

  int* dof_bodyid;              /* nv */
  int* dof_jntid;
  int* dof_parentid;
  mjtNum* dof_armature;
  mjtNum* dof_damping;
  mjtNum* dof_invweight0;

  int* geom_type;               /* ngeom */
  int* geom_contype;
  int* geom_conaffinity;
  int* geom_condim;
  int* geom_bodyid;
  mjtNum* geom_solmix;
  mjtNum* geom_solref;          /* ngeom x 2 */
  mjtNum* geom_solimp;          /* ngeom x 5 */
  mjtNum* geom_size;            /* ngeom x 3 */
  mjtNum* geom_rbound;
  mjtNum* geom_pos;             /* ngeom x 3 */
  mjtNum* geom_quat;            /* ngeom x 4 */
  mjtNum* geom_friction;        /* ngeom x 3 */
  mjtNum* geom_margin;
  mjtNum* geom_gap;

  int* actuator_trnid;          /* nu (joint id) */
  int* actuator_ctrllimited;
  int* actuator_forcelimited;
  mjtNum* actuator_gear;        /* nu (first gear component) */
  mjtNum* actuator_ctrlrange;   /* nu x 2 */
  mjtNum* actuator_forcerange;  /* nu x 2 */
  mjtNum* actuator_gainprm;     /* nu (first gain parameter) */

  void* _arena;                 /* owner of every array above */
};
typedef struct _mjModel mjModel;

struct _mjContact {
  mjtNum dist;
  mjtNum pos[3];
  mjtNum frame[9];
  mjtNum includemargin;
  mjtNum friction[5];
  mjtNum solref[mjNREF];
  mjtNum solimp[mjNIMP];
  int dim;
  int geom1;
  int geom2;
  int efc_address;
};
typedef struct _mjContact mjContact;

struct _mjData {
  int nstack;
  int nbuffer;
  int pstack;
  int maxuse_stack;
  int ncon;
  int nefc;
  int solver_iter;

  mjtNum time;

  /* state + control (the cpMjData record, util.cpp:4-14) */
  mjtNum* qpos;
  mjtNum* qvel;
  mjtNum* act;
  mjtNum* qacc_warmstart;
  mjtNum* ctrl;
  mjtNum* qfrc_applied;
  mjtNum* xfrc_applied;
  mjtNum* qacc;

  /* position stage */
  mjtNum* xpos;  mjtNum* xquat;  mjtNum* xmat;
  mjtNum* xipos; mjtNum* ximat;
  mjtNum* xanchor; mjtNum* xaxis;
  mjtNum* geom_xpos; mjtNum* geom_xmat;
  mjtNum* subtree_com;
  mjtNum* cdof;
  mjtNum* cinert;
  mjtNum* crb;
  mjtNum* qM;                   /* nv x nv dense, symmetric */
  mjtNum* qLD;                  /* nv x nv dense: L (ancestor entries) + D on diagonal */
  mjtNum* qLDiagInv;
  mjtNum* actuator_moment;      /* nu x nv */
  mjtNum* actuator_length;
  mjContact* contact;           /* nconmax */
  int* efc_type;                /* njmax */
  int* efc_id;
  mjtNum* efc_J;                /* njmax x nv */
  mjtNum* efc_pos;
  mjtNum* efc_margin;
  mjtNum* efc_diagApprox;
  mjtNum* efc_R;
  mjtNum* efc_D;
  mjtNum* efc_KBIP;             /* njmax x 4 */
  mjtNum* efc_AR;               /* njmax x njmax (MuJoCo 2.0 arena sizing; unused by Newton) */

  /* velocity stage */
  mjtNum* cvel;
  mjtNum* cdof_dot;
  mjtNum* qfrc_passive;
  mjtNum* qfrc_bias;
  mjtNum* efc_vel;
  mjtNum* efc_aref;

  /* acceleration stage */
  mjtNum* actuator_force;
  mjtNum* qfrc_actuator;
  mjtNum* qfrc_smooth;
  mjtNum* qacc_smooth;
  mjtNum* qfrc_constraint;
  mjtNum* efc_force;
  mjtNum* efc_b;
  int* efc_state;

  mjtNum* stack;                /* nstack mjtNums */
  void* buffer;                 /* arena */
};
typedef struct _mjData mjData;

/* ---- model / data lifecycle ---- */
mjModel* mj_loadBlob(const void* blob, size_t nbytes, char* error, int error_sz);
void mj_deleteModel(mjModel* m);
mjData* mj_makeData(const mjModel* m);
void mj_deleteData(mjData* d);
void mj_resetData(const mjModel* m, mjData* d);
int mj_activate(const char* filename);
void mj_deactivate(void);

/* ---- pipeline ---- */
void mj_step(const mjModel* m, mjData* d);
void mj_forward(const mjModel* m, mjData* d);
void mj_forwardSkip(const mjModel* m, mjData* d, int skipstage, int skipsensor);
void mj_Euler(const mjModel* m, mjData* d);
void mj_RungeKutta(const mjModel* m, mjData* d, int N);

/* ---- stack ---- */
mjtNum* mj_stackAlloc(mjData* d, int size);

/* ---- utilities used by the reference ---- */
void mju_copy(mjtNum* res, const mjtNum* data, int n);
void mju_zero(mjtNum* res, int n);
void* mju_malloc(size_t size);
void mju_free(void* ptr);
void mju_error(const char* msg);
void mju_error_s(const char* msg, const char* text);
void mju_quatIntegrate(mjtNum quat[4], const mjtNum vel[3], mjtNum scale);

/* deterministic sin/cos shared by the restatement (fdlibm kernels, no libm) */
mjtNum ora_sin(mjtNum x);
mjtNum ora_cos(mjtNum x);

#ifdef __cplusplus
}
#endif
