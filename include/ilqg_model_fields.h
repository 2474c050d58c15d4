/*
 * Field list of the compiled-model record (see ilqg_model_blob.h).  Shared by
 * the writer (product MJCF compiler) and every reader (oracle, device upload,
 * Python fixtures) so the record has one definition.
 *
 * X(name, count-expression-in-terms-of-sizes)
 */
#pragma once

/* int32 scalars, in this order, precede every array */
#define ILQG_MODEL_I32_SCALARS(X) \
  X(nq) X(nv) X(nu) X(nbody) X(njnt) X(ngeom) X(nconmax) X(njmax) X(nstack) \
  X(opt_integrator) X(opt_cone) X(opt_solver) X(opt_iterations) \
  X(opt_disableflags) X(opt_enableflags)

/* float64 scalars */
#define ILQG_MODEL_F64_SCALARS(X) \
  X(opt_timestep) X(opt_impratio) X(opt_tolerance) \
  X(opt_gravity0) X(opt_gravity1) X(opt_gravity2) X(stat_meaninertia)

#define ILQG_MODEL_F64_ARRAYS(X) \
  X(qpos0, nq) X(qpos_spring, nq) \
  X(body_pos, nbody * 3) X(body_quat, nbody * 4) X(body_ipos, nbody * 3) \
  X(body_iquat, nbody * 4) X(body_mass, nbody) X(body_subtreemass, nbody) \
  X(body_inertia, nbody * 3) X(body_invweight0, nbody * 2) \
  X(jnt_solref, njnt * 2) X(jnt_solimp, njnt * 5) X(jnt_pos, njnt * 3) \
  X(jnt_axis, njnt * 3) X(jnt_stiffness, njnt) X(jnt_range, njnt * 2) \
  X(jnt_margin, njnt) \
  X(dof_armature, nv) X(dof_damping, nv) X(dof_invweight0, nv) \
  X(geom_solmix, ngeom) X(geom_solref, ngeom * 2) X(geom_solimp, ngeom * 5) \
  X(geom_size, ngeom * 3) X(geom_rbound, ngeom) X(geom_pos, ngeom * 3) \
  X(geom_quat, ngeom * 4) X(geom_friction, ngeom * 3) X(geom_margin, ngeom) \
  X(geom_gap, ngeom) \
  X(actuator_gear, nu) X(actuator_ctrlrange, nu * 2) \
  X(actuator_forcerange, nu * 2) X(actuator_gainprm, nu)

#define ILQG_MODEL_I32_ARRAYS(X) \
  X(body_parentid, nbody) X(body_rootid, nbody) X(body_weldid, nbody) \
  X(body_jntnum, nbody) X(body_jntadr, nbody) X(body_dofnum, nbody) \
  X(body_dofadr, nbody) X(body_geomnum, nbody) X(body_geomadr, nbody) \
  X(jnt_type, njnt) X(jnt_qposadr, njnt) X(jnt_dofadr, njnt) \
  X(jnt_bodyid, njnt) X(jnt_limited, njnt) \
  X(dof_bodyid, nv) X(dof_jntid, nv) X(dof_parentid, nv) \
  X(geom_type, ngeom) X(geom_contype, ngeom) X(geom_conaffinity, ngeom) \
  X(geom_condim, ngeom) X(geom_bodyid, ngeom) \
  X(actuator_trnid, nu) X(actuator_ctrllimited, nu) X(actuator_forcelimited, nu)
