"""The product's MJCF compiler (csrc/model/mjcf.cpp + setconst.cpp) against an
independent compile of the same XML (tests/mjcf_indep.py), field by field.
The oracle loads the product's compiled record, so without this check the
model compile would be a common-mode input of every parity test.  Frame-
dependent fields are compared as world-frame invariants at qpos0 (hopper.xml:23's
malformed body pos moves the body frame, not the physics).  Tolerance: 1e-10
relative (+1e-12 absolute); integer and flag fields exactly."""
import numpy as np
import pytest

import mjcf_indep as mi
from conftest import model_path
from test_model_compile import _fields

MODELS = ["inverted_pendulum", "hopper", "humanoid"]
RTOL, ATOL = 1e-10, 1e-12


def close(a, b, what):
    a, b = np.asarray(a, float), np.asarray(b, float)
    if a.size == 1 and b.size == 1:
        a, b = a.reshape(()), b.reshape(())
    assert a.shape == b.shape, (what, a.shape, b.shape)
    assert np.allclose(a, b, rtol=RTOL, atol=ATOL), f"{what}: max|diff| {np.max(np.abs(a - b)):.3e}\n{a}\n{b}"


def qmat(q):
    return mi.qmat(np.asarray(q, float))


def world_frames(f, qpos0):
    """body world frames of the product's record at qpos0 (joint displacements
    qpos - qpos0 are zero; a free joint places its body at its qpos0 pose)"""
    nb = len(f["body_parentid"])
    bp, bq = f["body_pos"].reshape(-1, 3), f["body_quat"].reshape(-1, 4)
    xpos, xq = np.zeros((nb, 3)), np.zeros((nb, 4))
    xq[0] = [1, 0, 0, 0]
    for b in range(1, nb):
        p = f["body_parentid"][b]
        xpos[b] = xpos[p] + qmat(xq[p]) @ bp[b]
        xq[b] = mi.qmul(xq[p], bq[b])
        for j in range(f["body_jntadr"][b], f["body_jntadr"][b] + f["body_jntnum"][b]):
            if f["jnt_type"][j] == 0:
                a = f["jnt_qposadr"][j]
                xpos[b], xq[b] = qpos0[a:a + 3], qpos0[a + 3:a + 7]
    return xpos, xq


@pytest.fixture(scope="module", params=MODELS)
def pair(request, ia):
    m = ia.Model.load(model_path(request.param))
    return request.param, _fields(m.blob()), m, mi.compile_mjcf(model_path(request.param))


def test_sizes_topology_options(pair):
    name, f, m, r = pair
    assert (m.nq, m.nv, m.nu, m.nbody, m.ngeom) == (r.nq, r.nv, len(r.act), r.nbody, r.ngeom)
    assert list(f["body_parentid"]) == [b["parent"] for b in r.bodies]
    assert list(f["jnt_type"]) == [mi.TYPES[j["type"]] for j in r.joints]
    assert list(f["jnt_bodyid"]) == [j["body"] for j in r.joints]
    assert list(f["dof_jntid"]) == r.dof_joint and list(f["dof_bodyid"]) == r.dof_body
    assert list(f["geom_bodyid"]) == [g["body"] for g in r.geoms]
    assert list(f["geom_type"]) == [{"plane": 0, "sphere": 2, "capsule": 3}[g["type"]] for g in r.geoms]
    close(f["opt_timestep"], r.timestep, "timestep")
    close([f["opt_gravity0"][0], f["opt_gravity1"][0], f["opt_gravity2"][0]], r.gravity, "gravity")
    assert f["opt_integrator"][0] == r.integrator
    assert f["opt_iterations"][0] == r.iterations
    close(f["opt_tolerance"], r.tolerance, "tolerance")


def test_joint_and_dof_parameters(pair):
    name, f, m, r = pair
    J = r.joints
    close(m.qpos0, r.qpos0, "qpos0 (joint ref, free-joint pose)")
    assert list(f["jnt_limited"]) == [int(j["limited"]) for j in J]
    close(f["jnt_range"].reshape(-1, 2), [j["range"] for j in J], "jnt_range (radians)")
    close(f["jnt_stiffness"], [j["stiffness"] for j in J], "jnt_stiffness")
    close(f["jnt_solref"].reshape(-1, 2), [j["solreflimit"] for j in J], "jnt_solref")
    close(f["jnt_solimp"].reshape(-1, 5), [j["solimplimit"] for j in J], "jnt_solimp")
    close(f["dof_armature"], [J[j]["armature"] for j in r.dof_joint], "dof_armature")
    close(f["dof_damping"], [J[j]["damping"] for j in r.dof_joint], "dof_damping")


def test_geom_parameters(pair):
    name, f, m, r = pair
    G = r.geoms
    assert list(f["geom_contype"]) == [int(g["contype"]) for g in G]
    assert list(f["geom_conaffinity"]) == [int(g["conaffinity"]) for g in G]
    assert list(f["geom_condim"]) == [int(g["condim"]) for g in G]
    close(f["geom_friction"].reshape(-1, 3), [g["friction"] for g in G], "geom_friction")
    close(f["geom_margin"], [g["margin"] for g in G], "geom_margin")
    close(f["geom_solref"].reshape(-1, 2), [g["solref"] for g in G], "geom_solref")
    close(f["geom_solimp"].reshape(-1, 5), [g["solimp"] for g in G], "geom_solimp")
    close(f["geom_solmix"], [g["solmix"] for g in G], "geom_solmix")
    sz = f["geom_size"].reshape(-1, 3)
    for i, g in enumerate(G):
        n = {"plane": 3, "sphere": 1, "capsule": 2}[g["type"]]
        close(sz[i, :n], g["size"][:n], f"geom_size[{i}]")


def test_actuators(pair):
    name, f, m, r = pair
    A = r.act
    assert list(f["actuator_trnid"]) == [a["joint"] for a in A]
    close(f["actuator_gear"], [a["gear"][0] for a in A], "gear")
    close(f["actuator_ctrlrange"].reshape(-1, 2), [a["ctrlrange"] for a in A], "ctrlrange")
    close(f["actuator_forcerange"].reshape(-1, 2), [a["forcerange"] for a in A], "forcerange")
    assert list(f["actuator_ctrllimited"]) == [int(a["ctrllimited"]) for a in A]


def test_world_frame_invariants(pair):
    """joint anchors/axes, geom centres and axes, body COMs and inertia tensors in
    the world frame at qpos0 -- independent of where each body frame was put"""
    name, f, m, r = pair
    xpos, xq = world_frames(f, m.qpos0)
    for j, jr in enumerate(r.joints):
        b = f["jnt_bodyid"][j]
        R = qmat(xq[b])
        if jr["type"] != "free":
            close(xpos[b] + R @ f["jnt_pos"].reshape(-1, 3)[j], jr["gpos"], f"joint {j} anchor")
            close(R @ f["jnt_axis"].reshape(-1, 3)[j], jr["gaxis"], f"joint {j} axis")
    for g, gr in enumerate(r.geoms):
        b = f["geom_bodyid"][g]
        R = qmat(xq[b])
        close(xpos[b] + R @ f["geom_pos"].reshape(-1, 3)[g], gr["gpos"], f"geom {g} centre")
        if gr["type"] == "capsule":  # the symmetry axis (z of the geom frame)
            zp = (R @ qmat(f["geom_quat"].reshape(-1, 4)[g]))[:, 2]
            zr = qmat(gr["gquat"])[:, 2]
            close(zp, zr, f"geom {g} axis")
    close(f["body_mass"], r.body_mass, "body_mass")
    for b in range(1, r.nbody):
        if r.body_mass[b] <= 0:
            continue
        R = qmat(xq[b])
        close(xpos[b] + R @ f["body_ipos"].reshape(-1, 3)[b], r.body_com[b], f"body {b} COM")
        Ri = R @ qmat(f["body_iquat"].reshape(-1, 4)[b])
        Iw = Ri @ np.diag(f["body_inertia"].reshape(-1, 3)[b]) @ Ri.T
        close(Iw, r.body_I[b], f"body {b} inertia tensor")
        close(np.sort(f["body_inertia"].reshape(-1, 3)[b]), np.sort(np.linalg.eigvalsh(r.body_I[b])),
              f"body {b} principal inertia")


def test_set_const(pair):
    """mj_setConst at qpos0: subtree masses, M(qpos0) diagonal inverse weights,
    body inverse weights (efc_R's diagApprox), mean inertia"""
    name, f, m, r = pair
    close(f["body_subtreemass"], r.body_subtreemass, "body_subtreemass")
    close(f["dof_invweight0"], r.dof_invweight0, "dof_invweight0")
    close(f["body_invweight0"].reshape(-1, 2), r.body_invweight0, "body_invweight0")
    close(f["stat_meaninertia"], r.stat_meaninertia, "stat_meaninertia")


def test_dynamics_at_qpos0(pair, ora):
    """the oracle's physics on the product's record at rest at qpos0 against the
    independent model: qfrc_bias = -sum_b m_b Jp_b' g (gravity; qvel = 0) and
    qacc_smooth = M(qpos0)^-1 (-qfrc_bias) (no springs, dampers or controls act
    at rest at qpos0) -- the whole mass matrix, frames, masses and inertias"""
    name, f, m, r = pair
    om = ora.OModel(m.blob())
    d = om.make_data()
    d.set_state(qpos=m.qpos0, qvel=np.zeros(m.nv), ctrl=np.zeros(m.nu))
    d.forward()
    g = np.asarray(r.gravity, float)
    bias = -sum(r.body_mass[b] * r.body_jac[b][0].T @ g for b in range(1, r.nbody))
    assert np.allclose(d.arr("qfrc_bias"), bias, rtol=1e-9, atol=1e-9)
    assert np.allclose(d.arr("qacc_smooth"), np.linalg.solve(r.Mq0, -bias), rtol=1e-9, atol=1e-9)
