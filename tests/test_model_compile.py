"""MJCF subset compiler (product, host-only) -- counts, units, inertia, record
round trip into the oracle.  SURVEY.md §4 item 1."""
import math

import numpy as np
import pytest

from conftest import model_path


@pytest.mark.parametrize("name,counts", [
    ("inverted_pendulum", (2, 2, 1, 3, 3)),
    ("hopper", (6, 6, 3, 5, 5)),
    ("humanoid", (28, 27, 21, 14, 20)),
])
def test_counts(ia, name, counts):
    m = ia.Model.load(model_path(name))
    assert (m.nq, m.nv, m.nu, m.nbody, m.ngeom) == counts


def test_pendulum_units_and_options(ia, ora):
    m = ia.Model.load(model_path("inverted_pendulum"))
    assert m.timestep == 0.02
    om = ora.OModel(m.blob())
    assert om.nstack == 3000  # <size nstack="3000">
    blob = _fields(m.blob())
    # hinge range -90..90 deg -> radians (2.0 default angle unit: degree)
    assert np.allclose(blob["jnt_range"].reshape(-1, 2)[1], [-math.pi / 2, math.pi / 2])
    assert np.allclose(blob["jnt_range"].reshape(-1, 2)[0], [-1, 1])  # slide: no conversion
    assert blob["opt_integrator"][0] == 1  # RK4
    # motor: gear 100, ctrllimited defaults to false in 2.0
    assert blob["actuator_gear"][0] == 100 and blob["actuator_ctrllimited"][0] == 0
    # all geoms contype 0 -> no contact pairs
    assert m.maxcon == 0


def test_pendulum_pole_mass(ia):
    m = ia.Model.load(model_path("inverted_pendulum"))
    b = _fields(m.blob())
    r, L = 0.049, math.hypot(0.001, 0.6)
    expect = 1000 * (math.pi * r * r * L + 4.0 / 3.0 * math.pi * r ** 3)
    assert b["body_mass"][2] == pytest.approx(expect, rel=1e-12)
    # COM at the capsule midpoint in the pole body frame
    assert np.allclose(b["body_ipos"].reshape(-1, 3)[2], [0.0005, 0, 0.3])


def test_hopper_global_coordinates(ia):
    m = ia.Model.load(model_path("hopper"))
    b = _fields(m.blob())
    # rootz ref=1.25 -> qpos0
    assert np.allclose(m.qpos0, [0, 1.25, 0, 0, 0, 0])
    # default joint armature/damping only on the leg joints
    assert np.allclose(b["dof_armature"], [0, 0, 0, 1, 1, 1])
    assert np.allclose(b["dof_damping"], [0, 0, 0, 1, 1, 1])
    # thigh range -150..0 deg
    assert np.allclose(b["jnt_range"].reshape(-1, 2)[3], [-150 * math.pi / 180, 0])
    # malformed pos="0.13/2 0 0.1" (hopper.xml:23) must not break compilation; the foot
    # geom must still sit at its global fromto midpoint
    xpos_foot = _global_geom_pos(b, 4)
    assert np.allclose(xpos_foot, [0.065, 0, 0.1], atol=1e-12)
    # floor x body geoms, capsule pairs not parent-child: 4x2 + 3x2 contacts
    assert m.maxcon == 14
    assert b["geom_condim"][0] == 3 and b["geom_condim"][1] == 1


def test_humanoid_free_joint(ia):
    m = ia.Model.load(model_path("humanoid"))
    b = _fields(m.blob())
    assert b["jnt_type"][0] == 0  # free
    assert np.allclose(m.qpos0[:7], [0, 0, 1.4, 1, 0, 0, 0])
    # freejoint ignores joint defaults (damping=1 in the default class)
    assert np.all(b["dof_damping"][:6] == 0)
    assert m.nconmax == 50 and m.njmax == 200


def test_record_roundtrip_into_oracle(ia, ora):
    for name in ("inverted_pendulum", "hopper", "humanoid"):
        m = ia.Model.load(model_path(name))
        om = ora.OModel(m.blob())
        assert (om.nq, om.nv, om.nu, om.nbody, om.ngeom) == (m.nq, m.nv, m.nu, m.nbody, m.ngeom)


def test_bad_model_reports_error(ia):
    with pytest.raises(ia.IlqgError, match="could not open"):
        ia.Model.load("/nonexistent.xml")
    with pytest.raises(ia.IlqgError, match="mismatched"):
        ia.Model.from_string("<mujoco><worldbody></body></mujoco>")


def _fields(blob):
    import struct
    assert blob[:8] == b"ILQGMDL1"
    (n,) = struct.unpack_from("<i", blob, 8)
    off, out = 16, {}
    for _ in range(n):
        name = blob[off:off + 48].split(b"\0")[0].decode()
        dtype, count = struct.unpack_from("<ii", blob, off + 48)
        off += 56
        sz = count * (8 if dtype == 0 else 4)
        out[name] = np.frombuffer(blob, dtype=np.float64 if dtype == 0 else np.int32, count=count, offset=off).copy()
        off += (sz + 7) & ~7
    return out


def _global_geom_pos(b, g):
    """compose body frames (quaternions) down the tree to get a geom's global position at qpos0"""
    def qmul(a, c):
        return np.array([a[0] * c[0] - a[1] * c[1] - a[2] * c[2] - a[3] * c[3],
                         a[0] * c[1] + a[1] * c[0] + a[2] * c[3] - a[3] * c[2],
                         a[0] * c[2] - a[1] * c[3] + a[2] * c[0] + a[3] * c[1],
                         a[0] * c[3] + a[1] * c[2] - a[2] * c[1] + a[3] * c[0]])

    def rot(q, v):
        qv = np.concatenate([[0], v])
        return qmul(qmul(q, qv), q * np.array([1, -1, -1, -1]))[1:]
    parent = b["body_parentid"]
    bpos, bquat = b["body_pos"].reshape(-1, 3), b["body_quat"].reshape(-1, 4)
    body = b["geom_bodyid"][g]
    chain = []
    while body:
        chain.append(body)
        body = parent[body]
    p, q = np.zeros(3), np.array([1.0, 0, 0, 0])
    for bb in reversed(chain):
        p = p + rot(q, bpos[bb])
        q = qmul(q, bquat[bb])
    return p + rot(q, b["geom_pos"].reshape(-1, 3)[g])


def test_static_specialisations_selected(ia):
    """the bundled models map to their compiled model-specific kernels
    (csrc/device/static_models.h, regenerated by tools/gen_static_models.py);
    anything else, e.g. the humanoid, runs the generic kernels"""
    ids = {n: ia.Model.load(model_path(n)).static_id() for n in ("inverted_pendulum", "hopper", "humanoid")}
    assert ids == {"inverted_pendulum": 1, "hopper": 2, "humanoid": 0}


def _chain_xml(n):
    """a planar chain of n hinged capsules over a floor (n dofs, every link can touch the floor)"""
    body = ""
    for i in reversed(range(n)):
        body = (f'<body name="b{i}" pos="0 0 {0.3 if i == 0 else 0.2}"><joint name="j{i}" type="hinge" axis="0 1 0"/>'
                f'<geom type="capsule" fromto="0 0 0 0 0 0.2" size="0.05"/>{body}</body>')
    acts = "".join(f'<motor joint="j{i}" gear="1"/>' for i in range(n))
    return (f'<mujoco><worldbody><geom type="plane" size="5 5 0.1"/>{body}</worldbody>'
            f'<actuator>{acts}</actuator></mujoco>')


def test_model_lds_limit_refused_at_load(ia):
    """the device paths keep one evaluation's workspace in one CU's LDS
    (include/ilqg_amd.h, model-size limit): a model over 160 KB fails cleanly
    at load with ILQG_ERR_UNSUPPORTED (no GPU needed), a small one loads"""
    small = ia.Model.from_string(_chain_xml(4))
    assert (small.nv, small.nu) == (4, 4)
    with pytest.raises(ia.IlqgError, match=r"code 4\).*exceeds one CU's LDS"):
        ia.Model.from_string(_chain_xml(48))
