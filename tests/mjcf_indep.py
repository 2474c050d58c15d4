"""TEST INFRASTRUCTURE: an independent MJCF compiler for the reference's three
models (res/inverted_pendulum.xml, res/hopper.xml, res/humanoid.xml), written
from MuJoCo 2.0's documented XML semantics with numpy, sharing no code with
the product's compiler (ilqg-mujoco_amd/csrc/model/mjcf.cpp, setconst.cpp)
or the oracle (which loads the product's compiled record).  It removes the
model compile as a common-mode input of every parity test (VERDICT r1
"Missing" #2): tests/test_model_indep.py compares the product's record with
this one field by field.

Semantics restated (MuJoCo 2.0 XML reference):
  * compiler: angle (default "degree"), coordinate ("local" | "global"),
    inertiafromgeom (body mass / COM / inertia from the geoms, density 1000)
  * one unnamed top-level <default> class; element attributes override it;
    a partially given vector attribute keeps the class/builtin values for the
    components it does not give (friction="0.9", solimp=".8 .8 .01")
  * numbers are read as C strtod prefixes ("0.13/2" -> 0.13, hopper.xml:23)
  * fromto: pos = midpoint, frame z along the segment (minimal rotation from +z),
    size[1] = half length; capsule = cylinder + two solid hemispheres
  * global coordinates: body, joint and geom frames given in the world frame
  * hinge/ball angles (range, ref, springref) in degrees when angle="degree"
  * freejoint: qpos0 = the body's world pose, joint defaults not applied
  * mj_setConst at qpos0: M(qpos0) from body COM Jacobians (sum_b J'M_bJ +
    armature), dof_invweight0 = diag(M^-1), body_invweight0 = mean diagonal of
    J M^-1 J' (translation, rotation) at the body COM, stat_meaninertia = tr(M)/nv
"""
import math
import re
import xml.etree.ElementTree as ET

import numpy as np

_NUM = re.compile(r"^\s*([-+]?(?:\d+\.?\d*|\.\d+)(?:[eE][-+]?\d+)?)")

JOINT_BUILTIN = dict(type="hinge", pos=[0, 0, 0], axis=[0, 0, 1], limited=False, range=[0, 0], ref=0.0,
                     springref=0.0, stiffness=0.0, armature=0.0, damping=0.0, margin=0.0,
                     solreflimit=[0.02, 1.0], solimplimit=[0.9, 0.95, 0.001, 0.5, 2.0])
GEOM_BUILTIN = dict(type="sphere", size=[0, 0, 0], pos=[0, 0, 0], quat=[1, 0, 0, 0], contype=1, conaffinity=1,
                    condim=3, friction=[1, 0.005, 0.0001], margin=0.0, gap=0.0, solref=[0.02, 1.0],
                    solimp=[0.9, 0.95, 0.001, 0.5, 2.0], solmix=1.0, density=1000.0)
MOTOR_BUILTIN = dict(gear=[1, 0, 0, 0, 0, 0], ctrlrange=[0, 0], forcerange=[0, 0], ctrllimited=False,
                     forcelimited=False)
TYPES = {"free": 0, "ball": 1, "slide": 2, "hinge": 3}


def strtod_list(s):
    out = []
    for tok in s.split():
        mm = _NUM.match(tok)
        if mm:
            out.append(float(mm.group(1)))
    return out


def _merge(builtin, dflt, elem):
    """builtin <- default class <- element; vectors overwrite a prefix only"""
    out = {k: (list(v) if isinstance(v, list) else v) for k, v in builtin.items()}
    for src in (dflt, elem):
        for k, v in src.items():
            if k not in out:
                continue
            cur = out[k]
            if isinstance(cur, list):
                vals = strtod_list(v)
                out[k] = vals + cur[len(vals):]
            elif isinstance(cur, bool):
                out[k] = v.strip() == "true"
            elif isinstance(cur, (int, float)) and not isinstance(cur, bool):
                vals = strtod_list(v)
                out[k] = type(cur)(vals[0]) if vals else cur
            else:
                out[k] = v.strip()
    return out


def qmul(a, b):
    return np.array([a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3],
                     a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2],
                     a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1],
                     a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0]])


def qconj(q):
    return np.array([q[0], -q[1], -q[2], -q[3]])


def qmat(q):
    w, x, y, z = q
    return np.array([[w * w + x * x - y * y - z * z, 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), w * w - x * x + y * y - z * z, 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), w * w - x * x - y * y + z * z]])


def z_to_vec(v):
    """minimal rotation taking +z onto v (MuJoCo's frame for fromto)"""
    v = np.asarray(v, float) / np.linalg.norm(v)
    z = np.array([0.0, 0.0, 1.0])
    c = float(np.dot(z, v))
    axis = np.cross(z, v)
    s = np.linalg.norm(axis)
    if s < 1e-15:
        return np.array([1.0, 0, 0, 0]) if c > 0 else np.array([0.0, 1, 0, 0])
    ang = math.atan2(s, c)
    axis /= s
    return np.concatenate([[math.cos(ang / 2)], math.sin(ang / 2) * axis])


def geom_mass_inertia(g):
    """solid of density g.density: sphere, capsule (cylinder + hemispheres, each
    hemisphere's centroid 3r/8 from its face, I_perp about the centroid 83/320 m r^2)"""
    rho, r = g["density"], g["size"][0]
    if g["type"] == "sphere":
        m = rho * 4.0 / 3.0 * math.pi * r ** 3
        return m, np.full(3, 0.4 * m * r * r)
    if g["type"] == "capsule":
        h = 2 * g["size"][1]
        mc = rho * math.pi * r * r * h
        ms = rho * 4.0 / 3.0 * math.pi * r ** 3
        hemi_perp = (ms / 2) * (83.0 / 320.0 * r * r + (h / 2 + 3 * r / 8) ** 2)
        ip = mc * (3 * r * r + h * h) / 12 + 2 * hemi_perp
        ia = mc * r * r / 2 + ms * 2 * r * r / 5
        return mc + ms, np.array([ip, ip, ia])
    return 0.0, np.zeros(3)


class Compiled:
    pass


def compile_mjcf(path):
    root = ET.parse(path).getroot()
    comp = root.find("compiler")
    cattr = comp.attrib if comp is not None else {}
    degree = cattr.get("angle", "degree") == "degree"
    glob = cattr.get("coordinate", "local") == "global"
    ang = (math.pi / 180.0) if degree else 1.0
    dj, dg, dm = {}, {}, {}
    d = root.find("default")
    if d is not None:
        for c in d:
            {"joint": dj, "geom": dg, "motor": dm}.get(c.tag, {}).update(c.attrib)
    opt = root.find("option")
    oa = opt.attrib if opt is not None else {}
    M = Compiled()
    M.timestep = strtod_list(oa.get("timestep", "0.002"))[0]
    M.gravity = (strtod_list(oa.get("gravity", "0 0 -9.81")) + [0, 0, -9.81])[:3]
    M.integrator = {"Euler": 0, "RK4": 1}[oa.get("integrator", "Euler")]
    M.iterations = int(strtod_list(oa.get("iterations", "100"))[0])
    M.tolerance = strtod_list(oa.get("tolerance", "1e-8"))[0]
    bodies = [dict(name="world", parent=0, gpos=np.zeros(3), gquat=np.array([1.0, 0, 0, 0]))]
    joints, geoms = [], []

    def add_geom(e, b):
        g = _merge(GEOM_BUILTIN, dg, e.attrib)
        if "fromto" in e.attrib:
            f = np.array(strtod_list(e.attrib["fromto"]))
            pos, quat = 0.5 * (f[:3] + f[3:]), z_to_vec(f[3:] - f[:3])
            g["size"][1] = 0.5 * np.linalg.norm(f[3:] - f[:3])
        else:
            pos, quat = np.array(g["pos"], float), np.array(g["quat"], float)
            quat = quat / np.linalg.norm(quat)
        B = bodies[b]
        if glob or b == 0:  # world frame: to the body frame
            gpos, gq = (pos, quat) if glob else (pos, quat)
        else:
            gpos = B["gpos"] + qmat(B["gquat"]) @ pos
            gq = qmul(B["gquat"], quat)
        g.update(body=b, gpos=gpos, gquat=gq)
        g["mass"], g["inertia"] = geom_mass_inertia(g)
        geoms.append(g)

    def add_body(e, parent):
        a = e.attrib
        pos = np.array((strtod_list(a.get("pos", "0 0 0")) + [0, 0, 0])[:3])
        quat = np.array(strtod_list(a.get("quat", "1 0 0 0")), float)
        quat = quat / np.linalg.norm(quat)
        P = bodies[parent]
        if glob:
            gpos, gq = pos, quat
        else:
            gpos, gq = P["gpos"] + qmat(P["gquat"]) @ pos, qmul(P["gquat"], quat)
        b = len(bodies)
        bodies.append(dict(name=a.get("name", ""), parent=parent, gpos=gpos, gquat=gq))
        for c in e:
            if c.tag in ("joint", "freejoint"):
                free = c.tag == "freejoint" or c.attrib.get("type") == "free"
                j = _merge(JOINT_BUILTIN, {} if free else dj, c.attrib)
                j["type"] = "free" if free else j["type"]
                jp, ja = np.array(j["pos"], float), np.array(j["axis"], float)
                R = qmat(gq)
                if free:
                    j["gpos"], j["gaxis"] = gpos.copy(), np.array([0.0, 0, 1])
                elif glob:
                    j["gpos"], j["gaxis"] = jp, ja / np.linalg.norm(ja)
                else:
                    j["gpos"], j["gaxis"] = gpos + R @ jp, R @ (ja / np.linalg.norm(ja))
                j["body"] = b
                j["name"] = c.attrib.get("name", "")
                if free:
                    j.update(limited=False, armature=0.0, damping=0.0, stiffness=0.0)
                joints.append(j)
        for c in e:
            if c.tag == "geom":
                add_geom(c, b)
        for c in e:
            if c.tag == "body":
                add_body(c, b)

    wb = root.find("worldbody")
    for c in wb:
        if c.tag == "geom":
            add_geom(c, 0)
    for c in wb:
        if c.tag == "body":
            add_body(c, 0)
    M.bodies, M.joints, M.geoms = bodies, joints, geoms
    nb = len(bodies)
    # dofs, qpos0
    qpos0, dof_joint, dof_body = [], [], []
    for ji, j in enumerate(joints):
        t = j["type"]
        if t == "free":
            qpos0 += list(bodies[j["body"]]["gpos"]) + list(bodies[j["body"]]["gquat"])
            nd = 6
        elif t == "ball":
            qpos0 += [1.0, 0, 0, 0]
            nd = 3
        else:
            qpos0.append(j["ref"] * (ang if t == "hinge" else 1.0))
            nd = 1
        dof_joint += [ji] * nd
        dof_body += [j["body"]] * nd
        if t in ("hinge", "ball"):
            j["range"] = [x * ang for x in j["range"]]
    M.qpos0 = np.array(qpos0)
    M.nq, M.nv, M.nbody, M.njnt, M.ngeom = len(qpos0), len(dof_joint), nb, len(joints), len(geoms)
    M.dof_joint, M.dof_body = dof_joint, dof_body
    # body mass / COM / inertia (world frame at qpos0) from geoms
    M.body_mass = np.zeros(nb)
    M.body_com = np.zeros((nb, 3))
    M.body_I = np.zeros((nb, 3, 3))
    for b in range(1, nb):
        gs = [g for g in geoms if g["body"] == b]
        m = sum(g["mass"] for g in gs)
        M.body_mass[b] = m
        if m <= 0:
            M.body_com[b] = bodies[b]["gpos"]
            continue
        com = sum(g["mass"] * g["gpos"] for g in gs) / m
        I = np.zeros((3, 3))
        for g in gs:
            R = qmat(g["gquat"])
            dd = g["gpos"] - com
            I += R @ np.diag(g["inertia"]) @ R.T + g["mass"] * (dd @ dd * np.eye(3) - np.outer(dd, dd))
        M.body_com[b], M.body_I[b] = com, I
    # actuators
    M.act = []
    act = root.find("actuator")
    jidx = {j["name"]: i for i, j in enumerate(joints)}
    if act is not None:
        for c in act:
            a = _merge(MOTOR_BUILTIN, dm, c.attrib)
            a["joint"] = jidx[c.attrib["joint"]]
            M.act.append(a)
    _set_const(M)
    return M


def _set_const(M):
    """M(qpos0) = sum_b m_b Jp'Jp + Jr' I_b Jr (+ armature), from the body COM
    Jacobians; dof_invweight0, body_invweight0, stat_meaninertia"""
    nb, nv = M.nbody, M.nv
    dof_axes = []  # per dof: (kind, world axis, anchor, body)
    for ji, j in enumerate(M.joints):
        b = j["body"]
        if j["type"] == "free":
            R = qmat(M.bodies[b]["gquat"])
            for k in range(3):
                dof_axes.append(("slide", np.eye(3)[k], None, b))
            for k in range(3):
                dof_axes.append(("hinge", R[:, k], M.bodies[b]["gpos"], b))
        elif j["type"] == "ball":
            R = qmat(M.bodies[b]["gquat"])
            for k in range(3):
                dof_axes.append(("hinge", R[:, k], j["gpos"], b))
        else:
            dof_axes.append((j["type"], j["gaxis"], j["gpos"], b))

    def ancestors(b):
        out = set()
        while b:
            out.add(b)
            b = M.bodies[b]["parent"]
        return out

    def jac(b, point):
        Jp, Jr = np.zeros((3, nv)), np.zeros((3, nv))
        anc = ancestors(b)
        for i, (kind, ax, anc_pt, db) in enumerate(dof_axes):
            if db not in anc:
                continue
            if kind == "slide":
                Jp[:, i] = ax
            else:
                Jr[:, i] = ax
                Jp[:, i] = np.cross(ax, point - anc_pt)
        return Jp, Jr

    Mm = np.zeros((nv, nv))
    M.body_jac = {}
    for b in range(1, nb):
        Jp, Jr = jac(b, M.body_com[b])
        M.body_jac[b] = (Jp, Jr)
        Mm += M.body_mass[b] * Jp.T @ Jp + Jr.T @ M.body_I[b] @ Jr
    for i in range(nv):
        Mm[i, i] += M.joints[M.dof_joint[i]]["armature"]
    M.Mq0 = Mm
    Minv = np.linalg.inv(Mm)
    M.dof_invweight0 = np.diag(Minv).copy()
    M.stat_meaninertia = np.trace(Mm) / nv
    M.body_invweight0 = np.zeros((nb, 2))
    for b in range(1, nb):
        Jp, Jr = M.body_jac[b]
        if not np.any(Jp) and not np.any(Jr):
            continue
        tran = np.mean(np.diag(Jp @ Minv @ Jp.T))
        rot = np.mean(np.diag(Jr @ Minv @ Jr.T))
        if tran < 1e-15 and rot > 1e-15:
            tran = rot
        if rot < 1e-15:
            rot = tran
        M.body_invweight0[b] = tran, rot
    M.body_subtreemass = M.body_mass.copy()
    for b in range(nb - 1, 0, -1):
        M.body_subtreemass[M.bodies[b]["parent"]] += M.body_subtreemass[b]
