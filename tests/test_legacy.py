"""Legacy C++ boundary: include/legacy (mujoco.h subset,
mjderivative.h, util.h, update.h, differentiator.h, ilqr.h) over
libilqg_mujoco.so.

CPU: the library exports the reference's C++ symbols with the reference's
mangling and the MuJoCo C API subset; the reference's own controller
(src/inverted_pendulum/inverted_pendulum.cpp) compiles unmodified against the
headers and links (when /root/reference is present); without a GPU the path
fails loudly.
GPU: the headless cmd/basic.cpp loop (ilqg_headless, host-callback cost and
registered device cost) and the reference's controller linked against the
product reproduce the oracle's MPC loop bit for bit."""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, model_path

LIB = os.path.join(ROOT, "ilqg-mujoco_amd", "lib", "libilqg_mujoco.so")
HEADLESS = os.path.join(ROOT, "ilqg-mujoco_amd", "bin", "ilqg_headless")
REF_LOOP = os.path.join(ROOT, "oracle", "_ref", "ref_pendulum_legacy")
MEMBERS = os.path.join(ROOT, "ilqg-mujoco_amd", "bin", "legacy_members")

REF_SYMBOLS = [
    "_Z17calcMJDerivativesP8_mjModelP7_mjDataPdPFdPKS1_E",  # inc/mjderivative.h:7
    "_Z8cpMjDataPK8_mjModelP7_mjDataPKS2_",  # inc/util.h:6
    "_Z11forwardStepP8_mjModelP7_mjData",  # inc/update.h:6
    "_Z12forwardFrameP8_mjModelP7_mjData",  # inc/update.h:8
]
MJ_API = ["mj_activate", "mj_deactivate", "mj_loadXML", "mj_deleteModel", "mj_makeData", "mj_deleteData",
          "mj_resetData", "mj_stackAlloc", "mj_step", "mj_forward", "mj_forwardSkip", "mju_copy", "mju_zero",
          "mju_malloc", "mju_free", "mju_error", "mju_error_s", "mju_quatIntegrate"]


def _exports(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


def test_legacy_exports_reference_symbols():
    syms = _exports(LIB)
    for s in REF_SYMBOLS + MJ_API:
        assert s in syms, s


@pytest.mark.skipif(not os.path.isdir("/root/reference/src"), reason="/root/reference not present (GPU box)")
def test_reference_controller_compiles_against_legacy_headers():
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "legacy"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert os.path.exists(REF_LOOP)


def test_legacy_members_caller_compiles():
    """tests/legacy_members.cpp -- a caller touching every public type, member
    and method of Differentiator<nv,nu> and ILQR<nv,nu,N> that SURVEY.md §8b
    lists (inc/differentiator.h:14-93, inc/ilqr.h:19-186), and an ILQR
    subclass overriding the virtual initV -- compiles warning-free (-Wall
    -Wextra) against include/legacy and links against libilqg_mujoco.so"""
    src = os.path.join(ROOT, "tests", "legacy_members.cpp")
    pkg = os.path.join(ROOT, "ilqg-mujoco_amd")
    out = os.path.join(pkg, "build", "legacy_members_check")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Wextra", "-Werror",
                        "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "include", "legacy"),
                        "-o", out, src, "-L" + os.path.join(pkg, "lib"), "-lilqg_mujoco", "-lilqg_amd",
                        "-Wl,-rpath," + os.path.join(pkg, "lib")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    with open(src) as f:
        text = f.read()
    # every public member / method named in SURVEY.md §8b is touched
    for name in ("->m", "->d", "->deriv", "->dqaccdq", "->dqaccdqvel", "->dqaccdctrl", "->dgdx", "->dgdu",
                 "->x", "->u", "->A", "->B", "->stepCostFn", "setMJData", "updateDerivatives", "->differentiator",
                 "->dArray", "->V", "->v", "->K", "->xStar", "->uStar", "->mu", "initV", "setDInit",
                 "forwardPass", "backwardPass", "iterate"):
        assert name in text, name


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a GPU is visible")
def test_headless_fails_loudly_without_gpu():
    r = subprocess.run([HEADLESS, model_path("inverted_pendulum"), "1"], capture_output=True, text=True)
    assert r.returncode != 0 and "ERROR" in r.stderr


# ------------------------------------------------------------------ GPU
FRAMES = 3


def _parse(out):
    rows = []
    for line in out.splitlines():
        if line.startswith("frame "):
            rows.append([float.fromhex(x) for x in line.split()[2:]])
    return np.array(rows)


def _oracle_loop(ora, frames):
    """InvertedPendulum (src/inverted_pendulum/inverted_pendulum.cpp:7-30) on the oracle:
    10 passive steps, ILQR<2,1,20>; per frame setDInit, 10 iterate, first control, mj_step."""
    import ilqg_amd as ia
    m = ia.Model.load(model_path("inverted_pendulum"))
    om = ora.OModel(m.blob())
    d = om.make_data()
    d.step(10)
    il = ora.OILQR(om, d, 20, cost_fn="ora_cost_pendulum")

    def row():
        return [d.time] + list(d.arr("qpos")) + list(d.arr("qvel")) + list(d.arr("ctrl"))
    rows = [row()]
    for _ in range(frames):
        il.set_dinit(d)
        for _ in range(10):
            il.iterate()
        d.arr("ctrl")[:] = il.traj()["ctrl"][20]
        d.step(1)
        rows.append(row())
    return np.array(rows)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    return _parse(r.stdout)


@pytest.mark.gpu
@pytest.mark.parametrize("device_cost", [False, True])
def test_headless_loop_bitexact(ora, device_cost):
    cmd = [HEADLESS, model_path("inverted_pendulum"), str(FRAMES)] + (["--device-cost"] if device_cost else [])
    got = _run(cmd)
    ref = _oracle_loop(ora, FRAMES)
    assert got.shape == ref.shape
    assert np.array_equal(got, ref), np.abs(got - ref).max()


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(REF_LOOP), reason="oracle/_ref/ref_pendulum_legacy not built")
def test_reference_controller_on_gpu_bitexact(ora):
    got = _run([REF_LOOP, model_path("inverted_pendulum"), str(FRAMES)])
    ref = _oracle_loop(ora, FRAMES)
    assert np.array_equal(got, ref), np.abs(got - ref).max()


@pytest.mark.gpu
def test_legacy_members_semantics():
    """the public members keep the reference's meaning on the GPU path: x / u
    on d, xStar / uStar left on dArray[0] by forwardPass, d one step past the
    terminal point after the ctor, the differentiator left at dArray[N] with
    its A / B after backwardPass (inc/ilqr.h:82-93,121-129,153-154)"""
    r = subprocess.run([MEMBERS, model_path("inverted_pendulum"), "members"], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0 and "members ok" in r.stdout, r.stderr


def _hex_rows(out):
    rows = {}
    for line in out.splitlines():
        tag, *vals = line.split()
        rows.setdefault(tag, []).append([float.fromhex(x) for x in vals])
    return {k: np.array(v) for k, v in rows.items()}


@pytest.mark.gpu
@pytest.mark.parametrize("iters", [1, 2])
def test_initv_override_drives_recursion(ora, iters):
    """virtual initV (inc/ilqr.h:100,142): an ILQR subclass whose initV sets
    its own V0 / v0 gets the recursion started from them (uploaded through
    ilqg_solver_set_value) -- K, k, V, v and the trajectory bit-exact against
    the oracle's backwardPass seeded with the same V0 / v0"""
    import ilqg_amd as ia
    r = subprocess.run([MEMBERS, model_path("inverted_pendulum"), "initv", str(iters)], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    got = _hex_rows(r.stdout)
    m = ia.Model.load(model_path("inverted_pendulum"))
    om = ora.OModel(m.blob())
    d = om.make_data()
    d.step(10)
    il = ora.OILQR(om, d, 20, cost_fn="ora_cost_pendulum")
    il.set_dinit(d)
    nx = 4
    V0 = np.array([[(0.5 * (i + 1) if i == j else 0.0) + 0.125 * (i + j) for i in range(nx)] for j in range(nx)])
    v0 = np.arange(nx) - 1.5
    for _ in range(iters):
        il.iterate_v0(V0.ravel(), v0)  # V0 column-major: V0[j][i] = V(i, j)
    a, t = il.arrays(), il.traj()
    assert np.array_equal(got["K"], a["K"]) and np.array_equal(got["k"], a["k"])
    assert np.array_equal(got["V"][0], a["V"]) and np.array_equal(got["v"][0], a["v"])
    assert np.array_equal(got["qpos"], t["qpos"]) and np.array_equal(got["ctrl"], t["ctrl"])
    # and the override mattered: the default initV gives other gains
    il2 = ora.OILQR(om, d, 20, cost_fn="ora_cost_pendulum")
    il2.set_dinit(d)
    for _ in range(iters):
        il2.iterate()
    assert not np.array_equal(il2.arrays()["K"], a["K"])


@pytest.mark.gpu
def test_initv_override_changing_a_point(ora):
    """an initV override that changes a later point (dArray[N/2]->qvel[0] +=
    1e-3 after the default initV): the reference differentiates dArray[n]
    inside its loop, after initV (inc/ilqr.h:142-154), so the recursion sees
    the changed state -- the legacy backwardPass re-sweeps when an override
    changed the trajectory.  K, k, V, v and the trajectory bit-exact against
    the oracle's backwardPass run on the changed trajectory"""
    import ilqg_amd as ia
    r = subprocess.run([MEMBERS, model_path("inverted_pendulum"), "mutate"], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr
    got = _hex_rows(r.stdout)
    m = ia.Model.load(model_path("inverted_pendulum"))
    om = ora.OModel(m.blob())
    d = om.make_data()
    d.step(10)
    N = 20
    il = ora.OILQR(om, d, N, cost_fn="ora_cost_pendulum")
    il.set_dinit(d)
    il.forward_pass()  # iterate(): forwardPass; setDInit(dArray[N]); backwardPass
    il.set_dinit(il.point(N))
    il.point(N // 2).arr("qvel")[0] += 1e-3  # what the override does after the default initV
    il.backward_pass()
    a, t = il.arrays(), il.traj()
    assert np.array_equal(got["K"], a["K"]) and np.array_equal(got["k"], a["k"])
    assert np.array_equal(got["V"][0], a["V"]) and np.array_equal(got["v"][0], a["v"])
    assert np.array_equal(got["qvel"], t["qvel"]) and np.array_equal(got["ctrl"], t["ctrl"])


@pytest.mark.gpu
@pytest.mark.parametrize("iters", [1, 2])
def test_legacy_mu_is_live(ora, iters):
    """the public ILQR::mu (inc/ilqr.h:65) is read by every backward pass
    (inc/ilqr.h:166): a caller setting il.mu = 10 before iterate() gets the
    oracle's recursion at mu = 10 bit for bit, and mu = 1000 gives other gains"""
    import ilqg_amd as ia
    m = ia.Model.load(model_path("inverted_pendulum"))
    om = ora.OModel(m.blob())
    d = om.make_data()
    d.step(10)
    runs = {}
    for mu in (10.0, 1000.0):
        r = subprocess.run([MEMBERS, model_path("inverted_pendulum"), "mu", repr(mu), str(iters)], capture_output=True,
                           text=True, timeout=600)
        assert r.returncode == 0, r.stderr
        got = _hex_rows(r.stdout)
        il = ora.OILQR(om, d, 20, cost_fn="ora_cost_pendulum")
        il.set_mu(mu)
        il.set_dinit(d)
        for _ in range(iters):
            il.iterate()
        a, t = il.arrays(), il.traj()
        assert np.array_equal(got["K"], a["K"]) and np.array_equal(got["k"], a["k"]), mu
        assert np.array_equal(got["V"][0], a["V"]) and np.array_equal(got["v"][0], a["v"]), mu
        assert np.array_equal(got["qpos"], t["qpos"]) and np.array_equal(got["ctrl"], t["ctrl"]), mu
        runs[mu] = got
    assert not np.array_equal(runs[10.0]["K"], runs[1000.0]["K"])
