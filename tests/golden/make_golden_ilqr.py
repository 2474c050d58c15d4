"""Generate the iLQR known-answer fixtures of SURVEY.md §8c items 2-4:

  riccati_{pendulum,hopper}.npz   seeded synthetic FD records + trajectory ->
                                  initV + the Riccati recursion (inc/ilqr.h:100-107,
                                  :144-175): K, k and the final V, v
  iterate_pendulum_H{20,100}.npz  ILQR::iterate() x iters from the reference's
                                  initial state (src/inverted_pendulum/inverted_pendulum.cpp:12-13),
                                  K/k zero-initialised (inc/ilqr.h:75-80): trajectory,
                                  gains, value and the last FD records
  rollout_hopper_H100.npz         forwardPass (inc/ilqr.h:116-130) with fixed seeded
                                  gains from the cfg-3 hopper state: the trajectory

The iterate fixtures run the REFERENCE's own calcMJDerivatives (oracle/_ref,
src/mjderivative.cpp compiled unmodified) inside the oracle's ilqr.h
restatement, so they need /root/reference (build container only):
    python tests/golden/make_golden_ilqr.py
The Riccati and rollout fixtures come from the oracle restatement alone.  A
fixture is data only: inputs and expected outputs.
"""
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "ilqg-mujoco_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import ilqg_amd as ia  # noqa: E402  (host-only model compile)
import oracle as ora  # noqa: E402

MODELS = os.path.join(ROOT, "ilqg-mujoco_amd", "models")
_dp = ctypes.POINTER(ctypes.c_double)


def _p(a):
    return a.ctypes.data_as(_dp)


def riccati_reference(om, traj, deriv, mu=1000.0):
    """initV at point 0 then ora_riccati_step_c for n = 1..N with
    c = x*_{n-1} - x*_n (ilqr.h:100-107,144-175), exactly as ora_ilqr_backwardPass."""
    L = om.lib.L
    L.ora_state_diff.argtypes = [ctypes.c_void_p] + [_dp] * 5
    L.ora_riccati_step_c.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_double] + [_dp] * 6
    nv, nu, P = om.nv, om.nu, deriv.shape[0]
    nx = 2 * nv
    q0 = deriv[0, 2 * nv * nv + nv * nu: 2 * nv * nv + nv * nu + nx]
    v = q0.copy()
    V = np.zeros(nx * nx)
    for j in range(nx):
        for i in range(nx):
            V[i + j * nx] = v[i] * v[j]
    K = np.zeros((P, nu * nx))
    k = np.zeros((P, nu))
    for n in range(1, P):
        c = np.zeros(nx)
        L.ora_state_diff(om.m, _p(np.ascontiguousarray(traj["qpos"][n - 1])), _p(np.ascontiguousarray(traj["qvel"][n - 1])),
                         _p(np.ascontiguousarray(traj["qpos"][n])), _p(np.ascontiguousarray(traj["qvel"][n])), _p(c))
        Kn = np.zeros(nu * nx)
        kn = np.zeros(nu)
        L.ora_riccati_step_c(nv, nu, om.timestep, mu, _p(np.ascontiguousarray(deriv[n])), _p(c), _p(V), _p(v),
                             _p(Kn), _p(kn))
        K[n], k[n] = Kn, kn
    return dict(K=K, k=k, V=V, v=v)


def make_riccati(mname, P, seed):
    m = ia.Model.load(os.path.join(MODELS, mname + ".xml"))
    om = ora.OModel(m.blob())
    rng = np.random.default_rng(seed)
    nq, nv, nu = m.nq, m.nv, m.nu
    D = om.D
    # FD-record-shaped synthetic data: dynamics Jacobians O(1..10), cost gradients O(1)
    deriv = np.concatenate([rng.normal(0, 3.0, (P, 2 * nv * nv + nv * nu)),
                            rng.normal(0, 1.0, (P, 2 * nv + nu))], axis=1)
    assert deriv.shape == (P, D)
    traj = dict(time=np.arange(P) * m.timestep, qpos=rng.normal(0, 0.3, (P, nq)), qvel=rng.normal(0, 1.0, (P, nv)),
                warm=rng.normal(0, 1.0, (P, nv)), ctrl=rng.normal(0, 0.5, (P, nu)))
    out = riccati_reference(om, traj, deriv)
    return dict(model=np.array(mname), deriv=deriv, **{"traj_" + k: v for k, v in traj.items()}, **out)


def dmain_state(om, nstep, ctrl_shift=0.0):
    """the configs' initial state on the oracle: reset, nstep passive steps, ctrl += shift"""
    d = om.make_data()
    d.step(nstep)
    d.arr("ctrl")[:] += ctrl_shift
    s = d.state()
    return d, {k: np.atleast_1d(np.asarray(v, dtype=np.float64))[None] if k != "time" else np.array([v])
               for k, v in s.items()}


def make_iterate(H, iters):
    m = ia.Model.load(os.path.join(MODELS, "inverted_pendulum.xml"))
    rm = ora.OModel(m.blob(), ora.ref_lib())
    d, dm = dmain_state(rm, 10)  # src/inverted_pendulum/inverted_pendulum.cpp:12-13
    il = ora.OILQR(rm, d, H, cost_fn="ora_cost_pendulum", use_ref_fd=True)
    il.set_dinit(d)
    for _ in range(iters):
        il.iterate()
    t, a = il.traj(), il.arrays()
    return dict(model=np.array("inverted_pendulum"), horizon=np.array(H), iters=np.array(iters),
                **{"dmain_" + k: v for k, v in dm.items()},
                **{"traj_" + k: v for k, v in t.items()}, K=a["K"], k=a["k"], V=a["V"], v=a["v"], deriv=a["deriv"])


def make_rollout(H, seed):
    m = ia.Model.load(os.path.join(MODELS, "hopper.xml"))
    om = ora.OModel(m.blob())
    om.lib.L.ora_set_cost_desc(ora.CostDesc.from_cost(ia.HOPPER_COST, m.nq, m.nv, m.nu))
    d, dm = dmain_state(om, 500, -0.1)  # tst/test_derivatives.cpp:38-47
    il = ora.OILQR(om, d, H, cost_fn="ora_cost_desc_fn")
    il.set_dinit(d)
    rng = np.random.default_rng(seed)
    nx = 2 * m.nv
    K = rng.normal(0, 0.05, (H + 1, m.nu * nx))
    k = rng.normal(0, 0.02, (H + 1, m.nu))
    nominal = il.traj()
    il.set_gains(K, k)
    il.forward_pass()
    t = il.traj()
    return dict(model=np.array("hopper"), horizon=np.array(H), K=K, k=k, **{"dmain_" + k_: v for k_, v in dm.items()},
                **{"nominal_" + k_: v for k_, v in nominal.items()}, **{"traj_" + k_: v for k_, v in t.items()})


def main():
    ora.build(ref=True)
    specs = {
        "riccati_pendulum.npz": lambda: make_riccati("inverted_pendulum", 40, 101),
        "riccati_hopper.npz": lambda: make_riccati("hopper", 40, 102),
        "rollout_hopper_H100.npz": lambda: make_rollout(100, 103),
    }
    if os.path.exists("/root/reference/src/mjderivative.cpp"):
        specs["iterate_pendulum_H20.npz"] = lambda: make_iterate(20, 3)
        specs["iterate_pendulum_H100.npz"] = lambda: make_iterate(100, 2)
    else:
        print("no /root/reference: iterate fixtures (reference FD driver) skipped")
    for fname, fn in specs.items():
        out = fn()
        np.savez_compressed(os.path.join(HERE, fname), **out)
        print(fname, {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
