"""Algorithmic fp64 operation counts of the hot path (SURVEY.md §8d
"Algorithmic flops"), from the instrumented build of the CPU restatement
(oracle/flops: mjtNum counts every add/sub, mul, div, sqrt it takes part in):

    make -C oracle flops && python tests/fixtures/make_flops.py

writes tests/fixtures/flops.json.  Per model, at fixture states:
  stage_flops   F_pos / F_vel / F_acc of one evaluation with the FD solver
                settings (iterations 30, tolerance 0; mjderivative.cpp:241-242):
                forwardSkip(NONE) - forwardSkip(POS), forwardSkip(POS) -
                forwardSkip(VEL), forwardSkip(VEL)
  fd_point      one calcMJDerivatives call (mjderivative.cpp:212-255, restated
                driver, 1 thread: centre + warm-ups + 2(2nv+nu) columns)
  step          one mj_step with the model's own settings (the rollout's unit)
  riccati_step  one backward-pass step (ilqr.h:144-175) on synthetic inputs
flops = add + mul + div + sqrt; comparisons and transcendental calls
(sin/cos/atan2, fdlibm kernels) are reported beside them, not in flops.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "ilqg-mujoco_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import ctypes  # noqa: E402

import ilqg_amd as ia  # noqa: E402  (host-only model compile)
import oracle as ora  # noqa: E402

FLOPS_SO = os.path.join(ROOT, "oracle", "flops", "liboracle_flops.so")
GOLDEN = os.path.join(ROOT, "tests", "golden")
MODELS = os.path.join(ROOT, "ilqg-mujoco_amd", "models")
KEYS = ("add", "mul", "div", "sqrt", "cmp", "trans")


class Counter:
    def __init__(self, lib):
        self.L = lib.L
        self.L.ora_flops_get.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]

    def __call__(self, fn):
        self.L.ora_flops_reset()
        fn()
        c = (ctypes.c_ulonglong * 6)()
        self.L.ora_flops_get(c)
        d = dict(zip(KEYS, (int(x) for x in c)))
        d["flops"] = d["add"] + d["mul"] + d["div"] + d["sqrt"]
        return d


def mean(ds):
    return {k: float(np.mean([d[k] for d in ds])) for k in ds[0]}


def diff(a, b):
    return {k: a[k] - b[k] for k in a}


def states(name, m, om):
    if name == "inverted_pendulum":
        g = np.load(os.path.join(GOLDEN, "fd_pendulum.npz"))
        return [dict(time=g["time"][i], qpos=g["qpos"][i], qvel=g["qvel"][i], warm=g["warm"][i], ctrl=g["ctrl"][i])
                for i in range(len(g["time"]))]
    if name == "hopper":
        g = np.load(os.path.join(GOLDEN, "fd_hopper.npz"))
        return [dict(time=g["time"][i], qpos=g["qpos"][i], qvel=g["qvel"][i], warm=g["warm"][i], ctrl=g["ctrl"][i])
                for i in range(len(g["time"]))]
    # humanoid (cfg 5): qpos0, qvel 0, then points of its passive fall (contacts from ~step 60)
    d = om.make_data()
    out = []
    for n in (0, 40, 40, 40):
        d.step(n)
        out.append(d.state())
    return out


def count_model(name, cnt, lib):
    m = ia.Model.load(os.path.join(MODELS, name + ".xml"))
    om = ora.OModel(m.blob(), lib)
    cost = {"inverted_pendulum": None, "hopper": ia.HOPPER_COST,
            "humanoid": ia.Cost(wq=[1.0] * m.nq, wv=[0.1] * m.nv, wu=[0.01] * m.nu)}[name]
    cfn = "ora_cost_pendulum" if cost is None else "ora_cost_desc_fn"
    if cost is not None:
        lib.L.ora_set_cost_desc(ora.CostDesc.from_cost(cost, m.nq, m.nv, m.nu))
    own = _own_solver(om)  # the model's own solver settings, before any FD override
    sts = states(name, m, om)
    stage, fd, step = [], [], []
    for s in sts:
        d = om.make_data()

        def fwd(skip):
            d.set_state(**s)
            om.set_solver(30, 0.0)
            lib.L.mj_forwardSkip(om.m, d.d, skip, 0)

        full, skpos, skvel = cnt(lambda: fwd(0)), cnt(lambda: fwd(1)), cnt(lambda: fwd(2))
        om.set_solver(*own)
        stage.append({"pos": diff(full, skpos), "vel": diff(skpos, skvel), "acc": skvel})
        d.set_state(**s)
        fd.append(cnt(lambda: ora.calc_derivatives(om, d, cost_fn=cfn, nthread=1)))
        d.set_state(**s)
        step.append(cnt(lambda: d.step(1)))
    nv, nu = m.nv, m.nu
    rng = np.random.default_rng(0)
    D = om.D
    der = np.concatenate([rng.normal(0, 3.0, 2 * nv * nv + nv * nu), rng.normal(0, 1.0, 2 * nv + nu)])
    nx = 2 * nv
    c = rng.normal(0, 0.1, nx)
    v = rng.normal(0, 1.0, nx)
    V = np.outer(v, v).reshape(-1)
    K = np.zeros(nu * nx)
    k = np.zeros(nu)
    dp = ctypes.POINTER(ctypes.c_double)
    lib.L.ora_riccati_step_c.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_double] + [dp] * 6
    ric = cnt(lambda: lib.L.ora_riccati_step_c(nv, nu, om.timestep, 1000.0, *(a.ctypes.data_as(dp)
                                                                               for a in (der, c, V, v, K, k))))
    assert D == der.size
    return dict(nq=m.nq, nv=nv, nu=nu, points=len(sts),
                stage_flops={k: mean([x[k] for x in stage]) for k in ("pos", "vel", "acc")},
                fd_point=mean(fd), step=mean(step), riccati_step=ric)


def _own_solver(om):
    it = ctypes.c_int()
    tol = ctypes.c_double()
    om.lib.L.ora_get_solver(om.m, ctypes.byref(it), ctypes.byref(tol))
    return it.value, tol.value


def main():
    lib = ora.Lib(FLOPS_SO)
    cnt = Counter(lib)
    out = {"source": "oracle/flops (instrumented restatement), tests/fixtures/make_flops.py",
           "flops_definition": "fp64 add+sub, mul, div, sqrt; cmp and trans (sin/cos/atan2 calls) reported apart",
           "models": {}}
    for name in ("inverted_pendulum", "hopper", "humanoid"):
        out["models"][name] = count_model(name, cnt, lib)
        r = out["models"][name]
        print(name, "fd_point", round(r["fd_point"]["flops"]), "step", round(r["step"]["flops"]), "riccati",
              r["riccati_step"]["flops"])
    # per seed-iteration totals for the bench configs (P = H + 1 points, H Riccati steps, P rollout steps per candidate)
    cfg = {"cfg2_pendulum_H200": ("inverted_pendulum", 200, 1), "cfg3_hopper_H500_8alpha": ("hopper", 500, 8),
           "cfg5_humanoid_H200": ("humanoid", 200, 1)}
    out["per_seed_iteration"] = {}
    for k, (name, H, A) in cfg.items():
        r = out["models"][name]
        P = H + 1
        out["per_seed_iteration"][k] = dict(
            fd=P * r["fd_point"]["flops"], backward=H * r["riccati_step"]["flops"],
            forward=A * P * r["step"]["flops"], candidates=A)
    with open(os.path.join(HERE, "flops.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(json.dumps(out["per_seed_iteration"], indent=1))


if __name__ == "__main__":
    main()
