"""Step-by-step check of the fused sweep's ticket planner on the GPU, printing
as it goes (a fault shows how far it got): ILQG_PLAN=0 iterations, then one
identity-order sweep, the planner's schedule checked on the host (a
permutation, every column team after its centre team), then planned sweeps
compared bit for bit with the unplanned solver."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ilqg-mujoco_amd"))
import ilqg_amd as ia  # noqa: E402
import workloads  # noqa: E402


def check_order(order, S, P, ntm):
    n = S * P * (1 + ntm)
    assert order.size == n, (order.size, n)
    assert np.array_equal(np.sort(order), np.arange(n)), "not a permutation"
    pos = np.empty(n, dtype=np.int64)
    pos[order] = np.arange(n)
    nC = S * P
    cols = np.arange(nC, n)
    assert np.all(pos[(cols - nC) // ntm] < pos[cols]), "a column team before its centre"


def run(name, H, S, cost, iters):
    m = ia.Model.load(workloads.model_file(name))
    st = workloads.pendulum_dmain(m, S) if name == "inverted_pendulum" else workloads.hopper_dmain(m, S, sigma=0.01)
    ntm = min(m.nu, m.nv) + 2 * m.nv
    out = []
    for plan in ("0", "1"):
        os.environ["ILQG_PLAN"] = plan
        g = ia.ILQR(m, st, H, cost)
        g.iterate()
        g.synchronize()
        print(f"{name} S={S} H={H} ILQG_PLAN={plan}: first iterate ok", flush=True)
        if plan == "1":
            n = ctypes.c_int()
            ia._check(ia.lib().ilqg_solver_debug_plan(g._h, None, None, ctypes.byref(n)), "debug_plan")
            order = np.zeros(n.value, dtype=np.uint32)
            dur = np.zeros(n.value, dtype=np.uint32)
            ia._check(ia.lib().ilqg_solver_debug_plan(g._h, order.ctypes.data_as(ctypes.c_void_p),
                                                       dur.ctypes.data_as(ctypes.c_void_p), ctypes.byref(n)))
            print(f"  durations: {np.count_nonzero(dur)}/{dur.size} nonzero, mean {dur.mean() / 100:.1f} us, "
                  f"max {dur.max() / 100:.1f} us", flush=True)
            check_order(order.astype(np.int64), S, H + 1, ntm)
            print(f"  planned order valid; {np.count_nonzero(order != np.arange(order.size))} items moved", flush=True)
        for _ in range(iters - 1):
            g.iterate()
        g.synchronize()
        print(f"  {iters} iterations ok", flush=True)
        out.append((*g.gains(), *g.value(), g.deriv()))
    for a, b in zip(*out):
        assert np.array_equal(a, b), "planned sweep differs"
    print(f"{name}: planned == unplanned, bit for bit", flush=True)


run("inverted_pendulum", 20, 1, ia.PENDULUM_COST, 3)
run("hopper", 500, 8, ia.HOPPER_COST, 3)
