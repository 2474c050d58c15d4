"""Seed-group pipeline probe: seed-iterations/s of the bench workload for
several (ngroups, roll_cus) settings, and bit-identity of the trajectories and
gains against ngroups = 1."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ilqg-mujoco_amd"))
import ilqg_amd as ia, workloads

S, A, H = 8, 8, 500
m = ia.Model.load(workloads.model_file("hopper"))
alphas = tuple(2.0 ** -i for i in range(A))
ref = None
configs = [(1, 0), (2, 0), (2, 64), (2, 96), (4, 64), (4, 128), (2, 128)]
if len(sys.argv) > 1:
    configs = [tuple(int(x) for x in c.split(",")) for c in sys.argv[1:]]
for G, cus in configs:
    dmain = workloads.hopper_dmain(m, S, sigma=0.01, seed_offset=0)
    g = ia.ILQR(m, dmain, H, ia.HOPPER_COST, alphas=alphas, select="min_cost")
    g.set_groups(G, cus)
    g.iterate(); g.iterate(); g.synchronize()
    K = 20
    g.set_timing(True); g.timing()
    t = time.perf_counter()
    for _ in range(K):
        g.iterate()
    g.synchronize()
    dt = time.perf_counter() - t
    tm = g.timing()
    kt = {k: round(v[0] / v[1], 2) for k, v in tm.items() if v[1]}
    K_, k_ = g.gains()
    tr = g.traj()
    sig = (K_, k_, tr.qpos, tr.qvel)
    same = "ref" if ref is None else all(np.array_equal(a, b) for a, b in zip(sig, ref))
    if ref is None:
        ref = sig
    print(f"groups={G} roll_cus={cus}: {S * K / dt:7.1f} seed-it/s  ({dt / K * 1e3:6.2f} ms/it)  bitexact={same} avg ms {kt}",
          flush=True)
