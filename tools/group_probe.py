"""Probe: the bench workload (hopper H=500, 8 seeds x 8 candidates) iterated as
G seed groups on their own streams (ilqg_solver_set_groups).  Prints ms per
iteration of all seeds and per-kernel HIP-event averages.
  python tools/group_probe.py [G ...]     (ILQG_GROUP_TOKEN=0 drops the sweep token)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ilqg-mujoco_amd"))
import ilqg_amd as ia  # noqa: E402
import workloads  # noqa: E402

S, A, H, K = 8, 8, 500, 8
m = ia.Model.load(workloads.model_file("hopper"))
d = workloads.hopper_dmain(m, S, sigma=0.01)
g = ia.ILQR(m, d, H, ia.HOPPER_COST, alphas=tuple(2.0 ** -i for i in range(A)), select="min_cost")
for G in [int(x) for x in sys.argv[1:]] or [1, 2, 4]:
    g.set_groups(G)
    for _ in range(2):
        g.iterate()
    g.synchronize()
    g.set_timing(True)
    g.timing()
    t0 = time.perf_counter()
    for _ in range(K):
        g.iterate()
    g.synchronize()
    el = time.perf_counter() - t0
    t = g.timing()
    g.set_timing(False)
    f = lambda k: t[k][0] / max(1, t[k][1])  # noqa: E731
    print(f"G={G} {os.environ.get('PROBE_LABEL', '')}: {el / K * 1e3:.2f} ms/iteration, "
          f"{S * K / el:.1f} seed-it/s; per launch: rollout {f('rollout'):.2f} ms, fd_backward {f('fd_backward'):.2f} ms, "
          f"sweep {f('fd_cols'):.2f} ms, backward {f('backward'):.2f} ms",
          flush=True)
