"""Probe: per-kernel times of the bench workload's pieces (HIP events):
fused FD sweep alone, standalone backward pass, and the fused sweep with the
backward pass streamed behind it (iterate).  ILQG_FUSED=0 selects the
two-kernel sweep.   python tools/fd_probe.py [label]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ilqg-mujoco_amd"))
import ilqg_amd as ia  # noqa: E402
import workloads  # noqa: E402

S, A, H, K = 8, 8, 500, 4
m = ia.Model.load(workloads.model_file("hopper"))
d = workloads.hopper_dmain(m, S, sigma=0.01)
g = ia.ILQR(m, d, H, ia.HOPPER_COST, alphas=tuple(2.0 ** -i for i in range(A)), select="min_cost")
g.iterate()
g.synchronize()
g.set_timing(True)
g.timing()
for _ in range(K):
    g.fd_sweep()
    g.backward_pass()
g.synchronize()
t1 = g.timing()
for _ in range(K):
    g.iterate()
g.synchronize()
t2 = g.timing()
f = lambda t, k: t[k][0] / max(1, t[k][1])  # noqa: E731
label = sys.argv[1] if len(sys.argv) > 1 else ""
print(f"{label} sweep alone {f(t1, 'fd_cols') + f(t1, 'fd_centre'):.2f} ms, backward alone {f(t1, 'backward'):.2f} ms, "
      f"rollout {f(t2, 'rollout'):.2f} ms, fused sweep+backward {f(t2, 'fd_backward'):.2f} ms", flush=True)
