"""Rollout kernel time vs number of concurrent workgroups (diagnostic)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ilqg-mujoco_amd"))
import ilqg_amd as ia, workloads
m = ia.Model.load(workloads.model_file("hopper"))
for S, A in ((1, 1), (8, 1), (8, 8), (32, 8)):
    dmain = workloads.hopper_dmain(m, S, sigma=0.01)
    g = ia.ILQR(m, dmain, 500, ia.HOPPER_COST, alphas=tuple(2.0 ** -i for i in range(A)), select="min_cost")
    g.iterate(); g.synchronize()
    g.set_timing(True); g.timing()
    for _ in range(3):
        g.forward_pass()
    g.synchronize()
    t = g.timing()
    print(f"S={S} A={A} blocks={S*A}: rollout {t['rollout'][0]/t['rollout'][1]:.2f} ms/launch", flush=True)
