"""How often each seed's selected line-search candidate repeats from one
iteration to the next on the bench workload (hopper H=500, 8 seeds x 8
alphas, min-cost): the hit rate of a 'same alpha as last time' predictor."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ilqg-mujoco_amd"))
import ilqg_amd as ia  # noqa: E402
import workloads  # noqa: E402

m = ia.Model.load(workloads.model_file("hopper"))
S, iters = 8, int(sys.argv[1]) if len(sys.argv) > 1 else 12
g = ia.ILQR(m, workloads.hopper_dmain(m, S, sigma=0.01), 500, ia.HOPPER_COST,
            alphas=workloads.LINESEARCH_ALPHAS, select="min_cost")
sels, costs = [], []
for _ in range(iters):
    g.iterate()
    c, sel = g.costs()
    sels.append(sel.copy())
    costs.append(c[np.arange(S), sel])
sels = np.array(sels)
print("selected alpha index per iteration (rows) and seed (columns):")
print(sels)
hits = (sels[1:] == sels[:-1]).mean()
print(f"repeat rate {hits:.2f}; selected costs by iteration (seed 0): {np.round(np.array(costs)[:, 0], 2)}")
