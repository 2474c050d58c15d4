"""cfg 5 point sharding, one rank's critical path measured on one GPU.

BASELINE.json configs[4] runs one humanoid seed (H = 200, fp32 FD, fp64 MFMA
recursion) on 8 GPUs.  Under `bench.py --workload humanoid_cfg5 --gpus N`
every rank runs ilqg_forward_sharded(rank, N) (the whole pipelined rollout,
the FD sweep of its own points behind each chunk), one RCCL all-gather of the
fp64 records, then the recursion.  The 8-GPU run is the driver's to launch,
so this probe times, on one GPU, exactly what one rank executes per iteration
except the all-gather: forward_sharded(rank, world) + riccati_pass().

The records of the points the rank does not own must be the right ones for
the recursion's time to be representative, so every timed iteration rolls out
the SAME trajectory: the gains are zeroed before it (outside the timed region;
with K = 0, k = 0 the rollout u = u* reproduces the nominal trajectory bit
for bit, inc/ilqr.h:126), and a full iteration beforehand differentiated
every point of that trajectory.  world = 1 times ilqg_iterate the same way.
The all-gather (3.4 MB over xGMI) is not measured here.

  python3 tools/cfg5_shard_probe.py [world ...]    (default: 1 2 4 8)
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ilqg-mujoco_amd"))
import torch  # noqa: E402  (torch's HIP runtime first)
import ilqg_amd as ia  # noqa: E402
import workloads  # noqa: E402

H, STEPS = 200, 5
worlds = [int(w) for w in sys.argv[1:]] or [1, 2, 4, 8]
torch.cuda.is_available()
m = ia.Model.load(workloads.model_file("humanoid"))
st = m.reset_state(1)
st.qpos[0, 2] = 1.4
for world in worlds:
    for rank in sorted({0, world - 1}):
        g = ia.ILQR(m, st, H, ia.HUMANOID_COST)
        g.set_riccati("mfma")
        g.set_fd_precision("f32")
        g.iterate()  # a first update: the trajectory below is an iterate's, not the passive one
        g.synchronize()
        K, k = g.gains()
        Kz, kz = np.zeros_like(K), np.zeros_like(k)
        g.set_gains(Kz, kz)
        g.iterate()  # every point of the fixed trajectory differentiated
        g.synchronize()
        q0 = g.traj().qpos.copy()

        def one():
            if world == 1:
                g.iterate()
            else:
                g.forward_sharded(rank, world)
                g.riccati_pass()
        tot = 0.0
        g.set_timing(True)
        g.timing()
        for _ in range(STEPS):
            g.set_gains(Kz, kz)
            g.synchronize()
            t0 = time.perf_counter()
            one()
            g.synchronize()
            tot += time.perf_counter() - t0
        assert np.array_equal(g.traj().qpos, q0), "the fixed trajectory moved"
        dt = tot / STEPS
        kt = {k_: {"avg_ms": round(v[0] / v[1], 3), "launches_per_it": v[1] / STEPS}
              for k_, v in g.timing().items() if v[1]}
        own = int((g.point_owners(world) == rank).sum()) if world > 1 else H + 1
        print(json.dumps({"world": world, "rank": rank, "points_owned": own, "ms_per_iter": round(dt * 1e3, 3),
                          "it_per_s": round(1 / dt, 3), "kernels": kt}), flush=True)
        del g
