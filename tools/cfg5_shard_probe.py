"""cfg 5 point sharding: one rank's critical path, replayed exactly on one GPU.

BASELINE.json configs[4] runs one humanoid seed (H = 200, fp32 FD, fp64 MFMA
recursion) on 8 GPUs.  Under `bench.py --workload humanoid_cfg5 --gpus N`
every rank runs ilqg_forward_sharded(rank, N) (the whole pipelined rollout,
the FD sweep of its own points behind each chunk), one RCCL all-gather of the
fp64 records, then the recursion.  The 8-GPU run is the driver's to launch;
this probe replays, on one GPU, exactly what rank r executes in each of the
bench's iterations, all-gather excepted:

  * a reference solver runs the bench's sequence (1 warm-up + STEPS
    iterations, plain ilqg_iterate) and keeps, per iteration k, the state it
    starts from (trajectory, gains) and the FD records it computes;
  * the probe solver is set to iteration k's starting state with the records
    of iteration k already in its buffer -- the other ranks' share, as the
    all-gather would leave them -- and forward_sharded(r, N) + riccati_pass()
    are timed (host-synchronised around the two calls);
  * its gains then must equal the reference's bit for bit (they do: every
    record is the same, the owned ones recomputed).

The all-gather itself (3.4 MB over xGMI) is not measured here.

  python3 tools/cfg5_shard_probe.py [world ...]    (default: 1 8)
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

H, WARM, STEPS = 200, 1, 5
worlds = [int(w) for w in sys.argv[1:]] or [1, 8]
torch.cuda.is_available()
m = ia.Model.load(workloads.model_file("humanoid"))
st = m.reset_state(1)
st.qpos[0, 2] = 1.4


def solver():
    g = ia.ILQR(m, st, H, ia.HUMANOID_COST)
    g.set_riccati("mfma")
    g.set_fd_precision("f32")
    return g


# the bench's sequence on a reference solver: per timed iteration, its start and its records
ref = solver()
for _ in range(WARM):
    ref.iterate()
seq = []
for _ in range(STEPS):
    ref.synchronize()
    start = (ref.traj(), ref.gains())
    ref.iterate()
    ref.synchronize()
    seq.append((start, ref.deriv(), ref.gains()))
for world in worlds:
    for rank in sorted({0, world - 1}):
        g = solver()
        g.set_timing(True)
        g.timing()
        tot = 0.0
        for (traj0, gains0), deriv, gains1 in seq:
            g.set_traj(traj0)
            g.set_gains(*gains0)
            g.set_deriv(deriv)
            g.synchronize()
            t0 = time.perf_counter()
            if world == 1:
                g.iterate()
            else:
                g.forward_sharded(rank, world)
                g.riccati_pass()
            g.synchronize()
            tot += time.perf_counter() - t0
            K, k = g.gains()
            assert np.array_equal(K, gains1[0]) and np.array_equal(k, gains1[1]), "replay differs from the reference"
        dt = tot / STEPS
        kt = {k_: {"avg_ms": round(v[0] / v[1], 3), "launches_per_it": v[1] / STEPS}
              for k_, v in g.timing().items() if v[1]}
        own = int((g.point_owners(world) == rank).sum()) if world > 1 else H + 1
        print(json.dumps({"world": world, "rank": rank, "points_owned": own, "ms_per_iter": round(dt * 1e3, 3),
                          "it_per_s": round(1 / dt, 3), "kernels": kt, "gains_equal_reference": True}), flush=True)
        del g
