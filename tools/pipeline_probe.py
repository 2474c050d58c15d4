"""Probe: split the bench's 8 seeds into G solver groups on G streams and let
their iterate() chains overlap (rollout/backward latency of one group hidden
behind the FD throughput of another).  Prints ms per iteration of all seeds.
  python tools/pipeline_probe.py [G ...]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ilqg-mujoco_amd"))
import ilqg_amd as ia  # noqa: E402
import workloads  # noqa: E402

S, A, H, K = 8, 8, 500, 6
alphas = tuple(2.0 ** -i for i in range(A))
m = ia.Model.load(workloads.model_file("hopper"))
for G in [int(x) for x in sys.argv[1:]] or [1, 2, 4, 8]:
    sg = S // G
    sol = []
    for g in range(G):
        d = workloads.hopper_dmain(m, sg, sigma=0.01, seed_offset=g * sg)
        sol.append(ia.ILQR(m, d, H, ia.HOPPER_COST, alphas=alphas, select="min_cost"))
    for s in sol:
        s.iterate()
    for s in sol:
        s.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        for s in sol:
            s.iterate()
    for s in sol:
        s.synchronize()
    el = time.perf_counter() - t0
    print(f"G={G} ({sg} seeds/group, HWQ={os.environ.get('GPU_MAX_HW_QUEUES', 'default')}): "
          f"{el / K * 1e3:.2f} ms/iteration, {S * K / el:.1f} seed-it/s", flush=True)
    del sol
