"""World-size-2 gloo tests of the multi-GPU host logic on CPU:
seed sharding, the per-iteration cost all-gather + argmin, and the bench's
max-over-ranks timing rule.  The GPU run uses the same code with "nccl"."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ilqg-mujoco_amd"))

WORLD, S = 2, 8


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _seed_costs(seeds):
    """a deterministic stand-in for per-seed trajectory costs"""
    import workloads
    return np.array([abs(workloads.normals(g, 12)).sum() for g in seeds])


def _worker(rank, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        import workloads
        from seed_shard import CostExchange, max_over_ranks, seed_offset
        off = seed_offset(rank, S)
        mine = list(range(off, off + S))
        local = torch.tensor(_seed_costs(mine), dtype=torch.float64)
        ex = CostExchange(local, WORLD)
        best = int(ex().item())
        gathered = ex.gather().numpy().copy()
        slowest = max_over_ranks(1.0 + rank, WORLD, "cpu")
        z = np.stack([workloads.normals(g, 12) for g in mine])
        np.savez(os.path.join(outdir, f"r{rank}.npz"), best=best, gathered=gathered, slowest=slowest, z=z)
    finally:
        dist.destroy_process_group()


def test_seed_shard_exchange_gloo(tmp_path):
    import workloads
    mp.spawn(_worker, args=(_free_port(), str(tmp_path)), nprocs=WORLD, join=True)
    r = [np.load(tmp_path / f"r{i}.npz") for i in range(WORLD)]
    allc = _seed_costs(range(WORLD * S))
    for x in r:
        # every rank sees every seed's cost in rank order and picks the same global best
        assert np.array_equal(x["gathered"], allc)
        assert int(x["best"]) == int(np.argmin(allc))
        assert float(x["slowest"]) == float(WORLD)
    # the shards are disjoint and their union is the single-process seed set
    z_all = np.stack([workloads.normals(g, 12) for g in range(WORLD * S)])
    assert np.array_equal(np.concatenate([x["z"] for x in r]), z_all)


def test_single_rank_exchange_is_local_argmin():
    from seed_shard import CostExchange
    c = torch.tensor([3.0, 1.0, 2.0], dtype=torch.float64)
    assert int(CostExchange(c, 1)().item()) == 1
