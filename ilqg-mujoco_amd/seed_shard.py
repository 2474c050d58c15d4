"""Seed sharding and the one exchange step of the multi-GPU design.

Independent MPC seeds shard across ranks (one process per GPU): rank r owns
global seeds [r*S, (r+1)*S).  Per iteration the only collective is an
all-gather of every seed's selected-candidate trajectory cost (fp64), followed
by an argmin on every rank.  The reference has no multi-seed notion; this is
the north star's "RCCL all-gather of per-seed costs over xGMI".  With the
"nccl" backend (RCCL on ROCm) the gather runs on torch's current stream,
which is also the solver's launch stream, so no host round trip is needed.
"""
import torch
import torch.distributed as dist


def seed_offset(rank: int, seeds_per_rank: int) -> int:
    """First global seed index owned by `rank`."""
    return rank * seeds_per_rank


def device_view(ptr: int, n: int) -> torch.Tensor:
    """Zero-copy fp64 tensor over n doubles of device memory owned by the solver."""
    class _Arr:
        __cuda_array_interface__ = {"shape": (n,), "typestr": "<f8", "data": (ptr, False), "version": 3}
    return torch.as_tensor(_Arr(), device="cuda")


class CostExchange:
    """all-gather the per-seed costs of every rank; return the global best seed index."""

    def __init__(self, local: torch.Tensor, world: int, group=None):
        self.local = local
        self.world = world
        self.group = group
        self.glob = torch.empty(local.numel() * world, dtype=local.dtype, device=local.device)

    def gather(self) -> torch.Tensor:
        if self.world > 1:
            dist.all_gather_into_tensor(self.glob, self.local, group=self.group)
            return self.glob
        return self.local

    def __call__(self) -> torch.Tensor:
        return torch.argmin(self.gather())


def max_over_ranks(x: float, world: int, device) -> float:
    """The bench's timing rule: the slowest rank defines the step time."""
    t = torch.tensor([x], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
