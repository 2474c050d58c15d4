"""Seed sharding and the one exchange step of the multi-GPU design.

Independent MPC seeds shard across ranks (one process per GPU): rank r owns
global seeds [r*S, (r+1)*S).  Per iteration the only collective is an
all-gather of every seed's selected-candidate trajectory cost (fp64), followed
by an argmin on every rank, and (MPC) a broadcast of the winning seed's first
control from the rank that owns it.  The reference has no multi-seed notion;
this is the north star's "RCCL all-gather of per-seed costs over xGMI".

Stream ordering is part of the API: with the "nccl" backend (RCCL on ROCm) a
collective runs on torch's current stream, while the solver launches on its
own stream (or the one given to ILQR.set_stream).  CostExchange, given the
solver, makes torch's current stream wait on the solver's launch stream before
every gather, so the costs it reads are the ones the last iterate() wrote --
whichever stream the solver runs on.  No host round trip is involved.
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
    """all-gather the per-seed costs of every rank; return the global best seed index.

    solver: the ILQR whose device costs `local` views; its launch stream is
    waited on before every gather (see the module docstring)."""

    def __init__(self, local: torch.Tensor, world: int, group=None, solver=None):
        self.local = local
        self.world = world
        self.group = group
        self.solver = solver
        self.glob = torch.empty(local.numel() * world, dtype=local.dtype, device=local.device)

    def _order_after_solver(self):
        if self.solver is not None and self.local.is_cuda:
            cur = torch.cuda.current_stream(self.local.device)
            sst = self.solver.stream
            if sst and sst != cur.cuda_stream:
                cur.wait_stream(torch.cuda.ExternalStream(sst, device=self.local.device))

    def gather(self) -> torch.Tensor:
        self._order_after_solver()
        if self.world > 1:
            dist.all_gather_into_tensor(self.glob, self.local, group=self.group)
            return self.glob
        return self.local

    def __call__(self) -> torch.Tensor:
        return torch.argmin(self.gather())


def broadcast_winner_control(best: int, ctrl_first: torch.Tensor, seeds_per_rank: int, world: int,
                             group=None) -> torch.Tensor:
    """The optional MPC step of SURVEY.md §8e: the rank owning global seed
    `best` broadcasts that seed's first control (nu doubles) to every rank.
    ctrl_first: this rank's [seeds_per_rank, nu] first controls (on the GPU, a
    view of the resident trajectory at point N).  Returns the winner's control."""
    # owner: the rank within `group` (the all-gather concatenates in group-rank order)
    owner, local = divmod(int(best), seeds_per_rank)
    out = ctrl_first[local].clone() if owner == (dist.get_rank(group) if world > 1 else 0) else \
        torch.empty(ctrl_first.shape[1], dtype=ctrl_first.dtype, device=ctrl_first.device)
    if world > 1:
        # dist.broadcast takes a global rank
        src = owner if group is None else dist.get_global_rank(group, owner)
        dist.broadcast(out, src=src, group=group)
    return out


def first_controls_view(solver, nu: int) -> torch.Tensor:
    """[S, nu] zero-copy view of every seed's first control u*_N in the solver's
    resident trajectory ([S][N+1][nu], point N = the initial state, inc/ilqr.h:52)."""
    S, P = solver.S, solver.P
    full = device_view(solver.device_traj_ptr("ctrl"), S * P * nu).view(S, P, nu)
    return full[:, P - 1, :]


def max_over_ranks(x: float, world: int, device) -> float:
    """The bench's timing rule: the slowest rank defines the step time."""
    t = torch.tensor([x], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
