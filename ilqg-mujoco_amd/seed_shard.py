"""Seed sharding and the one exchange step of the multi-GPU design,
and point sharding of a single seed's FD sweep (cfg 5).

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

    def _solver_after_exchange(self):
        """the solver's next launches wait for the gather + argmin: its stream
        waits on torch's, and seed groups (whose streams otherwise wait on the
        solver's stream only for the solver's own work) join it, so the next
        rollout cannot overwrite the costs while the collective still reads them"""
        if self.solver is None or not self.local.is_cuda:
            return
        cur = torch.cuda.current_stream(self.local.device)
        sst = self.solver.stream
        if sst and sst != cur.cuda_stream:
            torch.cuda.ExternalStream(sst, device=self.local.device).wait_stream(cur)
        self.solver.join_stream()

    def __call__(self) -> torch.Tensor:
        best = torch.argmin(self.gather())
        self._solver_after_exchange()
        return best


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


# ---- point sharding of one seed's FD sweep (cfg 5: one humanoid seed on 8 GPUs)
# The FD sweep is independent across the N+1 trajectory points
# (src/mjderivative.cpp:212-255 runs once per point, inc/ilqr.h:153-154).  Every
# rank runs the (serial, deterministic) rollout itself, differentiates the
# points it owns, and one all-gather of the fp64 records gives every rank all
# of them; every rank then runs the recursion (identical inputs, identical
# K / k: no broadcast).  Ownership on the GPU follows the pipelined rollout
# (ilqg_point_owners: chunks dealt round-robin, the last chunks' points split
# over every rank, so each rank differentiates behind the rollout); the
# default for other callers is contiguous blocks (point_range).  Exchange per
# iteration: world x S x max-owned x Dp doubles (humanoid H = 200, 8 ranks:
# about 3.4 MB).

def point_range(rank: int, world: int, P: int):
    """(p0, np) of the contiguous block of points `rank` differentiates: blocks
    of ceil(P / world) points, the last ones shorter (possibly empty)."""
    chunk = -(-P // world)
    p0 = min(P, rank * chunk)
    return p0, min(P, p0 + chunk) - p0


def block_owners(world: int, P: int):
    """owner rank of every point under point_range's contiguous blocks"""
    import numpy as np
    own = np.zeros(P, dtype=np.int32)
    for r in range(world):
        p0, n = point_range(r, world, P)
        own[p0:p0 + n] = r
    return own


class RecordExchange:
    """all-gather every rank's FD records so that every rank holds the records
    of all points.

    records: the [S, P, stride] fp64 record array (on the GPU, a zero-copy view
    of the solver's resident records, ilqg_solver_device_deriv; on CPU any
    tensor -- the gloo tests); rank / world / group: the point-sharding group;
    owner: the owner rank of every point (default: contiguous blocks).
    solver: the ILQR writing `records`; torch's stream waits on its launch
    stream before the gather, and the solver's stream waits on torch's after
    it (the recursion reads what the gather wrote)."""

    def __init__(self, records: torch.Tensor, rank: int, world: int, group=None, solver=None, owner=None):
        import numpy as np
        S, P, D = records.shape
        self.records, self.rank, self.world, self.group, self.solver = records, rank, world, group, solver
        self.owner = np.asarray(block_owners(world, P) if owner is None else owner, dtype=np.int64)
        if self.owner.shape != (P,) or self.owner.min() < 0 or self.owner.max() >= world:
            raise ValueError("owner: one rank in [0, world) per point")
        self.idx = [torch.as_tensor(np.nonzero(self.owner == r)[0], device=records.device) for r in range(world)]
        self.nown = int(self.idx[rank].numel())
        self.nmax = max(int(i.numel()) for i in self.idx)
        self.send = torch.zeros(S, self.nmax, D, dtype=records.dtype, device=records.device)
        self.recv = torch.empty(world, S, self.nmax, D, dtype=records.dtype, device=records.device)

    @classmethod
    def for_solver(cls, solver, rank: int, world: int, group=None):
        """the solver's resident records, owned as its pipelined sharded
        iteration (ILQR.forward_sharded) differentiates them"""
        ptr, stride = solver.device_deriv()
        rec = device_view(ptr, solver.S * solver.P * stride).view(solver.S, solver.P, stride)
        return cls(rec, rank, world, group, solver, owner=solver.point_owners(world))

    def _solver_stream(self):
        if self.solver is None or not self.records.is_cuda:
            return None
        sst = self.solver.stream
        return torch.cuda.ExternalStream(sst, device=self.records.device) if sst else None

    def exchange(self):
        """every rank's points -> every rank's `records`"""
        ext = self._solver_stream()
        cur = torch.cuda.current_stream(self.records.device) if self.records.is_cuda else None
        if ext is not None and ext.cuda_stream != cur.cuda_stream:
            cur.wait_stream(ext)
        self.send[:, :self.nown] = self.records.index_select(1, self.idx[self.rank])
        if self.world > 1:
            dist.all_gather_into_tensor(self.recv.view(-1), self.send.view(-1), group=self.group)
        else:
            self.recv[0].copy_(self.send)
        for r in range(self.world):
            n = int(self.idx[r].numel())
            if n and r != self.rank:
                self.records.index_copy_(1, self.idx[r], self.recv[r, :, :n])
        if ext is not None and ext.cuda_stream != cur.cuda_stream:
            ext.wait_stream(cur)


def trajectory_digest(tensors) -> torch.Tensor:
    """an exact digest of fp64 tensors (their bit patterns, summed as int64 with
    wrap-around, weighted by position): equal trajectories give equal digests,
    and any bit that differs changes it with overwhelming likelihood"""
    acc = None
    for t in tensors:
        b = t.reshape(-1).contiguous().view(torch.int64)
        w = torch.arange(1, b.numel() + 1, dtype=torch.int64, device=b.device) * 2 + 1
        d = torch.stack([b.sum(), (b * w).sum()])
        acc = d if acc is None else acc * 31 + d
    return acc


def check_same_trajectory(tensors, world: int, group=None):
    """point sharding splices every rank's records into every other rank's
    recursion, which is right only if every rank rolled out the same
    trajectory bit for bit: all-gather the digests and raise on a mismatch"""
    d = trajectory_digest(tensors)
    if world > 1:
        allg = torch.empty(world * d.numel(), dtype=d.dtype, device=d.device)
        dist.all_gather_into_tensor(allg, d, group=group)
        allg = allg.view(world, -1)
        if not bool((allg == allg[0]).all()):
            raise RuntimeError(f"point sharding: the ranks' rollouts differ (trajectory digests {allg.tolist()})")
    return d


def max_over_ranks(x: float, world: int, device) -> float:
    """The bench's timing rule: the slowest rank defines the step time."""
    t = torch.tensor([x], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
