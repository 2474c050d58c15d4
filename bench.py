"""bench.py -- iLQR iterations/sec (FD + backward + forward) for Hopper H=500.

  python bench.py --gpus N --steps K --warmup W

A "step" is one ILQR::iterate() (inc/ilqr.h:179-186) of every seed on the
rank: forward rollout of all line-search candidates + selection, FD sweep at
all H+1 points, Riccati backward pass, then the one exchange step of the
multi-GPU design (RCCL all-gather of the per-seed trajectory costs).
Per GPU: cfg-4's share -- 8 MPC seeds (cfg-3 state + N(0, 0.01^2), splitmix64
+ Box-Muller) x 8 line-search candidates alpha = 2^-i (cfg 3).  value = seed
iterations/s summed over ranks (weak scaling).  Rank 0 at N=1 also times the
reference-faithful CPU path on the host cores (cpu_baseline).
"""
import argparse
import json
import os
import subprocess
import sys
import time

# torch first: its libamdhip64 (SONAME libamdhip64.so.7) then serves the HIP
# library too, so the process has one HIP runtime
import torch
import torch.distributed as dist

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ilqg-mujoco_amd"))
import ilqg_amd as ia  # noqa: E402
import workloads  # noqa: E402
from seed_shard import CostExchange, device_view, max_over_ranks, seed_offset  # noqa: E402

METRIC = "iLQR iterations/sec (FD+backward+forward) for Hopper H=500 at 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
# FP64 vector peak: 256 CUs x 4 SIMDs x 16 f64 FMA lanes/clk x 2 x 2.4 GHz (AMD spec
# 78.6 TFLOP/s; half the guide's 157.3 TFLOP/s FP32 vector rate)
FP64_PEAK_TFS = 78.6
FLOPS_JSON = os.path.join(ROOT, "tests", "fixtures", "flops.json")
SRC_SHA = ia.source_sha()


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC
    summaries (profiles/r*_pmc_traffic.json, tools/pmc_summary.py): the newest
    one taken on these kernel sources (src_sha); failing that the newest one,
    marked stale"""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]*_pmc_traffic.json")))
    docs = []
    for f in files:
        with open(f) as fh:
            docs.append((f, json.load(fh)))
    docs = [(f, d) for f, d in docs if d.get(kernel) is not None]
    if not docs:
        return {"bytes": None, "file": None, "src_sha": None, "head": None, "stale": None}
    match = [(f, d) for f, d in docs if d.get("src_sha") == SRC_SHA]
    f, d = (match or docs)[-1]
    return {"bytes": d[kernel], "file": os.path.relpath(f, ROOT), "src_sha": d.get("src_sha"),
            "head": d.get("head"), "stale": not match}


def algorithmic_flops(S, A, P):
    """fp64 flops per launch from the instrumented oracle's counts
    (tests/fixtures/flops.json): the rollout = S*A*P mj_steps,
    the fused sweep = S*P calcMJDerivatives calls + S*(P-1) Riccati steps."""
    with open(FLOPS_JSON) as f:
        h = json.load(f)["models"]["hopper"]
    return {"rollout": S * A * P * h["step"]["flops"],
            "fd_backward": S * (P * h["fd_point"]["flops"] + (P - 1) * h["riccati_step"]["flops"])}


def algorithmic_bytes(m, S, A, P):
    """per seed, state record Sr = nq+nv+nu+nv, D deriv doubles,
    Kk = nu*nx + nu.  FD = P(Sr+D)8, backward = (P(D+nx) + (P-1)Kk)8,
    forward = P(Kk + nx + nu + Sr)8 per candidate."""
    nx = 2 * m.nv
    Sr = m.nq + m.nv + m.nu + m.nv
    Kk = m.nu * nx + m.nu
    fd = P * (Sr + m.D) * 8
    bw = (P * (m.D + nx) + (P - 1) * Kk) * 8
    fw = P * (Kk + nx + m.nu + Sr) * 8
    return {"fd_sweep": S * fd, "backward": S * bw, "rollout": S * A * fw, "fd_backward": S * (fd + bw)}


def cpu_baseline(budget_s, horizon, threads, nalpha, model="hopper", cost=None):
    """The CPU side of the comparison, timed on this host (rank 0, N=1 only;
    oracle/cpu_bench.py, test infrastructure run as child processes):
      value   the reference-faithful iterate() (restated src/mjderivative.cpp
              OpenMP driver, nthread = omp_get_num_procs() on `threads` pinned
              cores, alpha = 1) -- 1 warm-up, then timed iterate() calls within
              the budget (<= 10), value = 1 / median (BASELINE.md's protocol,
              budget-limited: one run, not the median of 5);
      tuned   like-for-like throughput: `threads` single-threaded processes,
              one per pinned core, each iterating its own seed of the bench
              workload (8 alphas, min-cost selection) -> seed-iterations/s."""
    cost = cost or ia.HOPPER_COST
    m = ia.Model.load(workloads.model_file(model))
    tag = f"{os.getpid()}"
    blob_path = os.path.join("/tmp", f"ilqg_{model}_blob_{tag}.bin")
    cost_path = os.path.join("/tmp", f"ilqg_{model}_cost_{tag}.json")
    with open(blob_path, "wb") as f:
        f.write(m.blob())
    with open(cost_path, "w") as f:
        json.dump({k: list(v) for k, v in cost.packed(m.nq, m.nv, m.nu).items()}, f)
    state = "cfg-3 state" if model == "hopper" else "cfg-5 state: qpos0, root z = 1.4"
    state_arg = "cfg3" if model == "hopper" else "cfg5"
    script = os.path.join(ROOT, "oracle", "cpu_bench.py")
    allc = sorted(os.sched_getaffinity(0))
    cores = allc[:threads]

    def pinned(cs):
        return lambda: os.sched_setaffinity(0, cs)
    try:
        out = subprocess.run([sys.executable, script, "faithful", blob_path, cost_path, str(horizon), str(budget_s),
                              state_arg],
                             capture_output=True, text=True, preexec_fn=pinned(cores), timeout=budget_s * 4 + 120)
        ref = json.loads(out.stdout.strip().splitlines()[-1])
        tb = max(3.0, budget_s / 3)
        procs = [subprocess.Popen([sys.executable, script, "tuned", blob_path, cost_path, str(horizon), str(tb),
                                   state_arg, str(i), str(nalpha)], stdout=subprocess.PIPE, text=True,
                                  preexec_fn=pinned([c])) for i, c in enumerate(cores)]
        tuned = [json.loads(p.communicate(timeout=tb * 4 + 120)[0].strip().splitlines()[-1]) for p in procs]
    finally:
        for pth in (blob_path, cost_path):
            os.unlink(pth)
    cpu_model = ""
    phys = set()
    try:
        pid = core = None
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name") and not cpu_model:
                cpu_model = line.split(":", 1)[1].strip()
            elif line.startswith("physical id"):
                pid = line.split(":", 1)[1].strip()
            elif line.startswith("core id"):
                core = line.split(":", 1)[1].strip()
            elif not line.strip() and pid is not None:
                phys.add((pid, core))
                pid = core = None
    except OSError:
        pass
    host_cores = len(phys) or None
    thr = sum(t["iters"] / t["secs"] for t in tuned)
    per_core = thr / len(tuned)
    return {
        "value": 1.0 / ref["median_s"],
        "unit": "iLQR iterations/s (1 seed)",
        "cores": ref["threads"],
        "kind": ref["kind"],
        "sample": (f"{model} H={horizon}, 1 seed ({state}), alpha=1, fp64 FD: 1 warm-up + {ref['iters']} timed iterate() "
                   f"calls in {ref['secs']:.1f}s, value = 1/median; FD = "
                   + ("the reference's own src/mjderivative.cpp (oracle/_ref)" if ref["kind"] == "reference" else
                      "the restated src/mjderivative.cpp driver (oracle/ilqr_ora.c)")
                   + f" with OpenMP nthread=omp_get_num_procs()={ref['threads']}, per-call mjData; host {cpu_model},"
                   f" {len(allc)} cpus visible, pinned to {len(cores)}"),
        "protocol_note": (f"BASELINE.md's protocol (1 warm-up + 10 iterations, median of 5 runs) would take "
                          f"~{55 * ref['median_s']:.0f} s at this rate; the bench contract bounds the CPU sample to "
                          f"~10-30 s, so this is one run of up to 10 iterations within a {budget_s:.0f} s budget"),
        "tuned_throughput": {
            "value": thr, "unit": "seed-iterations/s", "cores": len(tuned),
            "per_core": per_core,
            "sample": (f"{len(tuned)} single-threaded processes, one per pinned core, each iterating its own bench "
                       f"seed ({model} H={horizon}, {nalpha} alphas{', min-cost selection' if nalpha > 1 else ''}, fp64 FD): "
                       f"{sum(t['iters'] for t in tuned)} iterations in ~{tb:.0f}s each"),
            # the GPU box gives one GPU a share of its host (16 CPUs); the whole
            # host is not measured, only extrapolated linearly from the share
            "host_physical_cores": host_cores,
            "host_extrapolated": per_core * host_cores if host_cores else None,
            "host_note": ("one GPU's CPU share of the box is 16 cores (the pool's per-GPU limit), so the tuned leg "
                          "runs 16 pinned processes; host_extrapolated = per_core x host_physical_cores is a linear "
                          "extrapolation to every physical core, not a measurement")},
    }


def visible_gpus():
    """GPUs this process may use, counted without initialising HIP: the KFD
    topology's GPU nodes (nodes with a nonzero simd_count), narrowed by
    HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES; None if the topology is absent
    (each rank then checks its own LOCAL_RANK when it binds its device)."""
    import glob
    n = 0
    for f in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties"):
        try:
            with open(f) as fh:
                props = dict(line.split() for line in fh if len(line.split()) == 2)
        except OSError:
            continue
        if int(props.get("simd_count", "0")) > 0:
            n += 1
    if n == 0:
        return None
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip() != ""]))
    return n


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv):
    """`bench.py --gpus N` without a launcher: start N ranks of this script as
    child processes (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, the same
    environment torchrun gives) and return the worst child exit code.  Runs
    before anything touches the GPU (the parent never initialises HIP); if one
    rank fails the others are stopped rather than left waiting in a collective."""
    env0 = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE=str(n),
                LOCAL_WORLD_SIZE=str(n))
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv,
                              env=dict(env0, RANK=str(r), LOCAL_RANK=str(r))) for r in range(n)]
    rcs = [None] * n
    while any(rc is None for rc in rcs):
        for i, p in enumerate(procs):
            if rcs[i] is None:
                rcs[i] = p.poll()
        if any(rc not in (None, 0) for rc in rcs):
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    p.terminate()
                    try:
                        rcs[i] = p.wait(timeout=30)
                    except subprocess.TimeoutExpired:
                        p.kill()
                        rcs[i] = p.wait()
            break
        time.sleep(0.05)
    bad = [rc for rc in rcs if rc != 0]
    return (bad[0] if bad[0] > 0 else 1) if bad else 0


class DrySolver:
    """`--dry-run`: the bench's host side (rank launch, process group, cost
    exchange, max-over-ranks timing, rank-0 printing) on CPU with gloo and no
    GPU.  Stands in for ilqg_amd.ILQR's iterate()/costs only; its per-seed
    costs are a deterministic function of (global seed, iteration).  Never a
    measurement: the line it prints carries "dry_run": true and no roofline."""

    def __init__(self, S, rank):
        self.S, self.rank, self.it = S, rank, 0
        self.costs = torch.zeros(S, dtype=torch.float64)
        self.stream = 0

    def iterate(self):
        self.it += 1
        g = np.arange(seed_offset(self.rank, self.S), seed_offset(self.rank, self.S) + self.S)
        self.costs.copy_(torch.from_numpy(np.abs(np.sin(1.0 + g * 0.37 + self.it)) * (1.0 + g)))

    def synchronize(self):
        pass

    def set_timing(self, on):
        pass

    def timing(self):
        return {}


CFG5_METRIC = ("iLQR iterations/sec (FD+backward+forward) for Humanoid H=200, fp32 FD + fp64 MFMA Riccati "
               "(BASELINE.json configs[4])")
FP32_PEAK_TFS = 157.3    # MI355X_MICROARCH.md chip table, FP32 vector
FP64_MFMA_PEAK_TFS = 78.6  # AMD spec, FP64 matrix (v_mfma_f64_16x16x4_f64); the guide lists no FP64 row


def run_humanoid_cfg5(args, world, rank, local_rank):
    """BASELINE.json configs[4]: humanoid, H = 200, one seed (qpos0 with the
    root at z = 1.4, humanoid.xml:49-50), fp32 FD (eps 1e-3) with the fp64
    Riccati recursion on the matrix cores (ilqg_solver_set_riccati MFMA).  On
    N > 1 GPUs the one seed's FD sweep is point-sharded (--cfg5-shard points,
    the default): every rank rolls out the same trajectory in the pipelined
    iterate's chunks and differentiates the points it owns behind them
    (ilqg_forward_sharded: chunks round-robin, the last chunks split over all
    ranks), one RCCL all-gather of the fp64 records (RecordExchange, 3.4 MB)
    gives every rank all of them, and every rank runs the recursion; the
    warm-up checks that every rank's trajectory is bit-identical.  value =
    iterations/s of that one seed (strong scaling).  --cfg5-shard replicas runs N independent replicas
    instead.  A separate line, not the headline."""
    H = 200
    P = H + 1
    m = ia.Model.load(workloads.model_file("humanoid"))
    st = m.reset_state(1)
    st.qpos[0, 2] = 1.4
    g = ia.ILQR(m, st, H, ia.HUMANOID_COST, device=local_rank)
    g.set_riccati("mfma")
    g.set_fd_precision("f32")
    shard = world > 1 and args.cfg5_shard == "points"
    if shard:
        from seed_shard import RecordExchange, check_same_trajectory, device_view
        stream = torch.cuda.Stream()
        g.set_stream(stream.cuda_stream)
        rx = RecordExchange.for_solver(g, rank, world)
        # the resident nominal trajectory (every rank's own rollout), for the
        # cross-rank check that the records spliced together describe one trajectory
        traj = [device_view(g.device_traj_ptr(f), P * n) for f, n in (("qpos", m.nq), ("qvel", m.nv), ("ctrl", m.nu))]

        def one_iter():
            with torch.cuda.stream(stream):
                # the pipelined rollout with this rank's points differentiated
                # behind its chunks, the gather, then the recursion on every rank
                g.forward_sharded(rank, world)
                rx.exchange()
                g.riccati_pass()
    else:
        def one_iter():
            g.iterate()
    for _ in range(args.warmup):
        one_iter()
        if shard:
            with torch.cuda.stream(stream):
                check_same_trajectory(traj, world)
    g.synchronize()
    if world > 1:
        dist.barrier()
    g.set_timing(True)
    g.timing()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_iter()
    g.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0, world, "cuda")
    kt = {k: {"ms_total": v[0], "launches": v[1], "avg_ms": v[0] / v[1] if v[1] else 0.0} for k, v in g.timing().items()}
    with open(FLOPS_JSON) as f:
        hf = json.load(f)["models"]["humanoid"]
    P = H + 1
    fd_ms = sum(kt[k]["avg_ms"] for k in ("fd_centre", "fd_cols") if k in kt)
    bw_ms = kt.get("backward", {}).get("avg_ms", 0.0)
    roll_ms = kt.get("rollout", {}).get("avg_ms", 0.0)
    # points one FD launch differentiates: this rank's block, over the chunks
    # of the pipelined iteration (ILQG_PIPE_CHUNK: one sweep launch per chunk)
    fd_launches = max((kt.get("fd_cols", {}).get("launches", 0) or kt.get("fd_centre", {}).get("launches", 0)), 1)
    fd_pts = (rx.nown if shard else P) / max(fd_launches / args.steps, 1.0)
    roll_pts = P / max(kt.get("rollout", {}).get("launches", 0) / args.steps, 1.0)
    fd_tf = fd_pts * hf["fd_point"]["flops"] / (fd_ms * 1e-3) / 1e12 if fd_ms else 0.0
    bw_tf = H * hf["riccati_step"]["flops"] / (bw_ms * 1e-3) / 1e12 if bw_ms else 0.0
    value = (1 if shard else world) * args.steps / elapsed
    out = {
        "metric": CFG5_METRIC, "value": value,
        "unit": "iLQR iterations/s (one seed, FD point-sharded over the GPUs)" if shard else
                "iLQR iterations/s (1 seed per GPU, replicas summed)",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": "strong" if shard else "weak", "vs_baseline": None,
        "dtype": "f32 (FD sweep) / f64 (rollout, Riccati)",
        "data": "synthetic (humanoid qpos0, root z = 1.4, qvel 0; state-only quadratic cost)",
        "config": {"workload": "humanoid_H200_cfg5", "model": "humanoid.xml", "horizon": H, "seeds_per_gpu": 1,
                   "fd_precision": "f32 (eps 1e-3)", "riccati": "fp64 MFMA (v_mfma_f64_16x16x4_f64)",
                   "parallelism": (f"FD point-sharded x{world} (RCCL all-gather of the fp64 records, "
                                   f"{P * g.device_deriv()[1] * 8 / 1e6:.1f} MB per iteration)") if shard else
                                  f"replicas x{world}"},
        "kernels": kt,
        "roofline": {
            # per serial step: one launch's time over the points it steps (the
            # pipelined iterate launches the rollout in chunks of ILQG_PIPE_CHUNK points)
            "rollout": {"bound": "latency", "avg_launch_ms": roll_ms, "points_per_launch": roll_pts,
                        "us_per_step": roll_ms / roll_pts * 1e3},
            "fd_sweep": {"bound": "fp32-valu", "flops_per_launch": fd_pts * hf["fd_point"]["flops"],
                         "avg_launch_ms": fd_ms, "achieved_tflops": fd_tf, "peak_tflops": FP32_PEAK_TFS,
                         "frac": fd_tf / FP32_PEAK_TFS,
                         "flops_source": "tests/fixtures/flops.json (instrumented oracle, fp64 op count)"},
            "backward": {"bound": "fp64-mfma", "flops_per_launch": H * hf["riccati_step"]["flops"],
                         "avg_launch_ms": bw_ms, "achieved_tflops": bw_tf, "peak_tflops": FP64_MFMA_PEAK_TFS,
                         "frac": bw_tf / FP64_MFMA_PEAK_TFS, "us_per_step": bw_ms / H * 1e3}},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cb = cpu_baseline(args.cpu_budget, H, args.cpu_threads, 1, model="humanoid", cost=ia.HUMANOID_COST)
        out["cpu_baseline"] = cb
        out["speedup_vs_cpu_per_seed"] = value / cb["value"]
        out["speedup_vs_cpu_throughput"] = value / cb["tuned_throughput"]["value"]
    if rank == 0:
        print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--seeds-per-gpu", type=int, default=8)
    ap.add_argument("--alphas", type=int, default=8)
    ap.add_argument("--horizon", type=int, default=500)
    ap.add_argument("--groups", type=int, default=1,
                    help="seed groups per GPU (ilqg_solver_set_groups): the seeds software-pipelined as G ranges")
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    # how the recursion reads the FD records: the reference's (quirk Q1, the
    # headline) or the corrected Jacobians (ilqg_solver_set_layout; same work)
    ap.add_argument("--layout", choices=("reference", "corrected"), default="reference")
    # host-side rehearsal of the multi-rank path on CPU (gloo, no GPU, no measurement)
    ap.add_argument("--dry-run", action="store_true")
    # the headline (cfg 4's per-GPU share) or cfg 5 as a separate line
    ap.add_argument("--workload", choices=("hopper_cfg4", "humanoid_cfg5"), default="hopper_cfg4")
    # cfg 5 on N > 1 GPUs: the one seed's FD sweep point-sharded, or N replicas
    ap.add_argument("--cfg5-shard", choices=("points", "replicas"), default="points")
    argv = sys.argv[1:]
    args = ap.parse_args(argv)

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # count the devices without touching HIP in this parent (ranks are fresh children)
        nvis = visible_gpus()
        if not args.dry_run and nvis is not None and nvis < args.gpus:
            sys.exit(f"bench.py: --gpus {args.gpus} but {nvis} GPUs visible")
        sys.exit(launch_ranks(args.gpus, argv))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}; refusing to print a mislabelled line")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    print(f"bench.py: rank {rank}/{world} started", file=sys.stderr, flush=True)
    if args.dry_run:
        dev = "cpu"
        if world > 1:
            dist.init_process_group("gloo", rank=rank, world_size=world)
    else:
        dev = "cuda"
        torch.cuda.set_device(local_rank)
        if world > 1:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    if args.workload == "humanoid_cfg5" and not args.dry_run:
        run_humanoid_cfg5(args, world, rank, local_rank)
        if world > 1:
            dist.destroy_process_group()
        return
    S, A, H = args.seeds_per_gpu, args.alphas, args.horizon
    P = H + 1
    alphas = tuple(2.0 ** -i for i in range(A))
    m = ia.Model.load(workloads.model_file("hopper"))
    if args.dry_run:
        solver = DrySolver(S, rank)
        exchange = CostExchange(solver.costs, world)
        stream = None
    else:
        dmain = workloads.hopper_dmain(m, S, sigma=0.01, seed_offset=seed_offset(rank, S))
        solver = ia.ILQR(m, dmain, H, ia.HOPPER_COST, alphas=alphas, select="min_cost", device=local_rank)
        # one explicit stream for the solver's launches and the cost exchange: the
        # all-gather (RCCL waits on torch's current stream) is then ordered after
        # the iteration that produced the costs (torch's default stream is the
        # legacy null stream, which does not order against the solver's own)
        stream = torch.cuda.Stream()
        solver.set_stream(stream.cuda_stream)
        if args.layout != "reference":
            solver.set_layout(args.layout)
        if args.groups > 1:
            solver.set_groups(args.groups)
        exchange = CostExchange(device_view(solver.device_costs_ptr(), S), world, solver=solver)

    def one_step():
        if stream is None:
            solver.iterate()
            return exchange()
        with torch.cuda.stream(stream):
            solver.iterate()
            return exchange()

    def device_sync():
        if not args.dry_run:
            torch.cuda.synchronize()

    for _ in range(args.warmup):
        one_step()
    device_sync()
    solver.synchronize()  # raises if a fused sweep's hand-off wait timed out
    if world > 1:
        dist.barrier()
    solver.set_timing(True)
    solver.timing()  # reset
    device_sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        best = one_step()
    device_sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # outside the timed region: a run whose hand-off waits tripped produced
    # garbage gains and costs and must not print a bench line (raises)
    solver.synchronize()
    ktime = solver.timing()
    elapsed = max_over_ranks(elapsed, world, dev)
    best_seed = int(best.item())
    gathered = exchange.gather()

    value = world * S * args.steps / elapsed
    if args.dry_run:
        if rank == 0:
            print(json.dumps({"metric": METRIC, "dry_run": True, "value": None, "n_gpus": world,
                              "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
                              "exchange": {"costs_gathered": int(gathered.numel()), "best_seed": best_seed,
                                           "costs": gathered.tolist()}}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return
    # roofline of the dominant kernel (largest device time in the timed region)
    # per launch: with seed groups every hot-path launch covers S / G seeds
    abytes = {k: v / args.groups for k, v in algorithmic_bytes(m, S, A, P).items()}
    per_kernel = {k: {"ms_total": v[0], "launches": v[1], "avg_ms": (v[0] / v[1] if v[1] else 0.0)}
                  for k, v in ktime.items()}
    # fd_backward: the fused FD sweep with the Riccati recursion streamed behind it
    groups = {"fd_sweep": ("fd_centre", "fd_cols"), "rollout": ("rollout",), "backward": ("backward",),
              "fd_backward": ("fd_backward",)}
    gtime = {g: sum(per_kernel[k]["ms_total"] for k in ks) for g, ks in groups.items()}
    dom = max(gtime, key=gtime.get)
    dom_avg_ms = gtime[dom] / max(1, max(per_kernel[k]["launches"] for k in groups[dom]))
    achieved = abytes[dom] / (dom_avg_ms * 1e-3) / 1e9
    traffic = pmc_traffic(dom)

    # the binding roof: FP64 VALU (algorithmic flops / launch time vs the vector peak)
    aflops = {k: v / args.groups for k, v in algorithmic_flops(S, A, P).items()}
    valu = {k: {"flops_per_launch": f, "avg_launch_ms": gtime[k] / max(1, per_kernel[k]["launches"]),
                "achieved_tflops": f / (gtime[k] / max(1, per_kernel[k]["launches"]) * 1e-3) / 1e12
                if per_kernel[k]["launches"] else 0.0} for k, f in aflops.items()}
    for v in valu.values():
        v["frac"] = v["achieved_tflops"] / FP64_PEAK_TFS

    out = {
        "metric": METRIC,
        "value": value,
        "unit": "iLQR iterations/s (seed-iterations, summed over GPUs)",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (cfg-3 hopper state + splitmix64/Box-Muller N(0,0.01^2) seed perturbations)",
        "config": {"workload": f"hopper_H{H}_{S}seeds_x_{A}alphas_per_gpu", "model": "hopper.xml",
                   "horizon": H, "seeds_per_gpu": S, "linesearch_candidates": A, "global_seeds": world * S,
                   "parallelism": f"seed-sharded x{world} (RCCL all-gather of per-seed costs)",
                   "layout": args.layout, "seed_groups": args.groups},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic["bytes"],
                     "traffic_file": traffic["file"], "traffic_src_sha": traffic["src_sha"],
                     "traffic_head": traffic["head"], "traffic_stale": traffic["stale"], "src_sha": SRC_SHA,
                     "algorithmic_bytes_per_launch": abytes[dom], "avg_launch_ms": dom_avg_ms,
                     "note": "latency/FP64-VALU-bound path; HBM fraction reported per contract",
                     "valu": {"bound": "fp64-valu", "peak_tflops": FP64_PEAK_TFS, "unit": "TFLOP/s",
                              "flops_source": "tests/fixtures/flops.json (instrumented oracle)", "kernels": valu}},
        "kernels": per_kernel,
        "best_seed": best_seed,
        "exchange": {"costs_gathered": int(gathered.numel()), "best_seed": best_seed},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cb = cpu_baseline(args.cpu_budget, H, args.cpu_threads, A)
        # per seed: one GPU seed-iteration rate vs the reference-faithful CPU iterate()
        out["speedup_vs_cpu_per_seed"] = (value / S) / cb["value"]
        # like-for-like: GPU seed-iterations/s vs the same workload on `cores` tuned host cores
        tt = cb["tuned_throughput"]
        out["speedup_vs_cpu_throughput"] = value / tt["value"]
        if tt["host_extrapolated"]:
            # one GPU against every physical core of its host (extrapolated), and
            # the node (8 GPUs at this per-GPU rate, weak scaling) against the host
            out["speedup_vs_cpu_host_extrapolated"] = value / tt["host_extrapolated"]
            out["node_8gpu_vs_cpu_host_extrapolated"] = 8 * value / tt["host_extrapolated"]
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
