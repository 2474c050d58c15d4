"""ORACLE / TEST INFRASTRUCTURE ONLY -- bench.py's cpu_baseline leg.

Times the CPU restatement on this host in a child process (the GPU path is
never involved):

  faithful  the reference-faithful iterate() (SURVEY.md §8d "CPU baseline"):
            ora_calcMJDerivatives = src/mjderivative.cpp:212-255 restated
            (OpenMP team of omp_get_num_procs() <= 16 threads, static chunk over
            nv columns, per-call per-thread mjData, redundant centre), or, when
            oracle/_ref was built in this container, the reference's own
            compiled calcMJDerivatives; Riccati/rollout = inc/ilqr.h:116-176 as
            written.  alpha = 1 only (the reference has no line search).
            BASELINE.md protocol, budget-limited: 1 warm-up iterate(), then
            timed iterate() calls until the budget is spent (10 at most);
            reported value = 1 / median per-iteration time.
  tuned     one single-threaded process per core, each iterating ITS OWN seed
            of the bench workload exactly as the GPU does: 8 line-search
            candidates alpha = 2^-i, min-cost selection
            (ora_ilqr_iterate_ls), FD by the restated driver on one thread.
            Aggregate seed-iterations/s = the like-for-like CPU throughput.

  python oracle/cpu_bench.py faithful <blob> <cost.json> <H> <budget_s> [seed]
  python oracle/cpu_bench.py tuned    <blob> <cost.json> <H> <budget_s> <seed> <nalpha>
prints one JSON line.
"""
import json
import os
import statistics
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "ilqg-mujoco_amd"))

import numpy as np  # noqa: E402

import oracle as ora  # noqa: E402


def normals(seed, n):
    from workloads import normals as _n  # pure Python (splitmix64 + Box-Muller)
    return _n(seed, n)


def setup(blob_path, cost_path, lib, seed, state):
    with open(blob_path, "rb") as f:
        blob = f.read()
    om = ora.OModel(blob, lib)
    with open(cost_path) as f:
        c = json.load(f)
    desc = ora.CostDesc()
    desc.nq, desc.nv, desc.nu = om.nq, om.nv, om.nu
    for k, v in c.items():
        arr = getattr(desc, k)
        for i, x in enumerate(v):
            arr[i] = x
    lib.L.ora_set_cost_desc(desc)
    d = om.make_data()
    if state == "cfg5":
        # cfg 5 (humanoid): qpos0 with the root at z = 1.4 (humanoid.xml:49-50), qvel 0
        # (one state: a humanoid leg has no per-seed perturbation)
        d.arr("qpos")[2] = 1.4
        return om, d
    if state != "cfg3":
        raise ValueError(f"unknown state {state!r} (cfg3 | cfg5)")
    # cfg 3 state (tst/test_derivatives.cpp:38-47) + cfg 4's per-seed perturbation
    d.step(500)
    d.arr("ctrl")[:] -= 0.1
    if seed >= 0:
        z = normals(seed, om.nq + om.nv)
        d.arr("qpos")[:] += 0.01 * z[: om.nq]
        d.arr("qvel")[:] += 0.01 * z[om.nq:]
    return om, d


def faithful(blob, cost, H, budget, state, seed=-1):
    kind = "reference" if os.path.exists(ora.REF_SO) else "port"
    lib = ora.ref_lib() if kind == "reference" else ora.oracle_lib()
    om, d = setup(blob, cost, lib, seed, state)
    lib.L.ora_set_nthread(0)  # omp_get_num_procs(), capped at 16 (mjderivative.cpp:32,217)
    il = ora.OILQR(om, d, H, cost_fn="ora_cost_desc_fn", use_ref_fd=(kind == "reference"))
    il.set_dinit(d)
    il.iterate()  # warm-up
    times = []
    t_start = time.perf_counter()
    while len(times) < 10:
        t0 = time.perf_counter()
        il.iterate()
        times.append(time.perf_counter() - t0)
        if time.perf_counter() - t_start > budget:
            break
    return dict(kind=kind, iters=len(times), secs=sum(times), median_s=statistics.median(times),
                threads=lib.L.ora_get_nthread(), nproc=os.cpu_count(), cores=len(os.sched_getaffinity(0)))


def tuned(blob, cost, H, budget, state, seed, nalpha):
    lib = ora.oracle_lib()
    om, d = setup(blob, cost, lib, seed, state)
    lib.L.ora_set_nthread(1)
    alphas = [2.0 ** -i for i in range(nalpha)]
    il = ora.OILQR(om, d, H, cost_fn="ora_cost_desc_fn")
    il.set_dinit(d)

    def one():
        if nalpha > 1:
            il.iterate_ls(alphas, "min_cost")
        else:
            il.iterate()
    one()  # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        one()
        n += 1
        el = time.perf_counter() - t0
        if el > budget:
            break
    return dict(iters=n, secs=el, cores=len(os.sched_getaffinity(0)))


if __name__ == "__main__":
    # cpu_bench.py faithful|tuned BLOB COST H BUDGET STATE(cfg3|cfg5) [SEED [NALPHA]]
    mode, blob, cost, H, budget, state = (sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]),
                                          float(sys.argv[5]), sys.argv[6])
    if mode == "faithful":
        out = faithful(blob, cost, H, budget, state, int(sys.argv[7]) if len(sys.argv) > 7 else -1)
    else:
        out = tuned(blob, cost, H, budget, state, int(sys.argv[7]), int(sys.argv[8]))
    print(json.dumps(out), flush=True)
