"""Line-search certification study (VERDICT r5 "Next" #2; tools/ls_study/study.c).

Builds the oracle with -DORA_LS_STUDY plus study.c, runs the bench workload's
iterations (hopper H = 500, cfg-4 seeds, 8 line-search candidates, min-cost
selection: the sweep ilqg_iterate's fused launch differentiates) on the CPU
oracle, and reports, per iteration's FD sweep, how many of the line searches'
bisection levels are decidable without evaluating d1 exactly.

  python3 tools/ls_study/run.py [seeds] [iterations]
"""
import ctypes
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "ilqg-mujoco_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
LIB = os.path.join(HERE, "liboracle_lsstudy.so")


def build():
    o = os.path.join(ROOT, "oracle")
    subprocess.run(["gcc", "-std=c99", "-O2", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-fopenmp", "-DORA_LS_STUDY",
                    "-I" + os.path.join(o, "include"), "-I" + os.path.join(ROOT, "include"), "-shared", "-o", LIB,
                    os.path.join(o, "mjsub.c"), os.path.join(o, "ilqr_ora.c"), os.path.join(o, "ora_api.c"),
                    os.path.join(HERE, "study.c"), "-lm"], check=True)


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    build()
    import ilqg_amd as ia
    import oracle as ora
    import workloads
    m = ia.Model.load(workloads.model_file("hopper"))
    lib = ora.Lib(LIB)
    om = ora.OModel(m.blob(), lib=lib)
    om.lib.L.ora_set_cost_desc(ora.CostDesc.from_cost(ia.HOPPER_COST, m.nq, m.nv, m.nu))
    om.lib.L.ora_set_nthread(1)
    ils = []
    for s in range(S):
        # cfg-3 state + cfg 4's perturbation of seed s (workloads.hopper_dmain, on the oracle)
        d = om.make_data()
        d.step(500)
        d.arr("ctrl")[:] -= 0.1
        z = workloads.normals(s, m.nq + m.nv)
        d.arr("qpos")[:] += 0.01 * z[: m.nq]
        d.arr("qvel")[:] += 0.01 * z[m.nq:]
        il = ora.OILQR(om, d, 500, cost_fn="ora_cost_desc_fn")
        il.set_dinit(d)
        ils.append(il)
    buf = ctypes.create_string_buffer(4096)
    out = []
    for it in range(iters):
        lib.L.ora_ls_study_reset()
        for il in ils:
            il.iterate_ls(workloads.LINESEARCH_ALPHAS, "min_cost")
        lib.L.ora_ls_study_report(buf, 4096)
        r = json.loads(buf.value.decode())
        r["iteration"] = it + 1
        r["seeds"] = S
        r["decidable_fraction_of_bisection_levels"] = r["decidable_levels"] / max(1, r["bisection_levels"])
        r["decidable_fraction_of_iterations"] = r["decidable_levels"] / max(1, r["iterations"])
        out.append(r)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
