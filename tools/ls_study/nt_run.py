"""Newton factor speculation study (tools/ls_study/nt_study.c): the bench
workload's rollouts (hopper H = 500, 8 alphas, min-cost selection) on the
oracle, counting Hessian rebuilds whose active set equals the alpha = 1 set.

  python3 tools/ls_study/nt_run.py [seeds] [iterations]
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
LIB = os.path.join(HERE, "liboracle_ntstudy.so")


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    o = os.path.join(ROOT, "oracle")
    subprocess.run(["gcc", "-std=c99", "-O2", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-fopenmp",
                    "-DORA_NT_STUDY", "-I" + os.path.join(o, "include"), "-I" + os.path.join(ROOT, "include"),
                    "-shared", "-o", LIB, os.path.join(o, "mjsub.c"), os.path.join(o, "ilqr_ora.c"),
                    os.path.join(o, "ora_api.c"), os.path.join(HERE, "nt_study.c"), "-lm"], check=True)
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
        d = om.make_data()
        d.step(500)
        d.arr("ctrl")[:] -= 0.1
        z = workloads.normals(s, m.nq + m.nv)
        d.arr("qpos")[:] += 0.01 * z[: m.nq]
        d.arr("qvel")[:] += 0.01 * z[m.nq:]
        il = ora.OILQR(om, d, 500, cost_fn="ora_cost_desc_fn")
        il.set_dinit(d)
        ils.append(il)
    buf = ctypes.create_string_buffer(1024)
    for it in range(iters):
        for il in ils:
            lib.L.ora_nt_study_reset()
            il.forward_candidates(workloads.LINESEARCH_ALPHAS, "min_cost")  # the rollouts alone
            lib.L.ora_nt_study_report(buf, 1024)
            print(json.dumps(dict(json.loads(buf.value.decode()), iteration=it + 1, what="rollouts")), flush=True)
            il.set_dinit(il.point(500))
            il.backward_pass()


if __name__ == "__main__":
    main()
