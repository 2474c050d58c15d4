"""Device time of the standalone Riccati recursion (ilqg_backward) on the
bench workload's records: python tools/bw_time.py [S] [reps]"""
import os, sys, json
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ilqg-mujoco_amd"))
import ilqg_amd as ia
import workloads

S = int(sys.argv[1]) if len(sys.argv) > 1 else 8
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
m = ia.Model.load(workloads.model_file("hopper"))
g = ia.ILQR(m, workloads.hopper_dmain(m, S, sigma=0.01), 500, ia.HOPPER_COST)
g.iterate()
g.synchronize()
g.backward_pass()
g.synchronize()
g.set_timing(True)
g.timing()
for _ in range(reps):
    g.backward_pass()
g.synchronize()
t = g.timing()
tot, n = t["backward"]
print(json.dumps({"S": S, "mw": os.environ.get("ILQG_BW_MW", "1"), "ms_per_launch": tot / n,
                  "us_per_step": tot / n / 500 * 1e3}))
