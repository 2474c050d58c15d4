"""cfg 5 (BASELINE.json configs[4]): humanoid H=200, one seed, from qpos0 at
z = 1.4.  Per-kernel HIP-event times of one iteration with the exact and the
MFMA Riccati engines with the fp64 FD sweep (the unfused pair on this model),
and cfg 5 proper: fp32 FD (eps 1e-3) with the fp64 MFMA recursion."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ilqg-mujoco_amd"))
import ilqg_amd as ia, workloads  # noqa: E402

H = int(sys.argv[1]) if len(sys.argv) > 1 else 200
m = ia.Model.load(workloads.model_file("humanoid"))
nx, nu = 2 * m.nv, m.nu
flops_step = 4 * nx**3 + 8 * nu * nx**2 + 6 * nx**2 + 4 * nu**2 * nx  # SURVEY.md §8d Riccati count
for mode, fdp in (("exact", "f64"), ("mfma", "f64"), ("mfma", "f32")):
    st = m.reset_state(1)
    st.qpos[0, 2] = 1.4
    g = ia.ILQR(m, st, H, ia.HUMANOID_COST)
    g.set_riccati(mode)
    g.set_fd_precision(fdp)
    g.iterate(); g.synchronize()
    g.set_timing(True); g.timing()
    K = 3
    t = time.perf_counter()
    for _ in range(K):
        g.iterate()
    g.synchronize()
    dt = (time.perf_counter() - t) / K
    tm = {k: v[0] / v[1] for k, v in g.timing().items() if v[1]}
    bw = tm.get("backward", 0.0)
    print(f"{mode:5s} FD {fdp}: {1 / dt:6.2f} it/s ({dt * 1e3:7.2f} ms/it); kernels avg ms "
          f"{ {k: round(v, 3) for k, v in tm.items()} }; backward {bw / H * 1e3:.2f} us/step, "
          f"{flops_step * H / (bw * 1e-3) / 1e12:.3f} TFLOP/s", flush=True)
