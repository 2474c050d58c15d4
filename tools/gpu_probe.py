"""First GPU probe: parity of step / forward / FD / iterate vs the oracle, plus rough timings."""
import sys, time, os, numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ilqg-mujoco_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import ilqg_amd as ia, oracle as ora
RES = os.path.join(ROOT, "ilqg-mujoco_amd", "models")

def rep(name, a, b):
    a = np.asarray(a); b = np.asarray(b)
    err = np.abs(a - b).max() if a.size else 0.0
    print(f"  {name:28s} bitexact={np.array_equal(a, b)} maxabs={err:.3e}", flush=True)

for mname, steps, cost, cfn in [("inverted_pendulum", 10, ia.PENDULUM_COST, "ora_cost_pendulum"),
                                ("hopper", 500, ia.HOPPER_COST, "ora_cost_desc_fn")]:
    print(mname, flush=True)
    m = ia.Model.load(os.path.join(RES, mname + ".xml"))
    om = ora.OModel(m.blob())
    om.lib.L.ora_set_cost_desc(ora.CostDesc.from_cost(cost, m.nq, m.nv, m.nu))
    d = om.make_data()
    st = m.reset_state(1)
    t = time.time(); m.step(st, steps); tg = time.time() - t
    d.step(steps)
    rep("step x%d qpos" % steps, st.qpos[0], d.arr("qpos")); rep("qvel", st.qvel[0], d.arr("qvel")); rep("warm", st.warm[0], d.arr("warm"))
    print("   gpu step batch wall %.3f s" % tg)
    if mname == "hopper":
        d.arr("ctrl")[:] -= 0.1; st.ctrl[:] -= 0.1
    qacc = m.forward(st.copy())
    d2 = om.make_data(); d2.set_state(**d.state()); d2.forward()
    rep("forward qacc", qacc[0], d2.arr("qacc"))
    der = m.calc_derivatives(st, cost)
    dro = ora.calc_derivatives(om, d, cost_fn=cfn, nthread=1)
    rep("fd deriv", der[0], dro)
    for H in ([20, 100, 200] if mname == "inverted_pendulum" else [50, 500]):
        dmain = om.make_data(); dmain.set_state(**d.state())
        oil = ora.OILQR(om, dmain, H, cost_fn=cfn)
        oil.set_dinit(dmain)
        t = time.time(); oil.iterate(); oil.iterate(); to = (time.time() - t) / 2
        gil = ia.ILQR(m, ia.State(**{k: np.atleast_1d(v)[None] if k != "time" else np.array([v]) for k, v in d.state().items()}), H, cost)
        gil.iterate(); gil.synchronize()
        t = time.time(); gil.iterate(); gil.synchronize(); tg = time.time() - t
        ot = oil.traj(); gt = gil.traj(); oa = oil.arrays(); K, k = gil.gains()
        print(f"  H={H} oracle iterate {to*1e3:.1f} ms (1 thread), gpu iterate {tg*1e3:.1f} ms", flush=True)
        rep(" traj qpos", gt.qpos, ot["qpos"]); rep(" traj ctrl", gt.ctrl, ot["ctrl"])
        rep(" deriv", gil.deriv()[0], oa["deriv"]); rep(" K", K[0], oa["K"]); rep(" k", k[0], oa["k"])
        V, v = gil.value(); rep(" V", V[0], oa["V"])
