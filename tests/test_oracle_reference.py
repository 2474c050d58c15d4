"""Pin the oracle: its FD restatement against the reference's own
src/mjderivative.cpp + src/util.cpp + src/update.cpp compiled unmodified
(oracle/_ref/libilqg_ref.so) and against the committed golden vectors
(tests/golden/*.npz, made by tests/golden/make_golden.py from that build)."""
import numpy as np
import pytest

from conftest import has_ref, load_golden, model_path

needs_ref = pytest.mark.skipif(not has_ref(), reason="oracle/_ref not built (needs /root/reference)")


def _models(ia, ora, name, lib=None):
    m = ia.Model.load(model_path(name))
    return m, ora.OModel(m.blob(), lib)


@pytest.mark.parametrize("fixture,cfn,cost", [
    ("fd_pendulum.npz", "ora_cost_pendulum", None),
    ("fd_hopper.npz", "ora_cost_desc_fn", "HOPPER_COST"),
    ("fd_hopper_dummycost.npz", "ora_cost_desc_fn", "DUMMY"),
])
def test_oracle_fd_matches_golden(ia, ora, fixture, cfn, cost):
    """oracle restatement == golden vectors written by the reference's calcMJDerivatives (bit exact)"""
    g = load_golden(fixture)
    m, om = _models(ia, ora, str(g["model"]))
    if cost is not None:
        c = ia.HOPPER_COST if cost == "HOPPER_COST" else ia.Cost(lq=[1.0])
        om.lib.L.ora_set_cost_desc(ora.CostDesc.from_cost(c, m.nq, m.nv, m.nu))
    for p in range(len(g["time"])):
        d = om.make_data()
        d.set_state(time=g["time"][p], qpos=g["qpos"][p], qvel=g["qvel"][p], warm=g["warm"][p], ctrl=g["ctrl"][p])
        der = ora.calc_derivatives(om, d, cost_fn=cfn, nthread=2)
        assert np.array_equal(der, g["deriv"][p]), f"point {p}: max|diff| {np.abs(der - g['deriv'][p]).max()}"


@needs_ref
@pytest.mark.parametrize("nthread", [1, 2, 3, 8])
def test_oracle_fd_equals_reference_driver(ia, ora, nthread):
    """restated worker/calcMJDerivatives == reference mjderivative.cpp, any thread schedule"""
    for name, steps, shift, cfn, cost in (("inverted_pendulum", 10, 0.0, "ora_cost_pendulum", None),
                                          ("hopper", 500, -0.1, "ora_cost_desc_fn", ia.HOPPER_COST)):
        m, om = _models(ia, ora, name)
        _, rm = _models(ia, ora, name, ora.ref_lib())
        if cost is not None:
            for mm in (om, rm):
                mm.lib.L.ora_set_cost_desc(ora.CostDesc.from_cost(cost, m.nq, m.nv, m.nu))
        d = om.make_data()
        d.step(steps)
        d.arr("ctrl")[:] += shift
        rng = np.random.default_rng(nthread)
        for trial in range(3):
            st = d.state()
            if trial:
                st["qpos"] = st["qpos"] + rng.normal(0, 0.01, m.nq)
                st["qvel"] = st["qvel"] + rng.normal(0, 0.01, m.nv)
            a, b = om.make_data(), rm.make_data()
            a.set_state(**st)
            b.set_state(**st)
            da = ora.calc_derivatives(om, a, cost_fn=cfn, nthread=nthread)
            db = ora.calc_derivatives(rm, b, cost_fn=cfn, use_ref=True, nthread=nthread)
            assert np.array_equal(da, db), (name, trial, np.abs(da - db).max())


@needs_ref
def test_reference_driver_restores_solver_options(ia, ora):
    """mjderivative.cpp:231-254 mutates m->opt during FD and restores it"""
    m, rm = _models(ia, ora, "hopper", ora.ref_lib())
    d = rm.make_data()
    ora.calc_derivatives(rm, d, cost_fn="ora_cost_pendulum", use_ref=True)
    import ctypes
    it, tol = ctypes.c_int(), ctypes.c_double()
    rm.lib.L.ora_get_solver(rm.m, ctypes.byref(it), ctypes.byref(tol))
    assert (it.value, tol.value) == (100, 1e-8)


@needs_ref
def test_cpMjData_and_update_cpp(ia, ora):
    """util.cpp cpMjData and update.cpp forwardStep/forwardFrame (the reference's, on restated physics)"""
    for name, dt in (("inverted_pendulum", 0.02), ("hopper", 0.002)):
        m, rm = _models(ia, ora, name, ora.ref_lib())
        a, b = rm.make_data(), rm.make_data()
        a.step(7)
        rm.lib.L.ref_cpMjData(rm.m, b.d, a.d)
        for k in ("qpos", "qvel", "warm", "ctrl"):
            assert np.array_equal(a.arr(k), b.arr(k))
        assert a.time == b.time
        # forwardFrame: steps until 1/60 s elapsed
        c = rm.make_data()
        c.set_state(**a.state())
        rm.lib.L.ref_forwardFrame(rm.m, c.d)
        n = 1
        while n * dt < 1.0 / 60.0 - 1e-12:
            n += 1
        a.step(n)
        assert np.array_equal(a.arr("qpos"), c.arr("qpos"))
        rm.lib.L.ref_forwardStep(rm.m, c.d)
        a.step(1)
        assert np.array_equal(a.arr("qvel"), c.arr("qvel"))
