"""The oracle against the committed iLQR known-answer fixtures (SURVEY.md §8c
items 2-4; tests/golden/make_golden_ilqr.py).  CPU only: these pin the
checker itself, so a regression in the oracle cannot move both sides of a GPU
parity test together.  The iterate fixtures were written by the reference's own
calcMJDerivatives (oracle/_ref); here the oracle's restated FD driver must
reproduce them bit for bit."""
import importlib.util
import os

import numpy as np
import pytest

from conftest import GOLDEN, load_golden, model_path


def _gen():
    spec = importlib.util.spec_from_file_location("make_golden_ilqr", os.path.join(GOLDEN, "make_golden_ilqr.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _traj(g, pre):
    return {k: g[pre + k] for k in ("time", "qpos", "qvel", "warm", "ctrl")}


@pytest.mark.parametrize("fixture", ["riccati_pendulum.npz", "riccati_hopper.npz"])
def test_oracle_riccati_fixture(ia, ora, fixture):
    g = load_golden(fixture)
    m = ia.Model.load(model_path(str(g["model"])))
    om = ora.OModel(m.blob())
    out = _gen().riccati_reference(om, _traj(g, "traj_"), g["deriv"])
    for k in ("K", "k", "V", "v"):
        assert np.array_equal(out[k], g[k]), k


@pytest.mark.parametrize("fixture", ["iterate_pendulum_H20.npz", "iterate_pendulum_H100.npz"])
def test_oracle_iterate_fixture(ia, ora, fixture):
    g = load_golden(fixture)
    m = ia.Model.load(model_path("inverted_pendulum"))
    om = ora.OModel(m.blob())
    d = om.make_data()
    d.step(10)
    assert np.array_equal(d.arr("qpos"), g["dmain_qpos"][0]) and np.array_equal(d.arr("qvel"), g["dmain_qvel"][0])
    il = ora.OILQR(om, d, int(g["horizon"]), cost_fn="ora_cost_pendulum")  # restated FD driver
    il.set_dinit(d)
    for _ in range(int(g["iters"])):
        il.iterate()
    t, a = il.traj(), il.arrays()
    for k, v in t.items():
        assert np.array_equal(v, g["traj_" + k]), k
    for k in ("K", "k", "V", "v", "deriv"):
        assert np.array_equal(a[k], g[k]), k


def test_oracle_rollout_fixture(ia, ora):
    g = load_golden("rollout_hopper_H100.npz")
    m = ia.Model.load(model_path("hopper"))
    om = ora.OModel(m.blob())
    om.lib.L.ora_set_cost_desc(ora.CostDesc.from_cost(ia.HOPPER_COST, m.nq, m.nv, m.nu))
    d = om.make_data()
    d.set_state(**{k: g["dmain_" + k][0] for k in ("time", "qpos", "qvel", "warm", "ctrl")})
    il = ora.OILQR(om, d, int(g["horizon"]), cost_fn="ora_cost_desc_fn")
    il.set_dinit(d)
    for k, v in il.traj().items():
        assert np.array_equal(v, g["nominal_" + k]), "nominal " + k
    il.set_gains(g["K"], g["k"])
    il.forward_pass()
    for k, v in il.traj().items():
        assert np.array_equal(v, g["traj_" + k]), k
