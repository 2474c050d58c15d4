"""The instrumented flop-counting oracle (oracle/flops): same
arithmetic as the plain oracle, and the committed counts in
tests/fixtures/flops.json reproduce."""
import importlib.util
import json
import os

import numpy as np
import pytest

from conftest import ROOT, load_golden, model_path

FLOPS_SO = os.path.join(ROOT, "oracle", "flops", "liboracle_flops.so")
FIX = os.path.join(ROOT, "tests", "fixtures")


@pytest.fixture(scope="module")
def flib(ora):
    if not os.path.exists(FLOPS_SO):
        import subprocess
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "flops"], check=True)
    return ora.Lib(FLOPS_SO)


def test_counted_build_same_bits(ia, ora, flib):
    g = load_golden("fd_hopper.npz")
    m = ia.Model.load(model_path("hopper"))
    for lib in (ora.oracle_lib(), flib):
        lib.L.ora_set_cost_desc(ora.CostDesc.from_cost(ia.HOPPER_COST, m.nq, m.nv, m.nu))
    out = []
    for lib in (ora.oracle_lib(), flib):
        om = ora.OModel(m.blob(), lib)
        d = om.make_data()
        d.set_state(time=g["time"][0], qpos=g["qpos"][0], qvel=g["qvel"][0], warm=g["warm"][0], ctrl=g["ctrl"][0])
        out.append(ora.calc_derivatives(om, d, cost_fn="ora_cost_desc_fn", nthread=1))
    assert np.array_equal(out[0], out[1])
    assert np.array_equal(out[0], g["deriv"][0])


def test_flops_json_reproduces(flib):
    spec = importlib.util.spec_from_file_location("make_flops", os.path.join(FIX, "make_flops.py"))
    mf = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mf)
    with open(os.path.join(FIX, "flops.json")) as f:
        ref = json.load(f)["models"]
    cnt = mf.Counter(flib)
    for name in ("inverted_pendulum", "hopper"):
        r = mf.count_model(name, cnt, flib)
        for k in ("fd_point", "step", "riccati_step"):
            assert r[k]["flops"] == ref[name][k]["flops"], (name, k)
