"""Synthetic inputs of the BASELINE.json configs, built
with the product's own GPU physics.

  cfg1/2  inverted_pendulum: mj_resetData, 10 passive steps
          (src/inverted_pendulum/inverted_pendulum.cpp:12-13)
  cfg3    hopper: reset, 500 passive steps, ctrl -= 0.1 (tst/test_derivatives.cpp:38-47)
  cfg4    cfg3 state + N(0, 0.01^2) on qpos and qvel per seed, from a fixed
          splitmix64 + Box-Muller stream (not std::normal_distribution)
"""
from __future__ import annotations

import math
import os

import numpy as np

import ilqg_amd as ia

HERE = os.path.dirname(os.path.abspath(__file__))
MODEL_DIR = os.path.join(HERE, "models")
LINESEARCH_ALPHAS = tuple(2.0 ** -i for i in range(8))  # cfg3: {2^-i, i=0..7}


def model_file(name: str) -> str:
    return os.path.join(MODEL_DIR, name + ".xml")


def splitmix64(state: int):
    while True:
        state = (state + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
        z = state
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
        yield z ^ (z >> 31)


def normals(seed: int, n: int) -> np.ndarray:
    """n standard normals: splitmix64 -> uniforms (53-bit) -> Box-Muller pairs"""
    g = splitmix64(seed)
    out = []
    while len(out) < n:
        u1 = ((next(g) >> 11) + 1) * 2.0 ** -53  # (0, 1]
        u2 = (next(g) >> 11) * 2.0 ** -53
        r = math.sqrt(-2.0 * math.log(u1))
        out.append(r * math.cos(2 * math.pi * u2))
        out.append(r * math.sin(2 * math.pi * u2))
    return np.array(out[:n])


def pendulum_dmain(model: "ia.Model", nseed: int = 1) -> "ia.State":
    st = model.reset_state(1)
    model.step(st, 10)
    return _tile(st, nseed)


def hopper_dmain(model: "ia.Model", nseed: int = 1, sigma: float = 0.0, seed_offset: int = 0) -> "ia.State":
    st = model.reset_state(1)
    model.step(st, 500)
    st.ctrl[:] -= 0.1
    out = _tile(st, nseed)
    if sigma > 0:
        for s in range(nseed):
            z = normals(seed_offset + s, model.nq + model.nv)
            out.qpos[s] += sigma * z[: model.nq]
            out.qvel[s] += sigma * z[model.nq:]
    return out


def _tile(st: "ia.State", n: int) -> "ia.State":
    return ia.State(np.repeat(st.time, n), np.repeat(st.qpos, n, 0), np.repeat(st.qvel, n, 0),
                    np.repeat(st.warm, n, 0), np.repeat(st.ctrl, n, 0))
