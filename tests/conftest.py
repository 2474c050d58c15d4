import os
import subprocess
import sys

import numpy as np
import pytest

# torch bundles a HIP runtime of its own and must initialise before the
# library's in a process that uses both (ilqg_amd.lib): tests that hand solver
# memory to torch (seed_shard.device_view) run after tests that loaded the library
try:
    import torch
    torch.cuda.is_available()
except Exception:  # torch absent: the tests that need it skip or fail on their own
    pass

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ilqg-mujoco_amd")
ORACLE = os.path.join(ROOT, "oracle")
GOLDEN = os.path.join(ROOT, "tests", "golden")
MODELS = os.path.join(PKG, "models")
for p in (PKG, ORACLE):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")


def _ensure_built():
    """Build the oracle and the HIP library if the .so files are missing (hipcc
    cross-compiles gfx950 without a GPU).  On the GPU box the prebuilt files
    from the build container are used as-is."""
    if not os.path.exists(os.path.join(ORACLE, "liboracle.so")):
        subprocess.run(["make", "-s", "-C", ORACLE, "all"], check=True)
    if os.path.exists("/root/reference/src/mjderivative.cpp") and not os.path.exists(
            os.path.join(ORACLE, "_ref", "libilqg_ref.so")):
        subprocess.run(["make", "-s", "-C", ORACLE, "ref"], check=True)
    if not all(os.path.exists(os.path.join(PKG, *p)) for p in
               (("lib", "libilqg_amd.so"), ("lib", "libilqg_mujoco.so"), ("bin", "ilqg_headless"))):
        subprocess.run(["make", "-s", "-j8", "-C", PKG], check=True)
    if os.path.exists("/root/reference/src/inverted_pendulum/inverted_pendulum.cpp") and not os.path.exists(
            os.path.join(ORACLE, "_ref", "ref_pendulum_legacy")):
        subprocess.run(["make", "-s", "-C", ORACLE, "legacy"], check=True)


_ensure_built()


def model_path(name):
    return os.path.join(MODELS, name + ".xml")


@pytest.fixture(scope="session")
def ia():
    import ilqg_amd
    return ilqg_amd


@pytest.fixture(scope="session")
def ora():
    import oracle
    return oracle


def has_ref():
    return os.path.exists(os.path.join(ORACLE, "_ref", "libilqg_ref.so"))


def load_golden(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}
