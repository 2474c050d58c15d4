"""C ABI: the HIP library loads without a GPU, exports every symbol
include/ilqg_amd.h declares, and its device entry points fail loudly (no CPU
fallback) when no device is present."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import PKG, ROOT, model_path

HEADER = os.path.join(ROOT, "include", "ilqg_amd.h")


def declared():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(ilqg_[a-z0-9_]+)\s*\(", txt)))


def test_header_symbols_exported(ia):
    lib = ia.lib()
    names = declared()
    assert len(names) >= 25
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) <= set(ia.EXPORTS) | {"ilqg_solver_stream"}


def test_only_api_symbols_exported():
    so = os.path.join(PKG, "lib", "libilqg_amd.so")
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True, check=True).stdout
    syms = [l.split()[-1] for l in out.splitlines() if " T " in l]
    assert syms and all(s.startswith("ilqg_") for s in syms), syms


def test_device_kernels_built_for_gfx950():
    """the fat binary carries a gfx950 code object (and no other target)"""
    data = open(os.path.join(PKG, "lib", "libilqg_amd.so"), "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
    assert not re.search(rb"amdgcn-amd-amdhsa--gfx9[0-4][0-9a-f]", data)


def test_version_and_errors(ia):
    lib = ia.lib()
    assert lib.ilqg_version() >= 100
    h = ctypes.c_void_p()
    assert lib.ilqg_model_load_xml(None, ctypes.byref(h)) == 1  # ILQG_ERR_ARG
    assert b"null" in lib.ilqg_last_error()


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="GPU present")
def test_device_entry_points_fail_without_gpu(ia):
    m = ia.Model.load(model_path("inverted_pendulum"))
    st = m.reset_state(2)
    with pytest.raises(ia.IlqgError, match="code 5"):  # ILQG_ERR_NODEVICE
        m.step(st)
    with pytest.raises(ia.IlqgError):
        ia.ILQR(m, st, 10, ia.PENDULUM_COST)


def test_model_sizes_and_blob(ia):
    m = ia.Model.load(model_path("hopper"))
    b = m.blob()
    assert b[:8] == b"ILQGMDL1" and len(b) > 1000
    assert m.D == 6 * 15 + 12 + 3
