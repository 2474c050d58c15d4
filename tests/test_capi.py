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


def test_library_carries_source_digest(ia):
    """binary provenance: the library in the tree was built from the sources
    beside it (the digest compiled in equals srcsha.py's of csrc/** + Makefile)"""
    lib = ia.lib()
    lib.ilqg_source_sha.restype = ctypes.c_char_p
    assert lib.ilqg_source_sha().decode() == ia.source_sha()
    assert re.fullmatch(r"[0-9a-f]{16}", ia.source_sha())


def test_stale_library_is_refused(tmp_path):
    """a library whose compiled-in digest differs from the sources (a stale
    prebuilt .so pushed beside newer sources) is refused with IlqgError before
    anything runs on it"""
    src = tmp_path / "stale.c"
    src.write_text('const char* ilqg_source_sha(void) { return "0123456789abcdef"; }\n'
                   'int ilqg_version(void) { return 999; }\n')
    so = tmp_path / "libstale.so"
    subprocess.run(["gcc", "-shared", "-fPIC", "-o", str(so), str(src)], check=True)
    code = ("import sys; sys.path.insert(0, %r); import ilqg_amd as ia\n"
            "try:\n    ia.lib()\nexcept ia.IlqgError as e:\n    print('REFUSED', e)\nelse:\n    print('LOADED')\n") % PKG
    r = subprocess.run(["python3", "-c", code], env=dict(os.environ, ILQG_LIB=str(so)), capture_output=True,
                       text=True, timeout=120)
    assert "REFUSED" in r.stdout and "0123456789abcdef" in r.stdout, r.stdout + r.stderr


def test_model_sizes_and_blob(ia):
    m = ia.Model.load(model_path("hopper"))
    b = m.blob()
    assert b[:8] == b"ILQGMDL1" and len(b) > 1000
    assert m.D == 6 * 15 + 12 + 3
