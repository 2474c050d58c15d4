"""CPU: the host code under AddressSanitizer + UndefinedBehaviorSanitizer.
tests/sanitize_main.cpp drives the product's MJCF compiler / setConst / blob
writer (ilqg-mujoco_amd/csrc/model) over every bundled model and two
malformed documents, then the oracle (oracle/*.c) -- physics, the FD driver
and the iLQR restatement with line search -- on the compiled blob; the legacy
C++ boundary (csrc/legacy/legacy.cpp) is compiled with the same flags (its
calls need a GPU, so only its build is checked here).  Any sanitizer report
fails the test (halt_on_error)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ilqg-mujoco_amd")
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_host_code_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "sanitize_main")
    src = [os.path.join(ROOT, "tests", "sanitize_main.cpp"),
           os.path.join(PKG, "csrc", "model", "mjcf.cpp"), os.path.join(PKG, "csrc", "model", "setconst.cpp")]
    objs = []
    for c in ("mjsub.c", "ilqr_ora.c", "ora_api.c"):
        o = str(tmp_path / (c + ".o"))
        subprocess.run(["gcc", "-std=c99", "-ffp-contract=off", "-fopenmp", *SAN, "-I" + os.path.join(ROOT, "oracle", "include"),
                        "-I" + os.path.join(ROOT, "include"), "-c", os.path.join(ROOT, "oracle", c), "-o", o], check=True)
        objs.append(o)
    subprocess.run(["g++", "-std=c++20", "-ffp-contract=off", "-fopenmp", *SAN, "-I" + os.path.join(ROOT, "include"),
                    "-I" + os.path.join(PKG, "csrc", "model"), "-I" + os.path.join(PKG, "csrc"),
                    "-I" + os.path.join(ROOT, "oracle"), "-I" + os.path.join(ROOT, "oracle", "include"),
                    *src, *objs, "-o", exe, "-lm"], check=True)
    models = [os.path.join(PKG, "models", n + ".xml") for n in ("inverted_pendulum", "hopper", "humanoid")]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe, *models], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr
    assert r.stdout.count("nq=") == 3


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_legacy_layer_builds_with_sanitizers(tmp_path):
    subprocess.run(["g++", "-std=c++17", "-ffp-contract=off", *SAN, "-fPIC", "-I" + os.path.join(ROOT, "include"),
                    "-I" + os.path.join(ROOT, "include", "legacy"), "-c",
                    os.path.join(PKG, "csrc", "legacy", "legacy.cpp"), "-o", str(tmp_path / "legacy.o")], check=True)
