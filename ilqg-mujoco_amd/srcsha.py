"""Digest of the sources libilqg_amd.so is built from (csrc/**, Makefile).

The Makefile compiles it into the library (`ilqg_source_sha()`, generated
build/srcsha.cpp) and `ilqg_amd.lib()` compares it with the digest of the
sources beside the library, so a stale prebuilt `.so` is refused instead of
being measured under a fresh source hash.  Standard library only: the build
runs it before anything else is importable.

  python3 srcsha.py        prints the digest (16 hex digits)
"""
import hashlib
import os

_HERE = os.path.dirname(os.path.abspath(__file__))


def source_sha(root: str = _HERE) -> str:
    h = hashlib.sha256()
    files = [os.path.join(root, "Makefile")]
    for d, _, fs in sorted(os.walk(os.path.join(root, "csrc"))):
        files += [os.path.join(d, f) for f in sorted(fs) if f.endswith((".h", ".hip", ".cpp", ".map"))]
    for f in files:
        h.update(os.path.relpath(f, root).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(source_sha())
