"""Register / spill / scratch / LDS report of every kernel in a built library,
read from the gfx950 code objects' metadata (no recompilation, no truncation).

The HIP fat binary (.hip_fatbin section) holds one clang offload bundle per
translation unit; each bundle's gfx950 entry is an ELF code object whose
AMDGPU metadata note lists, per kernel, the registers, spills, private
(scratch) segment and static LDS the compiler assigned.

  python3 tools/resource_report.py [lib.so] [--grep SUBSTR]
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def bundles(fatbin: bytes):
    """every gfx950 code object in the fat binary"""
    out = []
    pos = 0
    while True:
        pos = fatbin.find(MAGIC, pos)
        if pos < 0:
            return out
        p = pos + len(MAGIC)
        n = int.from_bytes(fatbin[p:p + 8], "little")
        p += 8
        for _ in range(n):
            off, size, tl = (int.from_bytes(fatbin[p + 8 * i:p + 8 * i + 8], "little") for i in range(3))
            triple = fatbin[p + 24:p + 24 + tl].decode()
            p += 24 + tl
            if "gfx950" in triple and size:
                out.append(fatbin[pos + off:pos + off + size])
        pos += len(MAGIC)


def kernels(code_object: bytes):
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(code_object)
        f.flush()
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", f.name], capture_output=True, text=True,
                               check=True).stdout
    # the kernels list in the YAML-like dump: blocks starting at "- .agpr_count" / ".args"
    out = []
    for blk in re.split(r"\n  - \.", notes):
        name = re.search(r"\.name:\s+(\S+)", blk)
        if not name or ".vgpr_count" not in blk:
            continue

        def g(k):
            m = re.search(r"(?:^|\.)" + k + r":\s+(\d+)", blk)
            return int(m.group(1)) if m else None
        out.append({"name": name.group(1), "vgpr": g("vgpr_count"), "agpr": g("agpr_count"), "sgpr": g("sgpr_count"),
                    "vgpr_spill": g("vgpr_spill_count"), "sgpr_spill": g("sgpr_spill_count"),
                    "scratch": g("private_segment_fixed_size"), "lds_static": g("group_segment_fixed_size")})
    return out


def demangle(names):
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    return r.stdout.splitlines() if r.returncode == 0 else names


def main():
    args = sys.argv[1:]
    grep = None
    if "--grep" in args:
        i = args.index("--grep")
        grep = args[i + 1]
        del args[i:i + 2]
    lib = args[0] if args else os.path.join(ROOT, "ilqg-mujoco_amd", "lib", "libilqg_amd.so")
    with tempfile.NamedTemporaryFile(suffix=".fatbin") as f:
        subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={f.name}", lib, "/dev/null"],
                       check=True)
        fat = open(f.name, "rb").read()
    rows = []
    for co in bundles(fat):
        rows += kernels(co)
    rows = [r for r in rows if not r["name"].endswith(".kd")]
    names = demangle([r["name"] for r in rows])
    print(f"# {os.path.relpath(lib, ROOT)}: {len(rows)} kernels (gfx950 code-object metadata; vgpr = the unified "
          f"count, arch VGPRs + AGPRs; scratch = private segment bytes per lane; lds = static group segment, the "
          f"dynamic LDS is set at launch)")
    print(f"{'vgpr':>5} {'agpr':>5} {'sgpr':>5} {'vspill':>6} {'sspill':>6} {'scratch':>7} {'lds':>6}  kernel")
    for r, n in sorted(zip(rows, names), key=lambda x: x[1]):
        if grep and grep not in n:
            continue
        n = re.sub(r"\(anonymous namespace\)::", "", n)
        n = re.sub(r"ilqg::(stat::|coopf?::)?", "", n)
        n = n[:n.index("(")] if "(" in n else n  # the kernel and its template arguments
        print(f"{r['vgpr']:>5} {r['agpr']:>5} {r['sgpr']:>5} {r['vgpr_spill']:>6} {r['sgpr_spill']:>6} "
              f"{r['scratch']:>7} {r['lds_static']:>6}  {n}")


if __name__ == "__main__":
    main()
