"""Summarise the SQ counter passes of tools/gpu_sqprof.sh per kernel (the last
launch of each kind = the timed iterate's).  Derived figures:
  valu_insts_per_wave   SQ_INSTS_VALU / SQ_WAVES
  f64_ops_issued        (ADD+MUL+FMA+TRANS)_F64 wave-instructions x 64 lanes
  issue_frac            SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES (a wave issuing vs resident)
  wait_frac             SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (waiting on a dependency)
  lds_frac              SQ_ACTIVE_INST_LDS / SQ_WAVE_CYCLES
  occupancy             SQ_WAVE_CYCLES / SQ_BUSY_CYCLES / (CUs x 4 SIMDs): mean resident waves per SIMD
(SQ_*_CYCLES are sampled per 4 cycles on gfx9: only ratios are used.)
Usage: python tools/sq_summary.py gpurun_out/sq profiles/r02_sq_counters.json"""
import collections
import csv
import glob
import json
import re
import sys

NCU = 256


def load(src):
    last = {}
    for path in sorted(glob.glob(f"{src}/p*/run_counter_collection.csv")):
        rows = collections.defaultdict(dict)
        for r in csv.DictReader(open(path)):
            mm = re.search(r"::(k_[a-z0-9_]+)[<(]", r["Kernel_Name"])
            if not mm:
                continue
            rows[(mm.group(1), int(r["Dispatch_Id"]))][r["Counter_Name"]] = float(r["Counter_Value"])
        for (k, disp), cs in sorted(rows.items(), key=lambda x: x[0][1]):
            last.setdefault(k, {}).update(cs)  # later dispatches overwrite: the last launch of a kind
    return last


def main(src, dst):
    out = {}
    for k, c in load(src).items():
        g = lambda n: c.get(n, 0.0)  # noqa: E731
        wc = g("SQ_WAVE_CYCLES") or 1.0
        d = dict(c)
        d["valu_insts_per_wave"] = g("SQ_INSTS_VALU") / max(1.0, g("SQ_WAVES"))
        d["f64_wave_insts"] = sum(g(f"SQ_INSTS_VALU_{x}_F64") for x in ("ADD", "MUL", "FMA", "TRANS"))
        d["issue_frac"] = g("SQ_ACTIVE_INST_ANY") / wc
        d["wait_frac"] = g("SQ_WAIT_INST_ANY") / wc
        d["valu_frac"] = g("SQ_ACTIVE_INST_VALU") / wc
        d["lds_frac"] = g("SQ_ACTIVE_INST_LDS") / wc
        if g("SQ_BUSY_CYCLES"):
            d["waves_per_simd"] = wc / g("SQ_BUSY_CYCLES") / (NCU * 4)
        out[k] = d
        print(f"{k:18s} waves {g('SQ_WAVES'):8.0f} VALU/wave {d['valu_insts_per_wave']:10.0f} "
              f"issue {d['issue_frac']:.2f} wait {d['wait_frac']:.2f} valu {d['valu_frac']:.2f} lds {d['lds_frac']:.2f} "
              f"waves/SIMD {d.get('waves_per_simd', 0):.2f}")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
