"""Summarise rocprofv3 PMC passes (tools/gpu_prof.sh) into per-kernel HBM bytes.

FETCH_SIZE / WRITE_SIZE are rocprofv3 derived counters in KiB.  Per
/opt/skills/guides/MI355X_MICROARCH.md (HBM section) FETCH_SIZE on gfx950
reports half the bytes of wide coalesced reads, so it is doubled here; that
calibration is for 16 B/lane streaming reads -- our accesses are narrower, so
the corrected figure is an upper-side estimate, not an exact byte count.
The summary records src_sha (ilqg_amd.source_sha(): the kernel sources the
counters were taken on) and, when GIT_HEAD is set, the commit; bench.py takes
roofline.traffic from the summary whose src_sha matches the code it runs.
Usage: python tools/pmc_summary.py gpurun_out/prof profiles/rNN_pmc_traffic.json"""
import collections, csv, json, os, re, sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ilqg-mujoco_amd"))
import ilqg_amd  # noqa: E402

# kernel-name alternatives per group (model-specific *_s, two-wave *2*, generic *_coop)
GROUPS = {"rollout": (("k_rollout2_s", "k_rollout_s", "k_rollout2_coop", "k_rollout_coop"),),
          "fd_sweep": (("k_fd_centre_s", "k_fd_centre_coop"), ("k_fd_cols_s", "k_fd_cols_coop")),
          "backward": (("k_backward",),), "select": (("k_select",),),
          "fd_backward": (("k_fd_fused_g", "k_fd_fused_s", "k_fd_fused_coop"),)}


def per_kernel(path, counter):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        mm = re.search(r"::(k_[a-z0-9_]+)[<(]", r["Kernel_Name"])
        if mm:
            agg[mm.group(1)].append(float(r["Counter_Value"]) * 1024.0)
    return agg


def main(src, dst):
    fetch = per_kernel(f"{src}/fetch/run_counter_collection.csv", "FETCH_SIZE")
    write = per_kernel(f"{src}/write/run_counter_collection.csv", "WRITE_SIZE")
    kern = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [])
        w = write.get(k, [])
        # the last launches are the timed-region ones (the first of a kind may be setup)
        fa = sum(f[-3:]) / max(1, len(f[-3:]))
        wa = sum(w[-3:]) / max(1, len(w[-3:]))
        kern[k] = {"launches_seen": len(f), "fetch_bytes_raw": fa, "fetch_bytes_x2": 2 * fa, "write_bytes": wa,
                   "traffic_bytes": 2 * fa + wa}
    out = {"per_kernel": kern, "note": "FETCH_SIZE doubled per the gfx950 calibration; KiB->bytes x1024",
           "src_sha": ilqg_amd.source_sha(), "head": os.environ.get("GIT_HEAD")}
    for g, alts in GROUPS.items():
        picks = [next((k for k in a if k in kern), None) for a in alts]
        if all(picks):
            out[g] = sum(kern[k]["traffic_bytes"] for k in picks)
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
