"""Diagnostic build only: timeline of one fused FD sweep + streamed backward pass
(the bench workload: hopper H=500, 8 seeds x 8 alphas): per FD team its start,
end and CU; concurrency over time, team durations per role, CUs used.
  ILQG_LIB=ilqg-mujoco_amd/lib/libilqg_amd_diag.so python tools/fused_timeline.py [S]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ilqg-mujoco_amd"))
import ilqg_amd as ia  # noqa: E402
import workloads  # noqa: E402

TL_N = 131072
L = ia.lib()
buf = (ctypes.c_ulonglong * (3 * TL_N + 128 + 8 * 512))()
S = int(sys.argv[1]) if len(sys.argv) > 1 else 8
m = ia.Model.load(workloads.model_file("hopper"))
g = ia.ILQR(m, workloads.hopper_dmain(m, S, sigma=0.01), 500, ia.HOPPER_COST,
            alphas=tuple(2.0 ** -i for i in range(8)), select="min_cost")
g.iterate()
g.synchronize()
L.ilqg_debug_timeline(buf, 1)
g.set_timing(True)
g.timing()
g.iterate()
g.synchronize()
t = g.timing()
L.ilqg_debug_timeline(buf, 0)
a = np.frombuffer(buf, dtype=np.uint64)
nv, nu, P = m.nv, m.nu, 501
ntm = nu + 2 * nv
HALVES = int(os.environ.get("ILQG_FD_HALVES", "0")) != 0  # every column as two items (+, -)
ncw = 2 * ntm if HALVES else ntm  # column items per (seed, point)
n_items = S * P * (1 + ncw)
tl = a[: 3 * TL_N].reshape(TL_N, 3)[:n_items]
tb = a[3 * TL_N:3 * TL_N + 128].reshape(64, 2)[:S].astype(np.int64)
bstep = a[3 * TL_N + 128:].reshape(8, 512).astype(np.int64)
st, en, hw = tl[:, 0].astype(np.int64), tl[:, 1].astype(np.int64), tl[:, 2]
ok = (st > 0) & (en > 0)
print(f"S={S}: fused launch {t['fd_backward'][0]:.3f} ms (HIP events); items {n_items}, recorded {ok.sum()}")
t0 = min(st[ok].min(), tb[:, 0].min())
us = lambda x: (x - t0) / 100.0  # noqa: E731  s_memrealtime: 100 MHz
dur = (en - st) / 100.0
u = np.arange(n_items)
nC = S * P
role = np.where(u < nC, 0, 0)
w = (u - nC) % (S * ncw) % ncw
if HALVES:
    w = w // 2
role = np.where(u < nC, 0, np.where(w < nu, 3, np.where(w < nu + nv, 1, 2)))
names = {0: "C (centre)", 1: "V (qvel col)", 2: "Q (qpos col)", 3: "U (ctrl col)"}
for r in (0, 3, 1, 2):
    d = dur[(role == r) & ok]
    print(f"  {names[r]:14s} teams {d.size:6d}  duration us: mean {d.mean():7.1f}  p50 {np.median(d):7.1f}  "
          f"p99 {np.percentile(d, 99):7.1f}  max {d.max():7.1f}")
print(f"  team-us in total {dur[ok].sum():.0f}; span of FD teams {us(en[ok].max()) - us(st[ok].min()):.0f} us "
      f"-> mean concurrency {dur[ok].sum() / (us(en[ok].max()) - us(st[ok].min())):.0f} teams")
for s in range(S):
    print(f"  backward role {s}: start {us(tb[s, 0]):7.1f} us, end {us(tb[s, 1]):7.1f} us")
# concurrency over time in 50-us buckets
T_end = us(max(en[ok].max(), tb[:, 1].max()))
edges = np.arange(0, T_end + 50, 50)
conc = []
for b0 in edges[:-1]:
    b1 = b0 + 50
    ov = np.clip(np.minimum(us(en[ok]), b1) - np.maximum(us(st[ok]), b0), 0, None)
    conc.append(ov.sum() / 50)
print("  concurrency per 50 us: " + " ".join(f"{c:.0f}" for c in conc))
# dispatch front: tickets started per 50 us
starts = np.histogram(us(st[ok]), bins=edges)[0]
print("  team starts per 50 us: " + " ".join(str(x) for x in starts))
# per point: time the record is complete (all teams of (s, p) ended), seed 0
pts = []
for p in range(P):
    idx = [p * S + 0] + [nC + p * S * ncw + 0 * ncw + k for k in range(ncw)]
    pts.append(us(en[idx].max()))
pts = np.array(pts)
print("  seed 0 record complete (us) at points 0,50,...: " + " ".join(f"{pts[p]:.0f}" for p in range(0, P, 50)))
# the recursion against its records (handoff.h g_bstep): step n of seed s needs
# record n (and prefetches n + 1); lag = step done - that record complete
for s_ in range(min(S, 8)):
    ready = np.array([us(en[[p * S + s_] + [nC + p * S * ncw + s_ * ncw + k for k in range(ncw)]].max())
                      for p in range(P)])
    done = bstep[s_, 1:P]
    if not np.all(done > 0):
        continue
    dn = us(done)
    lag = dn - ready[1:P]
    last_rec = ready.max()
    behind = int((dn > last_rec).sum())
    step_us = np.diff(dn)
    print(f"  seed {s_} recursion: last record {last_rec:.0f} us, last step {dn[-1]:.0f} us "
          f"({dn[-1] - last_rec:.0f} us after it, {behind} steps done after it); step time median "
          f"{np.median(step_us):.2f} us, over the last 50 steps {np.mean(step_us[-50:]):.2f} us; "
          f"lag behind its record: median {np.median(lag):.0f} us, max {lag.max():.0f} us")
cu = hw[ok]
xcc = (cu >> 32) & 0xF
hwid = cu & 0xFFFFFFFF
cu_id = (hwid >> 8) & 0xF
sh = (hwid >> 12) & 1
se = (hwid >> 13) & 0x7
key = xcc * 1000 + se * 100 + sh * 16 + cu_id
print(f"  distinct (xcc, se, sh, cu) used: {len(np.unique(key))}; xcc histogram {np.bincount(xcc.astype(np.int64))}")
if os.environ.get("TL_SAVE"):
    # raw per-item start / end (us from the first start) and role, for offline schedule studies
    np.savez(os.environ["TL_SAVE"], start=us(st), end=us(en), ok=ok, role=role, S=S, P=P, ncw=ncw,
             tb=np.array([[us(tb[s_, 0]), us(tb[s_, 1])] for s_ in range(S)]))
del g
