"""Offline schedule study of the fused FD sweep (no GPU): replays the measured
per-item durations of one launch (tools/fused_timeline.py with TL_SAVE=...)
through a slot model of the machine and reports the makespan of ticket
orders the kernel could use.

  python tools/sched_sim.py gpurun_out/r5g/tl.npz [slots]

Model: `slots` concurrent teams (default: the launch's measured steady-state
concurrency); a team takes the next item of its order when a slot frees; a
column item cannot start before its centre ends (it would wait in its slot:
the model charges the wait).  Item durations are the measured ones (so
co-scheduling effects are frozen at their measured values).
Orders:
  identity      centres, then columns point-major (the kernel's default)
  centre-long   centres; then, as centres finish, the columns of points whose
                centre ran longer than THR us first (a dynamic queue), the rest
                point-major
  lpt-oracle    centres, then columns longest-first by their true duration
                (a bound no predictor reaches)
  split-long    identity, with the columns of long-centre points as two
                halves of 0.68 x the column each (the measured cost of a half)
"""
import heapq
import sys

import numpy as np


def simulate(order, dur, centre_end_dep, nC, slots):
    """order: item ids in dispatch order; returns (makespan, end times)"""
    free = [0.0] * slots
    heapq.heapify(free)
    end = np.zeros(len(dur))
    for it in order:
        t = heapq.heappop(free)
        start = t
        if it >= nC:
            start = max(t, end[centre_end_dep[it]])  # waits in its slot for the centre
        end[it] = start + dur[it]
        heapq.heappush(free, end[it])
    return end.max(), end


def main():
    d = np.load(sys.argv[1])
    st, en, ok, role = d["start"], d["end"], d["ok"], d["role"]
    S, P, ncw = int(d["S"]), int(d["P"]), int(d["ncw"])
    nC = S * P
    n = len(st)
    dur = np.where(ok, en - st, np.median(en - st))
    # centre of column item u: nC + (p S + s) ncw + w -> p S + s
    dep = np.zeros(n, dtype=np.int64)
    dep[nC:] = (np.arange(nC, n) - nC) // ncw
    span = en[ok].max() - st[ok].min()
    conc = dur[ok].sum() / span
    slots = int(sys.argv[2]) if len(sys.argv) > 2 else int(round(np.percentile(
        [((st[ok] <= t) & (en[ok] > t)).sum() for t in np.linspace(st[ok].min(), en[ok].max(), 200)[20:120]], 90)))
    print(f"items {n} (centres {nC}), measured span {span:.0f} us, mean concurrency {conc:.0f}, model slots {slots}")
    cdur = dur[:nC]
    cols = np.arange(nC, n)
    # correlation of a point's centre duration with its columns' mean / max
    cmean = dur[nC:].reshape(nC, ncw).mean(1)
    cmax = dur[nC:].reshape(nC, ncw).max(1)
    print(f"corr(centre, mean of its columns) {np.corrcoef(cdur, cmean)[0, 1]:.3f}, "
          f"corr(centre, max of its columns) {np.corrcoef(cdur, cmax)[0, 1]:.3f}")
    ident = np.arange(n)
    mk, _ = simulate(ident, dur, dep, nC, slots)
    print(f"identity order: makespan {mk:.0f} us (measured {span:.0f})")
    # dynamic centre-informed order: simulate with an event loop
    for thr in (150, 250, 400, 600):
        mk2 = sim_centre_long(dur, dep, nC, ncw, slots, thr)
        print(f"centre-long thr {thr:4d} us: makespan {mk2:.0f} us")
    lpt = np.concatenate([np.arange(nC), cols[np.argsort(-dur[nC:], kind="stable")]])
    mk3, _ = simulate(lpt, dur, dep, nC, slots)
    print(f"lpt-oracle: makespan {mk3:.0f} us")
    print(f"bound: total team-us / slots = {dur.sum() / slots:.0f} us")
    for thr in (150, 300, 500, 800):
        mk4, work = split_long(sys.argv[1], thr, slots)
        print(f"split-long thr {thr:4d} us: makespan {mk4:.0f} us, team-us x{work:.3f}")


def sim_centre_long(dur, dep, nC, ncw, slots, thr):
    """centres first; a finished centre longer than thr pushes its columns to a
    priority queue that free slots serve before the point-major queue"""
    n = len(dur)
    free = [(0.0, k) for k in range(slots)]
    heapq.heapify(free)
    end = np.full(n, np.inf)
    taken = np.zeros(n, dtype=bool)
    long_pt = np.zeros(nC, dtype=np.int8)  # 0 pending, 1 long (priority), 2 claimed by the regular queue
    prio = []  # (ready time, item)
    reg = nC   # next regular column item
    ci = 0     # next centre
    done = 0
    while done < n:
        t, k = heapq.heappop(free)
        # centres finished by now push their columns
        item = None
        if ci < nC:
            item = ci
            ci += 1
            start = t
        else:
            # priority items whose centre has ended by t
            while prio and prio[0][0] <= t and taken[prio[0][1]]:
                heapq.heappop(prio)
            if prio and prio[0][0] <= t:
                _, item = heapq.heappop(prio)
                start = t
            else:
                while reg < n and (taken[reg] or long_pt[dep[reg]] == 1):
                    reg += 1
                if reg < n:
                    item = reg
                    reg += 1
                    p = dep[item]
                    if long_pt[p] == 0:
                        long_pt[p] = 2
                    start = max(t, end[p])
                elif prio:
                    rt, item = heapq.heappop(prio)
                    start = max(t, rt)
                else:
                    # wait for a centre to finish and push (nothing else left)
                    heapq.heappush(free, (t + 1.0, k))
                    continue
        taken[item] = True
        end[item] = start + dur[item]
        done += 1
        if item < nC and dur[item] > thr and long_pt[item] == 0:
            long_pt[item] = 1
            for w in range(ncw):
                heapq.heappush(prio, (end[item], nC + item * ncw + w))
        heapq.heappush(free, (end[item], k))
    return end.max()


def split_long(path, thr, slots, frac=0.68):
    """identity order, but the columns of points whose centre ran longer than
    thr us run as two halves of frac x the column's duration each (measured:
    a half costs 0.6-0.7 of the whole column, DESIGN.md 'Column halves')"""
    d = np.load(path)
    st, en, ok = d["start"], d["end"], d["ok"]
    S, P, ncw = int(d["S"]), int(d["P"]), int(d["ncw"])
    nC = S * P
    dur = np.where(ok, en - st, np.median(en - st))
    items, deps = list(dur[:nC]), list(range(nC))
    for u in range(nC, len(dur)):
        g = (u - nC) // ncw
        if dur[g] > thr:
            items += [frac * dur[u], frac * dur[u]]
            deps += [g, g]
        else:
            items.append(dur[u])
            deps.append(g)
    items, deps = np.array(items), np.array(deps)
    mk, _ = simulate(np.arange(len(items)), items, deps, nC, slots)
    return mk, items.sum() / dur.sum()



if __name__ == "__main__":
    main()
