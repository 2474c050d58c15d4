"""Per-stage cycle breakdown of the cooperative physics (diagnostic build).
ILQG_LIB=ilqg-mujoco_amd/lib/libilqg_amd_diag.so python tools/stamps.py"""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ilqg-mujoco_amd"))
import ilqg_amd as ia, workloads
NAMES = {10: " nt: start (warm/smooth choice, factor)", 0: "kinematics", 1: "com_pos", 2: "trn+crb", 3: "factor_ld(M)", 4: "collision", 5: "make_constraint",
         6: "fwd_velocity", 7: "fwd_acceleration", 8: "fwd_constraint(newton)", 9: "integrator",
         11: " kin: joint quats", 12: " kin: lane-0 chain / position chain", 13: " kin: body frames", 14: " nt: chol solve",
         15: " nt: Mv,Jv", 16: " nt: linesearch", 17: " nt: update", 18: " nt: cost+grad", 19: " nt: hessian",
         20: "empty sync", 21: "empty sync 2", 22: " kin: quat chain (lane 0)", 23: " kin: rotations (lanes)",
         24: "A: barrier 1 (wait for B)", 25: "A: barrier 2", 26: "A: barrier 3", 27: "A: barrier 4", 28: "A: barrier 5",
         32: "B: barrier 1 (wait for A kinematics)", 33: "B: collision", 34: "B: barrier 2", 35: "B: make_constraint",
         36: "B: barrier 3", 37: "B: passive+aref / contact rows+aref", 38: "B: euler prefactor / M and M+hD factors", 39: "B: barrier 4 (A com vel + RNE)",
         40: "B: barrier 6 (end of step)", 41: "B: control law + record", 42: "B: factor_ld(M) / limit rows+passive+act",
         43: "B: barrier 5",
         29: "A: barrier 5b (Euler factor)", 30: "B: Newton warm-start prep", 31: " nt: hessian build (M + J'DJ)"}
# the third wave of a three-wave rollout team (STAMPC, its own clock): partitions that wave's time
W2 = {48: "W2: limit rows+passive+frames", 49: "W2: barrier 1", 50: "W2: collision (non-plane pairs)",
      51: "W2: barrier 2", 52: "W2: barrier 3 (idle in phase 3)", 53: "W2: factors of M and M+hD",
      54: "W2: barrier 4", 55: "W2: barrier 5 (idle in phase 5)", 56: "W2: barrier 6 (end of step)",
      57: "W2: velocity stage (phase 3)"}
MFMA = len(sys.argv) > 2 and sys.argv[2] == "mfma"  # the backward section on the MFMA engine
L = ia.lib()
acc = (ctypes.c_ulonglong * 64)(); cnt = (ctypes.c_ulonglong * 64)()
m = ia.Model.load(workloads.model_file(sys.argv[1] if len(sys.argv) > 1 else "hopper"))
if m.nq != m.nv:  # humanoid, cfg 5's state (tools/cfg5_probe.py)
    dmain = m.reset_state(1)
    dmain.qpos[0, 2] = 1.4
    g = ia.ILQR(m, dmain, 200, ia.HUMANOID_COST)
else:
    dmain = workloads.hopper_dmain(m, 1) if m.nv == 6 else workloads.pendulum_dmain(m, 1)
    g = ia.ILQR(m, dmain, 500 if m.nv == 6 else 200, ia.HOPPER_COST if m.nv == 6 else ia.PENDULUM_COST)
g.iterate(); g.synchronize()
g.set_timing(True)
ls = (ctypes.c_ulonglong * 8)()
for what, fn, rd, rls in (("rollout (1 seed)", g.forward_pass, L.ilqg_debug_stamps, L.ilqg_debug_ls_rollout),
                          ("fd sweep", g.fd_sweep, L.ilqg_debug_stamps_fd, L.ilqg_debug_ls_fd)):
    rd(acc, cnt, 1)
    rls(ls, 1)
    g.timing()
    fn(); g.synchronize()
    tm = g.timing()
    rd(acc, cnt, 1)
    rls(ls, 1)
    if ls[0]:
        print(f"   line searches (all workgroups): {ls[0]} calls, {ls[1] / ls[0]:.2f} iterations per call, "
              f"{ls[2]} ran to LS_ITER, {ls[3] / ls[0]:.2f} constraint rows per call, "
              f"{ls[4] / ls[0]:.1%} on the uniform-row form")
    if ls[7]:
        print(f"   all FD teams: {ls[7] / 2.4e3:.0f} team-us in total; Newton solves {ls[6] / ls[7]:.1%} of it, "
              f"line searches {ls[5] / ls[7]:.1%}")
    # wave 0's stamps partition its time: top-level stages, their sub-stages
    # (11-23: kinematics and Newton pieces, which restart the stage clock) and
    # the barrier waits
    tot = sum(acc[i] for i in list(range(11)) + list(range(11, 24)) + list(range(24, 30)) + [31])
    ms = sum(v[0] for v in tm.values())
    if what == "fd sweep":
        # kernels_fd.hip stamps every 2^ILQG_STAMP_SAMPLE-th workgroup (a sample of
        # every team role): totals are sums over those teams, cycles/call per call
        print(f"== {what}: lane 0 of every 64th workgroup (ILQG_STAMP_SAMPLE 6), {tot} ticks summed over the "
              f"sampled teams; kernel time {ms:.3f} ms; cycles/call are per call of a sampled team")
    else:
        print(f"== {what}: block 0, lane 0, total {tot} ticks (wave-0 stages + barriers); kernel time {ms:.3f} ms "
              f"-> {tot / (ms * 1e3):.0f} ticks/us if the stages were all of it")
    if acc[45]:
        print(f"   Newton (all workgroups): {acc[45]} solves, {acc[44]} iterations, "
              f"{acc[44] / acc[45]:.2f} iterations per solve")
    if acc[46]:
        print(f"   block 0 lifetime: {acc[46] / 100:.0f} us realtime, {acc[47]} memtime ticks "
              f"-> shader clock {acc[47] / (acc[46] / 100) :.0f} MHz; the stamps attribute "
              f"{tot / acc[47]:.1%} of wave 0's lifetime")
    for i in range(44):
        if cnt[i]:
            print(f"  {NAMES[i]:24s} calls {cnt[i]:6d}  cycles/call {acc[i]/cnt[i]:9.0f}  share {acc[i]/max(tot,1):6.1%}")
    tot2 = sum(acc[i] for i in W2)
    if tot2:
        print(f"   wave 2 (own clock): {tot2} ticks, {tot2 / max(acc[47], 1):.1%} of the block's lifetime")
        for i in W2:
            if cnt[i]:
                print(f"  {W2[i]:24s} calls {cnt[i]:6d}  cycles/call {acc[i]/cnt[i]:9.0f}  share {acc[i]/tot2:6.1%}")

# ilqg_backward on the hopper: the one-wave recursion (riccati.h)
BN = ["A Vs col, T1, v(prev), w", "B T3, Mm, col", "C LDLT, k, K col, ABK, y", "D T4, T6", "E Vn, z, record"]
if MFMA:
    g.set_riccati("mfma")
    BN = ["1 sym/A/B/q/c/r", "2 T1=B'Vs (mfma)", "3 Mm,T3 (mfma), w", "4 LDLT(Quu), col", "5 perm, K,k solves",
          "6 ABK,T6 (mfma), y, kR", "7 T4 (mfma)", "8 Vn (mfma)", "9 z, vn, K/k out", "10 v copy, record"]
acc = (ctypes.c_ulonglong * 16)(); cnt = (ctypes.c_ulonglong * 16)()
L.ilqg_debug_bstamps(acc, cnt, 1)
g.backward_pass(); g.synchronize()
L.ilqg_debug_bstamps(acc, cnt, 1)
tot = sum(acc[i] for i in range(len(BN)))
print(f"== backward: block 0, lane 0, total {tot} cycles, {tot / max(cnt[0], 1):.0f} per step")
for i in range(len(BN)):
    if cnt[i]:
        print(f"  {BN[i]:26s} calls {cnt[i]:6d}  cycles/call {acc[i]/cnt[i]:9.0f}  share {acc[i]/max(tot,1):6.1%}")
