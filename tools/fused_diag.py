"""Diagnostic build only: timeline of the fused FD sweep + streamed backward pass
(backward role 0's cycles and record waits vs the last FD team's end).
  ILQG_LIB=ilqg-mujoco_amd/lib/libilqg_amd_diag.so python tools/fused_diag.py [S ...]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ilqg-mujoco_amd"))
import ilqg_amd as ia  # noqa: E402
import workloads  # noqa: E402

CLK = 2384.0  # s_memtime ticks per us (shader clock, tools/stamps.py)
L = ia.lib()
d = (ctypes.c_ulonglong * 24)()
m = ia.Model.load(workloads.model_file("hopper"))
for S in [int(x) for x in sys.argv[1:]] or [8, 2]:
    g = ia.ILQR(m, workloads.hopper_dmain(m, S, sigma=0.01), 500, ia.HOPPER_COST,
                alphas=tuple(2.0 ** -i for i in range(8)), select="min_cost")
    g.iterate()
    g.synchronize()
    g.set_timing(True)
    L.ilqg_debug_fused(d, 1)
    g.timing()
    g.iterate()
    g.synchronize()
    t = g.timing()
    L.ilqg_debug_fused(d, 1)
    us = lambda x: x / CLK  # noqa: E731
    print(f"S={S}: fused launch {t['fd_backward'][0]:.2f} ms; role 0: {us(d[0]):.0f} us total, {us(d[1]):.0f} us waiting "
          f"in {d[2]} polls, {us(d[0] - d[1]) / 500:.2f} us/step computing; "
          f"role durations (us): {[round(us(d[8 + i])) for i in range(min(S, 8))]}, "
          f"of which waiting: {[round(us(d[16 + i])) for i in range(min(S, 8))]}", flush=True)
    del g
