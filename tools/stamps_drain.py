"""Developer tool: where a drained segment's time goes -- the serial chain of one
pixel run by a whole wave (coop_pixel, the strong-scaling critical path).

With RTW_BUDGET_X=0.01 every pixel parks after its first sample and with
RTW_DRAIN_OFF=1 the persistent kernel drains none of them, so the leftover launch
(rtw_park_leftover, one 64-lane group per pixel) runs every remaining segment; the
diagnostic build (make stamps) records per-wave section sums there.
usage: RTW_LIB=raytracing_in_a_weekend_rust_amd/_lib/librtw_stamps.so \\
       python tools/stamps_drain.py [ROW_BEGIN ROW_STEP N_ROWS]   (default rows 455::675 x1 of the bench image)
"""
import ctypes as C
import os
os.environ.setdefault("RTW_AB", "1")  # the library reads tuning/diagnostic knobs only under RTW_AB
import sys

import numpy as np

os.environ.setdefault("RTW_BUDGET_X", "0.01")
os.environ.setdefault("RTW_DRAIN_OFF", "1")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raytracing_in_a_weekend_rust_amd as rtw  # noqa: E402
from raytracing_in_a_weekend_rust_amd import _capi as capi  # noqa: E402

shard = tuple(int(v) for v in sys.argv[1:4]) if len(sys.argv) >= 4 else (455, 675, 1)
cam, sph, n, mt, nm = rtw.builtin_scene("complex", rtw.DEFAULT_SEED, 675, 1200, 50)
for _ in range(2):
    fb, st = rtw.render_flat(cam.raw, sph, n, mt, nm, 23, rtw.DEFAULT_SEED, shard=shard)
f = capi.lib.rtw_diag_stamps
f.argtypes = [C.POINTER(C.c_uint64), C.c_uint64, C.POINTER(C.c_uint64)]
nr = C.c_uint64()
f(None, 0, C.byref(nr))
buf = np.zeros((nr.value, 16), dtype=np.uint64)
assert f(buf.ctypes.data_as(C.POINTER(C.c_uint64)), nr.value, C.byref(nr)) == 0
rows = buf[st.grid_blocks * 12:]  # after the persistent kernel's rows
rows = rows[rows[:, 14] > 0]
names = ["seg setup (Seg32)", "hit tail", "exact tests + min", "trap check", "fold+next sample", "filter",
         "hit record", "scatter", "lattice position", "defocus disk"]
tot = rows[:, :10].sum(axis=0).astype(np.float64)
segs = float(rows[:, 14].sum())
print(f"shard {shard}: kernel {st.kernel_ms:.2f} ms, leftover pixels {st.leftover_pixels}, drain waves {len(rows)}, "
      f"segments {segs:.0f}, {tot.sum() / segs:.0f} cycles per drained segment (stamped; stamps cost ~10 %)")
for k, nme in enumerate(names):
    if tot[k]:
        print(f"  {nme:20s} {tot[k] / tot.sum() * 100:6.2f}%  {tot[k] / segs:7.0f} cyc/segment")
# the waves that drained the longest chains (a wave drains one pixel at a time; the
# heaviest pixels dominate their wave's rows)
top = np.argsort(rows[:, 14])[::-1][:3]
for w in top:
    r = rows[w, :10].astype(np.float64)
    print(f"wave of {int(rows[w, 14])} segments: {r.sum() / rows[w, 14]:.0f} cyc/segment: " +
          ", ".join(f"{nme} {r[k] / rows[w, 14]:.0f}" for k, nme in enumerate(names) if r[k]))
