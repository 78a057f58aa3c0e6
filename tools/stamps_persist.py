"""Developer tool: per-section cycle breakdown of the persistent kernel's cursor
waves from the diagnostic build. Run with
RTW_LIB=raytracing_in_a_weekend_rust_amd/_lib/librtw_stamps.so."""
import ctypes as C
import sys

import numpy as np

import raytracing_in_a_weekend_rust_amd as rtw
from raytracing_in_a_weekend_rust_amd import _capi as capi

s = int(sys.argv[1]) if len(sys.argv) > 1 else 23
cam, sph, n, mt, nm = rtw.builtin_scene("complex", rtw.DEFAULT_SEED, 675, 1200, 50)
for _ in range(2):
    fb, st = rtw.render_flat(cam.raw, sph, n, mt, nm, s, rtw.DEFAULT_SEED)
f = capi.lib.rtw_diag_stamps
f.argtypes = [C.POINTER(C.c_uint64), C.c_uint64, C.POINTER(C.c_uint64)]
nr = C.c_uint64()
f(None, 0, C.byref(nr))
buf = np.zeros((nr.value, 16), dtype=np.uint64)
assert f(buf.ctypes.data_as(C.POINTER(C.c_uint64)), nr.value, C.byref(nr)) == 0
rows = buf[: st.grid_blocks * 12]
rows = rows[rows[:, 14] > 0]
names = ["loop top/refill", "hit tail", "walk", "scatter (after record)", "next sample/pixel", "seg setup+always",
         "hit record", "fold+sum", "lattice position", "defocus disk"]
tot = rows[:, :10].sum(axis=0).astype(np.float64)
wi = float(rows[:, 14].sum())
print(f"s={s} kernel_ms={st.kernel_ms:.1f} cursor waves={len(rows)} wave iterations={wi:.0f} "
      f"segments={st.segments} (per wave-iter {st.segments / wi:.1f} lanes)")
for k, nme in enumerate(names):
    print(f"  {nme:17s} {tot[k] / tot.sum() * 100:6.2f}%  {tot[k] / wi:8.0f} cyc/wave-iter")
print(f"  total {tot.sum() / wi:.0f} cycles per wave-iteration (sections are max over lanes: an upper bound)")
cnt = rows[:, 10:14].sum(axis=0).astype(np.float64)
if cnt.any():
    print(f"draws loop: {cnt[0] / wi:.2f} wave trips per wave-iteration; per wave-iteration lanes needing a unit "
          f"vector {cnt[1] / wi:.1f}, of them resumed from a speculation {cnt[2] / wi:.1f}, lanes needing the disk "
          f"{cnt[3] / wi:.1f}")
