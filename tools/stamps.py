"""Developer tool: per-section cycle breakdown of the megakernel from the
diagnostic build (librtw_stamps.so, -DRTW_STAMPS). Run with
RTW_LIB=raytracing_in_a_weekend_rust_amd/_lib/librtw_stamps.so."""
import ctypes as C
import sys

import numpy as np

import raytracing_in_a_weekend_rust_amd as rtw
from raytracing_in_a_weekend_rust_amd import _capi as capi

s = int(sys.argv[1]) if len(sys.argv) > 1 else 10
cam, sph, n, mt, nm = rtw.builtin_scene("complex", rtw.DEFAULT_SEED, 675, 1200, 50)
fb, st = rtw.render_flat(cam.raw, sph, n, mt, nm, s, rtw.DEFAULT_SEED)
fb, st = rtw.render_flat(cam.raw, sph, n, mt, nm, s, rtw.DEFAULT_SEED)
f = capi.lib.rtw_diag_stamps
f.argtypes = [C.POINTER(C.c_uint64), C.c_uint64, C.POINTER(C.c_uint64)]
nr = C.c_uint64()
f(None, 0, C.byref(nr))
buf = np.zeros((nr.value, 16), dtype=np.uint64)
rc = f(buf.ctypes.data_as(C.POINTER(C.c_uint64)), nr.value, C.byref(nr))
assert rc == 0, rc
names = ["setup", "hit-tail", "walk", "hit+scatter", "fold+next", "seg+always"]
tot = buf[:, :10].sum(axis=0).astype(np.float64)
print(f"s={s} kernel_ms={st.kernel_ms:.1f} waves={nr.value} segments={st.segments} wave_iters={st.wave_iterations}")
print(f"walk: lane visits/segment {st.node_visits / max(1, st.segments):.2f} (wrapped 16-bit per lane: lower bound); "
      f"wave-level walk iterations/wave-iter {st.brute_segments / max(1, st.wave_iterations):.2f}")
for k, nme in enumerate(names):
    print(f"  {nme:12s} {tot[k]/tot.sum()*100:6.2f}%  {tot[k]/max(1,st.wave_iterations):10.0f} cyc/wave-iter")
print(f"  total per wave-iter {tot.sum()/st.wave_iterations:.0f} cycles; waves resident-equivalent "
      f"{tot.sum() / (st.kernel_ms * 1e-3 * 2.4e9 * 1024):.2f} per SIMD (at 2.4 GHz)")

life = buf[:, :10].sum(axis=1).astype(np.float64)
segmax = buf[:, 14].astype(np.float64)
order = np.argsort(-life)
print("per-wave lifetime (Mcycles): mean %.1f p50 %.1f p90 %.1f p99 %.1f max %.1f; kernel %.1f Mcycles@2.4GHz"
      % (life.mean() / 1e6, np.percentile(life, 50) / 1e6, np.percentile(life, 90) / 1e6,
         np.percentile(life, 99) / 1e6, life.max() / 1e6, st.kernel_ms * 2.4e6 / 1e6))
print("per-wave max-lane segments: mean %.0f p99 %.0f max %.0f" % (segmax.mean(), np.percentile(segmax, 99), segmax.max()))
gx = (1200 + 15) // 16
for w in order[:8]:
    blk, wv = divmod(int(w), 4)
    by, bx = divmod(blk, gx)
    print(f"  wave {w}: tile x={bx*16} y={by*16 + wv*4} life {life[w]/1e6:.1f} Mcyc segmax {segmax[w]:.0f}")
