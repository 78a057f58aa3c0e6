"""Developer tool: per-section cycles per segment of the heaviest pixel's lane,
running (nearly) alone: row 455 of the bench image only, tile kernel, no parking.
Run with RTW_LIB=raytracing_in_a_weekend_rust_amd/_lib/librtw_stamps.so."""
import ctypes as C
import os

import numpy as np

os.environ.setdefault("RTW_PERSIST", "0")
os.environ.setdefault("RTW_BUDGET_X", "100000")  # RTW_BUDGET_X=10: heavy pixels finish in phase 2
import raytracing_in_a_weekend_rust_amd as rtw  # noqa: E402
from raytracing_in_a_weekend_rust_amd import _capi as capi  # noqa: E402

W, H, S = 1200, 675, int(os.environ.get("CHAIN_S", "23"))
ROW = int(os.environ.get("CHAIN_ROW", "455"))
cam, sph, n, mt, nm = rtw.builtin_scene("complex", rtw.DEFAULT_SEED, H, W, 50)
for _ in range(2):
    fb, st = rtw.render_flat(cam.raw, sph, n, mt, nm, S, rtw.DEFAULT_SEED, shard=(ROW, H, 1))
f = capi.lib.rtw_diag_stamps
f.argtypes = [C.POINTER(C.c_uint64), C.c_uint64, C.POINTER(C.c_uint64)]
nr = C.c_uint64()
f(None, 0, C.byref(nr))
buf = np.zeros((nr.value, 16), dtype=np.uint64)
assert f(buf.ctypes.data_as(C.POINTER(C.c_uint64)), nr.value, C.byref(nr)) == 0
names = ["setup", "hit-tail", "walk", "scatter", "fold+next", "seg+always"]
nt = ((W + 15) // 16) * 1 * 4  # tile-kernel rows (one image row), then phase-2 waves
print(f"kernel {st.kernel_ms:.2f} ms, segments {st.segments}, accel {st.accel}, parked {st.parked_pixels}")
for label, rows in (("tile", buf[:nt]), ("coop", buf[nt:])):
    life = rows[:, :10].sum(axis=1).astype(np.float64)
    for w in np.argsort(-life)[:3]:
        segs = float(rows[w, 14])
        print(f"{label} wave {int(w)}: life {life[w] / 1e6:.2f} Mcyc, max-lane segments {segs:.0f}, "
              f"{life[w] / max(1., segs):.0f} cyc/segment:",
              ", ".join(f"{nme} {float(rows[w, k]) / max(1., segs):.0f}" for k, nme in enumerate(names)))
