"""Developer tool: renders the final scene twice per configuration and reports
differing pixels (nondeterminism hunt) plus the park count."""
import os
os.environ.setdefault("RTW_AB", "1")  # the library reads tuning/diagnostic knobs only under RTW_AB
import sys

import numpy as np

import raytracing_in_a_weekend_rust_amd as rtw

seed = rtw.DEFAULT_SEED
H, W, S = (int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (675, 1200, 10)))
cam, sph, n, mt, nm = rtw.builtin_scene("complex", seed, H, W, 50)
configs = [
    {"RTW_BUDGET_X": "0", "RTW_RATE_X": "0"},
    {"RTW_BUDGET_X": "10", "RTW_RATE_X": "0", "RTW_HEAVY": "0"},
    {"RTW_BUDGET_X": "10", "RTW_RATE_X": "0", "RTW_HEAVY": "1"},
    {"RTW_BUDGET_X": "0", "RTW_RATE_X": "8", "RTW_HEAVY": "1"},
    {"RTW_BUDGET_X": "0", "RTW_RATE_X": "8", "RTW_HEAVY": "0"},
]
ref = None
for cfg in configs:
    for k in ("RTW_BUDGET_X", "RTW_RATE_X", "RTW_HEAVY"):
        os.environ.pop(k, None)
    os.environ.update(cfg)
    a, sa = rtw.render_flat(cam.raw, sph, n, mt, nm, S, seed)
    b, sb = rtw.render_flat(cam.raw, sph, n, mt, nm, S, seed)
    if ref is None:
        ref = a
    da = np.argwhere((a != b).any(axis=2))
    dr = np.argwhere((a != ref).any(axis=2))
    print(cfg, "parked", sa.parked_pixels, sb.parked_pixels, "run-vs-run diff px", len(da),
          "vs-ref diff px", len(dr), "segments", sa.segments, sb.segments, "ms", round(sa.kernel_ms, 1),
          "first", da[:5].tolist(), flush=True)
