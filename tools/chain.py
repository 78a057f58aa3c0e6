"""Developer tool: serial-chain latency of the heaviest pixels. Renders only
row 455 of the bench image (shard (455, 675, 1)), so the heavy pixels' chains run
nearly alone on the GPU, and prints the kernel time, the heaviest pixels and the
implied time per segment, per strategy knob set given as argv (K=V,...)."""
import os
os.environ.setdefault("RTW_AB", "1")  # the library reads tuning/diagnostic knobs only under RTW_AB
import sys

import numpy as np
import torch

import raytracing_in_a_weekend_rust_amd as rtw

W, H, S = 1200, 675, 23
ROW = int(os.environ.get("CHAIN_ROW", "455"))
os.environ["RTW_DIAG"] = "1"
seed = rtw.DEFAULT_SEED
cam, sph, n, mt, nm = rtw.builtin_scene("complex", seed, H, W, 50)
sess = rtw.Session(0)
sess.set_scene(sph, n, mt, nm)
fb = torch.zeros((1, W, 3), dtype=torch.float64, device="cuda:0")
for spec in sys.argv[1:] or ["-"]:
    saved = dict(os.environ)
    if spec != "-":
        for kv in spec.split(","):
            k, v = kv.split("=")
            os.environ[k] = v
    for rep in range(2):
        sess.render(cam.raw, S, seed, fb.data_ptr(), shard=(ROW, H, 1))
    torch.cuda.synchronize()
    st = sess.stats()
    d, t0 = sess.diag(W)
    seg = d[:, 0].astype(np.float64)
    t = (d[:, 1].astype(np.float64) - t0) / 1e5
    top = np.argsort(-seg)[:5]
    print(f"[{spec}] kernel {st.kernel_ms:.2f} ms, parked {st.parked_pixels}, segments {st.segments}; "
          f"heaviest (x, segs, done ms, us/seg): "
          f"{[(int(i), int(seg[i]), round(float(t[i]), 2), round(float(t[i]) * 1e3 / seg[i], 2)) for i in top]}",
          flush=True)
    os.environ.clear()
    os.environ.update(saved)
