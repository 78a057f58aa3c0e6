"""Developer tool: per-pixel segment counts and completion times of the bench
workload (RTW_DIAG=1): cost distribution, row profile, drain timeline."""
import os
os.environ.setdefault("RTW_AB", "1")  # the library reads tuning/diagnostic knobs only under RTW_AB
import sys

import numpy as np
import torch

import raytracing_in_a_weekend_rust_amd as rtw

os.environ["RTW_DIAG"] = "1"
W, H, S = 1200, 675, int(sys.argv[1]) if len(sys.argv) > 1 else 23
NSH, RSH = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (1, 0)  # shard N:r
seed = rtw.DEFAULT_SEED
cam, sph, n, mt, nm = rtw.builtin_scene("complex", seed, H, W, 50)
sess = rtw.Session(0)
sess.set_scene(sph, n, mt, nm)
fb = torch.zeros((H, W, 3), dtype=torch.float64, device="cuda:0")
from raytracing_in_a_weekend_rust_amd import shard as _sh  # noqa: E402
rb, rstep, H = _sh.rows_of(RSH, NSH, H)  # H: this shard's rows from here on
sess.render(cam.raw, S, seed, fb.data_ptr(), shard=(rb, rstep, H))
st = sess.stats()
d, t0 = sess.diag(W * H)
seg = d[:, 0].astype(np.float64) / (S * S)
t = d[:, 1].astype(np.float64)
ran = d[:, 1] > 0
t = (t - (t0 if t0 else t[ran].min())) / 1e5  # ms since the launch (100 MHz real-time clock)
print(f"kernel {st.kernel_ms:.1f} ms parked {st.parked_pixels} budget_x {os.environ.get('RTW_BUDGET_X')}")
print("seg/sample percentiles 50/90/99/99.9/99.99/max:",
      [round(float(np.percentile(seg, q)), 2) for q in (50, 90, 99, 99.9, 99.99)], round(float(seg.max()), 2))
for thr in (4, 6, 8, 10, 15, 20, 30):
    print(f"  pixels > {thr} seg/sample: {int((seg > thr).sum())}")
rows = seg.reshape(H, W).mean(axis=1)
print("row means (every 45th row):", [round(float(v), 2) for v in rows[::45]])
order = np.argsort(-seg)[:10]
print("heaviest pixels (x, y, seg/sample, done ms):",
      [(int(i % W), int(i // W), round(float(seg[i]), 1), round(float(t[i]), 1)) for i in order])
done = np.sort(t[ran])
print("completion timeline: % of pixels done at ms:",
      [(q, round(float(np.percentile(done, q)), 1)) for q in (10, 25, 50, 75, 90, 95, 99, 99.9, 100)])
cost = d[:, 0].astype(np.float64)
# work done per 10 ms bucket (segments of pixels completing in the bucket)
bins = np.arange(0, done.max() + 10, 10)
h, _ = np.histogram(t[ran], bins=bins, weights=cost[ran])
print("segments completed per 10 ms (M):", [round(float(v) / 1e6, 1) for v in h])
sess.close()
last = np.argsort(-np.where(ran, t, -1))[:12]
print("last finishers (x, y, seg/sample, done ms):",
      [(int(i % W), int(i // W), round(float(seg[i]), 1), round(float(t[i]), 1)) for i in last])
late = ran & (t > np.percentile(done, 99.9))
print(f"pixels done after the 99.9% mark: {int(late.sum())}, their seg/sample: "
      f"p50 {np.percentile(seg[late], 50):.1f} max {seg[late].max():.1f}")
