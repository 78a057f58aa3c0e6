"""Developer tool: per-pixel event timeline of one shard (RTW_DIAG=2): hand-out,
first park, first drain claim and completion of the heaviest pixels and of the
last finishers, and the park -> claim waits of every parked pixel.
usage: python tools/diag_events.py [S] [N r]   (shard r of an N-row-cyclic split)"""
import os
os.environ.setdefault("RTW_AB", "1")  # the library reads tuning/diagnostic knobs only under RTW_AB
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["RTW_DIAG"] = "2"
import raytracing_in_a_weekend_rust_amd as rtw  # noqa: E402
from raytracing_in_a_weekend_rust_amd import shard as _sh  # noqa: E402

W, H, S = 1200, 675, int(sys.argv[1]) if len(sys.argv) > 1 else 23
NSH, RSH = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (1, 0)
seed = rtw.DEFAULT_SEED
cam, sph, n, mt, nm = rtw.builtin_scene("complex", seed, H, W, 50)
sess = rtw.Session(0)
sess.set_scene(sph, n, mt, nm)
fb = torch.zeros((H, W, 3), dtype=torch.float64, device="cuda:0")
rb, rstep, H = _sh.rows_of(RSH, NSH, H)
sess.render(cam.raw, S, seed, fb.data_ptr(), shard=(rb, rstep, H))
st = sess.stats()
d, t0 = sess.diag_events(W * H)
sess.close()
seg = d[:, 0].astype(np.float64) / (S * S)


def ms(c):
    c = c.astype(np.int64)
    return np.where(c > 0, (c - t0) / 1e5, np.nan)


done, ho, pk, cl = ms(d[:, 1]), ms(d[:, 2]), ms(d[:, 3]), ms(d[:, 4])
print(f"shard {NSH}:{RSH} kernel {st.kernel_ms:.1f} ms, parked {st.parked_pixels}, segments {st.segments}")


def show(title, idx):
    print(title)
    print("   x    y  seg/smp  hand-out  park   claim   done   cursor  wait   drain (ms)")
    for i in idx:
        print(f"{i % W:5d} {i // W:4d} {seg[i]:7.1f} {ho[i]:8.1f} {pk[i]:6.1f} {cl[i]:6.1f} {done[i]:6.1f}"
              f"  {pk[i] - ho[i]:6.1f} {cl[i] - pk[i]:6.1f} {done[i] - cl[i]:6.1f}")


show("heaviest pixels:", np.argsort(-seg)[:15])
show("last finishers:", np.argsort(-np.nan_to_num(done, nan=-1))[:15])
p = ~np.isnan(pk)
w = cl[p] - pk[p]
print(f"parked pixels {int(p.sum())}: wait park->claim ms p50 {np.nanpercentile(w, 50):.2f} p90 {np.nanpercentile(w, 90):.2f} "
      f"max {np.nanmax(w):.2f}; park time p10/p50/p90 {np.nanpercentile(pk[p], 10):.1f}/{np.nanpercentile(pk[p], 50):.1f}/"
      f"{np.nanpercentile(pk[p], 90):.1f} ms; seg/sample of parked p10/p50/p90 {np.percentile(seg[p], 10):.1f}/"
      f"{np.percentile(seg[p], 50):.1f}/{np.percentile(seg[p], 90):.1f}")
for thr in (4, 6, 8, 10, 15, 20, 30):
    m = seg > thr
    print(f"  pixels > {thr:2d} seg/sample: {int(m.sum()):6d}, parked {int((m & p).sum()):6d}, "
          f"done p50/max {np.nanpercentile(done[m], 50):.1f}/{np.nanmax(done[m]):.1f} ms")
# throughput over the kernel: each pixel's segments spread evenly between its hand-out and
# its completion, summed per 2 ms bin (how much of the launch the tail leaves idle)
ok = ~np.isnan(done) & ~np.isnan(ho)
segs_px = d[:, 0].astype(np.float64)
t_end = np.nanmax(done)
edges = np.arange(0.0, t_end + 2.0, 2.0)
rate = np.zeros(len(edges) - 1)
for a, b, s_ in zip(ho[ok], done[ok], segs_px[ok]):
    b = max(b, a + 1e-3)
    lo = np.clip(edges[:-1], a, b)
    hi = np.clip(edges[1:], a, b)
    rate += s_ * (hi - lo) / (b - a)
peak = rate.max()
print("segment rate per 2 ms bin (fraction of the peak bin): " +
      " ".join(f"{e:.0f}:{r / peak:.2f}" for e, r in zip(edges[:-1], rate)))
