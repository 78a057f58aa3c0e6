"""Developer tool: per-rank render time of the N-GPU bench, simulated on one GPU.

bench.py at --gpus N gives rank r the rows r, r+N, ... (shard.rows_of). Each rank
renders its shard independently, so the job's time is the slowest rank's render.
This renders every rank's shard (or the first `--ranks`) on cuda:0 and prints
the kernel times, the implied whole-job Msamples/s and the strong-scaling
efficiency against N=1.

usage: python tools/shard_time.py [--fast] [--size WxHxS] [--ranks K] [N ...]
  (default 1 2 4 8 on 1200x675x23; --fast: f32 mode; --ranks K: time only the
  first K ranks of each N, e.g. for BASELINE's 4096x2304x45 stress config)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raytracing_in_a_weekend_rust_amd as rtw  # noqa: E402
from raytracing_in_a_weekend_rust_amd import shard  # noqa: E402

W, H, S, DEPTH = 1200, 675, 23, 50  # --size overrides W, H, S
SEED = rtw.DEFAULT_SEED


def main():
    global W, H, S
    args = sys.argv[1:]
    fast = "--fast" in args
    args = [x for x in args if x != "--fast"]
    max_ranks = None
    if "--size" in args:
        i = args.index("--size")
        W, H, S = (int(v) for v in args[i + 1].split("x"))
        del args[i:i + 2]
    if "--ranks" in args:
        i = args.index("--ranks")
        max_ranks = int(args[i + 1])
        del args[i:i + 2]
    ns_list = [int(x) for x in args] or [1, 2, 4, 8]
    cam, sph, n, mt, nm = rtw.builtin_scene("complex", SEED, H, W, DEPTH)
    sess = rtw.Session(0)
    sess.set_scene(sph, n, mt, nm)
    stream = torch.cuda.current_stream()
    base = None
    for N in ns_list:
        rm = shard.rows_max(N, H)
        fb = torch.zeros((rm, W, 3), dtype=torch.float32 if fast else torch.float64, device="cuda:0")
        render = sess.render_fast if fast else sess.render
        times = []
        for r in range(N if max_ranks is None else min(N, max_ranks)):
            rb, rstep, rows = shard.rows_of(r, N, H)
            best = None
            for rep in range(2 if max_ranks is None else 1):  # first call warms up
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                render(cam.raw, S, SEED, fb.data_ptr(), stream=stream.cuda_stream,
                       shard=(rb, rstep, rows))
                e1.record(stream)
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1)
                best = ms if best is None else min(best, ms)
            st = sess.stats()
            times.append((best, st.segments, st.parked_pixels))
        tmax = max(t for t, _, _ in times)
        msps = W * H * S * S / (tmax / 1e3) / 1e6
        if N == 1:
            base = msps
        eff = msps / (N * base) if base else float("nan")
        print(f"N={N}: rank ms {[round(t, 1) for t, _, _ in times]} max {tmax:.1f} -> "
              f"{msps:.0f} Msamples/s, efficiency {eff:.2f}; segments/rank "
              f"{[round(s / 1e6, 1) for _, s, _ in times]} M, parked {[p for _, _, p in times]}",
              flush=True)
    sess.close()


if __name__ == "__main__":
    main()
