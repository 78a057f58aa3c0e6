"""Developer tool: kernel time of chosen shards of the bench image under knob
settings (environment variables read per render), for tuning the tail policy.

usage: python tools/knob_sweep.py 'N:r,N:r,...' 'KNOB=v KNOB=v;KNOB=v;...'
e.g.   python tools/knob_sweep.py 1:0,4:0,8:0 ';RTW_TAIL=100000;RTW_COOPG=16'
(an empty setting = the defaults)
"""
import os
os.environ.setdefault("RTW_AB", "1")  # the library reads tuning/diagnostic knobs only under RTW_AB
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raytracing_in_a_weekend_rust_amd as rtw  # noqa: E402
from raytracing_in_a_weekend_rust_amd import shard  # noqa: E402

W, H, S, DEPTH = 1200, 675, 23, 50
if os.environ.get("RTW_SWEEP_SIZE"):  # e.g. 4096x2304x45 (BASELINE's stress config)
    W, H, S = (int(v) for v in os.environ["RTW_SWEEP_SIZE"].split("x"))
SEED = rtw.DEFAULT_SEED


def main():
    shards = [tuple(int(v) for v in x.split(":")) for x in sys.argv[1].split(",")]
    settings = sys.argv[2].split(";")
    cam, sph, n, mt, nm = rtw.builtin_scene("complex", SEED, H, W, DEPTH)
    sess = rtw.Session(0)
    sess.set_scene(sph, n, mt, nm)
    stream = torch.cuda.current_stream()
    fb = torch.zeros((H, W, 3), dtype=torch.float64, device="cuda:0")
    base_env = dict(os.environ)
    ref = {}  # the first setting's image per shard: every other setting must match it bit for bit
    for st in settings:
        os.environ.clear()
        os.environ.update(base_env)
        for kv in st.split():
            k, v = kv.split("=")
            os.environ[k] = v
        row = []
        for N, r in shards:
            rb, rstep, rows = shard.rows_of(r, N, H)
            best = None
            for _ in range(1 if W * H * S * S > 2e9 else 2):
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                sess.render(cam.raw, S, SEED, fb.data_ptr(), stream=stream.cuda_stream, shard=(rb, rstep, rows))
                e1.record(stream)
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1)
                best = ms if best is None else min(best, ms)
            s = sess.stats()
            img = fb[:rows].clone()
            same = ref.setdefault((N, r), img).equal(img)
            row.append(f"{N}:{r} {best:7.1f} ms{'' if same else ' IMAGE DIFFERS'} (parked {s.parked_pixels}, inside {s.inside_segments / max(1, s.segments):.3f}, trap {s.trap_segments / max(1, s.segments):.4f})")
        print(f"[{st or 'defaults'}] " + " | ".join(row), flush=True)
    sess.close()


if __name__ == "__main__":
    main()
