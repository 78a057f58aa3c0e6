"""Developer tool: BASELINE configs 1 and 2 on one GPU box, for BASELINE.md's table.

Config 1: the 3-sphere Lambertian scene (three_lambertian), 400x225, spp 8 -> s=3,
depth 8, rendered by the C oracle on ONE thread (the reference's CPU plumbing case;
the oracle is test infrastructure, timed here as the CPU side). Config 2: the same
scene on the MI355X through the resident session (scene in HBM, K renders timed with
HIP events around the whole render, seeds and cost order included) and once through
the one-shot ABI with host buffers; the PPM bytes must equal the oracle's.
Prints one JSON object.
usage: python tools/config12.py [K]
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raytracing_in_a_weekend_rust_amd as rtw  # noqa: E402
from oracle import oracle_ctypes as orc  # noqa: E402  (checker / CPU side only)

SEED = rtw.DEFAULT_SEED


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    cam, sph, n, mt, nm = rtw.builtin_scene("three_lambertian", SEED)  # 400x225, depth 8
    s = 3
    samples = cam.raw.img_width * cam.raw.img_height * s * s
    t0 = time.perf_counter()
    ref, seg = orc.render(cam.raw, sph, n, mt, nm, s, SEED, nthreads=1, scheduler=0)
    cpu_s = time.perf_counter() - t0
    fb, st = rtw.render_flat(cam.raw, sph, n, mt, nm, s, SEED)  # one-shot (host buffers)
    t0 = time.perf_counter()
    fb, st = rtw.render_flat(cam.raw, sph, n, mt, nm, s, SEED)
    one_shot_ms = (time.perf_counter() - t0) * 1e3
    ok = np.array_equal(fb, ref) and rtw.format_ppm(fb) == orc.format_ppm(ref) and st.segments == seg
    sess = rtw.Session(0)
    sess.set_scene(sph, n, mt, nm)
    out = torch.empty((cam.raw.img_height, cam.raw.img_width, 3), dtype=torch.float64, device="cuda:0")
    stream = torch.cuda.current_stream()
    for _ in range(3):
        sess.render(cam.raw, s, SEED, out.data_ptr(), stream=stream.cuda_stream)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(k):
        sess.render(cam.raw, s, SEED, out.data_ptr(), stream=stream.cuda_stream)
    e1.record(stream)
    torch.cuda.synchronize()
    gpu_ms = e0.elapsed_time(e1) / k
    st2 = sess.stats()
    ok = ok and np.array_equal(out.cpu().numpy(), ref)
    sess.close()
    print(json.dumps({
        "config1_cpu": {"workload": "three_lambertian_400x225_s3_d8", "seconds": round(cpu_s, 4),
                        "msamples_per_s": round(samples / cpu_s / 1e6, 3), "threads": 1,
                        "kind": "port (C oracle, ref-faithful scheduler)", "segments": seg},
        "config2_gpu": {"render_ms": round(gpu_ms, 4), "msamples_per_s": round(samples / gpu_ms / 1e3, 1),
                        "main_kernel_ms": round(st2.main_kernel_ms, 4), "one_shot_ms": round(one_shot_ms, 3),
                        "speedup_vs_config1_cpu": round(cpu_s * 1e3 / gpu_ms, 1),
                        "note": "resident session, seeds + cost order + persistent kernel, HIP events over "
                                f"{k} renders; one_shot_ms: host buffers (PCIe) included"},
        "parity_identical_ppm": bool(ok),
    }), flush=True)


if __name__ == "__main__":
    main()
