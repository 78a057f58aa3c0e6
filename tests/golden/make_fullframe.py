"""Pins the benchmarked images in full (VERDICT r02 "pin the benchmarked image").

Renders whole BASELINE frames with the C oracle (oracle/rtw_oracle.c, test
infrastructure; the Rust reference cannot be built here) and
writes, per frame, the SHA-256 of the f64 framebuffer (H x W x 3, little-endian,
row 0 = top), the SHA-256 of the PPM text (Color::wire_full_file, color.rs:196-247),
the traced-segment count and a short per-row hash so a failing GPU test can name
the first differing row. Scene and camera come from the pure-Python restatement
(oracle/pyoracle.py: raytracing/mod.rs:54-126, camera.rs:138-221), so nothing of
the product's host mirror enters the fixture.

Frames: BASELINE configs[2] (1200x675, spp 100 -> s=10, depth 50) and the headline
configs[3] workload (1200x675, spp 500 -> s=23, depth 50). The stress config
(4096x2304, s=45: 19.1e9 samples, ~10 h on this container's 8 cores) is not
rendered in full; its parity is pinned through sampled rows and shard invariance
(tests/test_gpu_parity.py).

    python tests/golden/make_fullframe.py [--threads 8] [--only s10|s23]
"""
import argparse
import ctypes as C
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from oracle import oracle_ctypes as orc  # noqa: E402
from oracle import pyoracle as py  # noqa: E402
from make_golden import c_camera, c_scene  # noqa: E402

SEED = 1764892800000  # the package's DEFAULT_SEED (scene and render seed)
FRAMES = {"s10": ("complex", 675, 1200, 50, 10), "s23": ("complex", 675, 1200, 50, 23)}


def row_hashes(fb):
    return [hashlib.sha256(fb[y].tobytes()).hexdigest()[:16] for y in range(fb.shape[0])]


def frame_digest(fb, ppm):
    fb = np.ascontiguousarray(fb, dtype="<f8")
    return {"fb_sha256": hashlib.sha256(fb.tobytes()).hexdigest(),
            "ppm_sha256": hashlib.sha256(ppm).hexdigest(), "ppm_bytes": len(ppm),
            "row_sha256_16": row_hashes(fb)}


def render(key, threads):
    scene, h, w, d, s = FRAMES[key]
    pc, objs = py.scene_builtin(scene, SEED, h, w, d)
    cam = c_camera(pc)
    sph, mat = c_scene(objs)
    fb = np.zeros((h, w, 3))
    seg = C.c_uint64()
    t0 = time.time()
    rc = orc.lib().orc_render(C.byref(cam), C.byref(sph), len(objs), C.byref(mat), len(objs), s,
                              *orc.split(SEED), 0, 1, h, threads, 1,
                              fb.ctypes.data_as(C.POINTER(C.c_double)), C.byref(seg))
    assert rc == 0
    dt = time.time() - t0
    ppm = orc.format_ppm(fb)
    out = {"scene": scene, "seed": hex(SEED), "height": h, "width": w, "max_depth": d,
           "samples_sqrt": s, "segments": seg.value, "n_spheres": len(objs),
           "oracle_seconds": round(dt, 1), "oracle_threads": threads, **frame_digest(fb, ppm)}
    return out


def main():
    a = argparse.ArgumentParser()
    a.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    a.add_argument("--only", choices=sorted(FRAMES))
    args = a.parse_args()
    for key in ([args.only] if args.only else sorted(FRAMES)):
        out = render(key, args.threads)
        scene, h, w, d, s = FRAMES[key]
        name = f"fullframe_{scene}_{w}x{h}_s{s}_d{d}.json"
        with open(os.path.join(ROOT, "tests", "golden", name), "w") as f:
            json.dump(out, f, indent=0)
            f.write("\n")
        print(f"wrote {name}: {out['segments']} segments, {out['oracle_seconds']} s, "
              f"fb {out['fb_sha256'][:16]}", flush=True)


if __name__ == "__main__":
    main()
