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
rendered in full (~6 h here); instead `--only s45rows` renders a row sample of it with
the same oracle -- every 16th row plus every 8th row across the big glass sphere
(the longest dielectric paths) -- and writes per-row SHA-256 and per-row segment
counts to rowsample_complex_4096x2304_s45_d50.json (tests/test_gpu_fullframe.py
renders the whole frame on the GPU and checks those rows).

    python tests/golden/make_fullframe.py [--threads 8] [--only s10|s23|s45rows]
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
ROW_SAMPLES = {"s45rows": ("complex", 2304, 4096, 50, 45)}


def sphere_rows(pc, center, radius, col_step=4):
    """Image rows whose camera rays (pixel corners, pinhole from look_from) meet the
    sphere: the row band the sphere covers on screen (row selection only)."""
    o = np.array(pc.look_from)
    p00, du, dv = (np.array(v) for v in (pc.pixel00, pc.pixel_delta_u, pc.pixel_delta_v))
    xs = np.arange(0, pc.width, col_step, dtype=np.float64)
    hit = []
    for y in range(pc.height):
        d = p00[None, :] + du[None, :] * xs[:, None] + dv[None, :] * float(y) - o[None, :]
        oc = o - np.array(center)
        a = (d * d).sum(1)
        hb = d @ oc
        disc = hb * hb - a * (oc @ oc - radius * radius)
        if (disc >= 0).any():
            hit.append(y)
    return hit


def sample_rows(pc, objs):
    glass = next(o for o in objs if o[1] == 1.0 and o[2][0] == py.DIELECTRIC)
    band = sphere_rows(pc, glass[0], glass[1])
    return sorted(set(range(0, pc.height, 16)) | {y for y in band if y % 8 == 0}), (band[0], band[-1])


def render_rowsample(key, threads):
    scene, h, w, d, s = ROW_SAMPLES[key]
    pc, objs = py.scene_builtin(scene, SEED, h, w, d)
    cam = c_camera(pc)
    sph, mat = c_scene(objs)
    rows, band = sample_rows(pc, objs)
    t0 = time.time()
    fb, seg, row_seg = orc.render_rows(cam, sph, len(objs), mat, len(objs), s, SEED, rows,
                                       nthreads=threads, scheduler=1)
    dt = time.time() - t0
    fb = np.ascontiguousarray(fb, dtype="<f8")
    ppm_rows = [hashlib.sha256(orc.format_ppm(fb[k:k + 1]).split(b"\n", 3)[3]).hexdigest()[:16]
                for k in range(len(rows))]
    return {"scene": scene, "seed": hex(SEED), "height": h, "width": w, "max_depth": d,
            "samples_sqrt": s, "n_spheres": len(objs), "rows": rows, "glass_band": list(band),
            "segments": int(seg), "row_segments": [int(v) for v in row_seg],
            "row_sha256": [hashlib.sha256(fb[k].tobytes()).hexdigest() for k in range(len(rows))],
            "ppm_row_sha256_16": ppm_rows,
            "oracle_seconds": round(dt, 1), "oracle_threads": threads}


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
    a.add_argument("--only", choices=sorted(FRAMES) + sorted(ROW_SAMPLES))
    args = a.parse_args()
    if args.only in ROW_SAMPLES:
        out = render_rowsample(args.only, args.threads)
        scene, h, w, d, s = ROW_SAMPLES[args.only]
        name = f"rowsample_{scene}_{w}x{h}_s{s}_d{d}.json"
        with open(os.path.join(ROOT, "tests", "golden", name), "w") as f:
            json.dump(out, f, indent=0)
            f.write("\n")
        print(f"wrote {name}: {len(out['rows'])} rows, {out['segments']} segments, "
              f"{out['oracle_seconds']} s", flush=True)
        return
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
