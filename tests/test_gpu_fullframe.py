"""The benchmarked images in full, bit-exact against the C oracle.

tests/golden/make_fullframe.py rendered BASELINE configs[2] (1200x675, s=10) and
the headline workload (1200x675, s=23) with the C oracle in this container and
committed the SHA-256 of each f64 framebuffer and PPM, the segment count and a
short hash per row. Here the HIP path renders the same frames -- through the
one-shot ABI and through the multi-device ABI with 2, 4 and 8 sessions on the one
GPU (the row-cyclic config-4 splits; their shard sizes take the small-shard
scheduling: half the waves draining at 4, probe-hot pixels parked before their first
sample at 4 and 8) -- and must reproduce all of it: every one of the 675 rows."""
import hashlib
import os

import numpy as np
import pytest

import raytracing_in_a_weekend_rust_amd as rtw
from tests.golden_io import GOLDEN, load

pytestmark = pytest.mark.gpu

FRAMES = sorted(f[:-5] for f in os.listdir(GOLDEN) if f.startswith("fullframe_") and f.endswith(".json"))


def check_frame(fb, st, fix):
    fb = np.ascontiguousarray(fb, dtype="<f8")
    rows = [hashlib.sha256(fb[y].tobytes()).hexdigest()[:16] for y in range(fb.shape[0])]
    bad = [y for y, (a, b) in enumerate(zip(rows, fix["row_sha256_16"])) if a != b]
    assert not bad, f"{len(bad)} rows differ from the oracle, first {bad[:8]}"
    assert hashlib.sha256(fb.tobytes()).hexdigest() == fix["fb_sha256"]
    ppm = rtw.format_ppm(fb)
    assert len(ppm) == fix["ppm_bytes"] and hashlib.sha256(ppm).hexdigest() == fix["ppm_sha256"]
    assert st.segments == fix["segments"]


def test_fixtures_present():
    assert {"fullframe_complex_1200x675_s10_d50", "fullframe_complex_1200x675_s23_d50"} <= set(FRAMES)


@pytest.mark.parametrize("via", ["one_shot", "multi2", "multi4", "multi8"])
@pytest.mark.parametrize("frame", FRAMES)
def test_full_frame_bit_exact(frame, via):
    fix = load(frame)
    seed = int(fix["seed"], 16)
    cam, sph, n, mt, nm = rtw.builtin_scene(fix["scene"], seed, fix["height"], fix["width"], fix["max_depth"])
    assert n == fix["n_spheres"]
    if via == "one_shot":
        fb, st = rtw.render_flat(cam.raw, sph, n, mt, nm, fix["samples_sqrt"], seed)
    else:
        fb, st = rtw.render_flat_multi(cam.raw, sph, n, mt, nm, fix["samples_sqrt"], seed,
                                       devices=[0] * int(via[len("multi"):]))
    check_frame(fb, st, fix)
