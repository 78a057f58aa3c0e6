"""The oracle (test infrastructure) pinned against the reference's own tests and
the committed golden fixtures; the C and Python restatements agree bit-for-bit."""
import math
import sys

import numpy as np
import pytest

from oracle import oracle_ctypes as orc
from oracle import pyoracle as py
from tests.golden_io import fb_of, load, renders
from tests.golden.make_golden import OCam, c_camera, c_scene

MIN_POSITIVE = sys.float_info.min
MAX = sys.float_info.max
INF, NAN = math.inf, math.nan


def impls():
    return [("c", lambda a, b, x: bool(orc.lib().orc_interval_contains_inc(a, b, x)),
             lambda a, b, x: bool(orc.lib().orc_interval_contains_ex(a, b, x))),
            ("py", py.contains_inc, py.contains_ex)]


# ---- the reference's own unit tests (src/util/interval.rs:65-145) ----
@pytest.mark.parametrize("name,inc,ex", impls())
def test_interval_reference_tests(name, inc, ex):
    universe, empty, rng = (-INF, INF), (INF, -INF), (-10.0, 0.3)
    # universe_contains_inc
    for x in (0.0, INF, -INF, MIN_POSITIVE, MAX):
        assert inc(*universe, x)
    assert not inc(*universe, NAN)
    # empty_contains_inc
    for x in (0.0, INF, -INF, MIN_POSITIVE, MAX, NAN):
        assert not inc(*empty, x)
    # range_contains_inc
    for x in (-10.0, 0.3, 0.0, MIN_POSITIVE):
        assert inc(*rng, x)
    for x in (-11.0, 0.301, -INF, INF, MAX, NAN):
        assert not inc(*rng, x)
    # universe_contains_ex
    for x in (0.0, MIN_POSITIVE, MAX):
        assert ex(*universe, x)
    for x in (INF, -INF, NAN):
        assert not ex(*universe, x)
    # empty_contains_ex
    for x in (0.0, INF, -INF, MIN_POSITIVE, MAX, NAN):
        assert not ex(*empty, x)
    # range_contains_ex
    for x in (-9.99, 0.299, 0.0, MIN_POSITIVE):
        assert ex(*rng, x)
    for x in (-11.0, 0.301, -10.0, 0.3, -INF, INF, MAX, NAN):
        assert not ex(*rng, x)


# ---- camera_tests::display_offsets (src/raytracing/camera.rs:467-505) ----
def test_offset_lattice_reference_sizes():
    dx = py.unit((1.0, 0.0, -1.0))
    dy = py.unit((0.0, -1.0, 0.0))
    for s, n in ((0, 1), (1, 1), (2, 4), (3, 9)):
        c = orc.offset_lattice(dx, dy, s)
        p = py.offset_lattice(dx, dy, s)
        assert len(c) == len(p) == n
        assert c == p


def test_offset_lattice_order_and_values():
    dx, dy = (0.0, -0.25, 0.0), (0.5, 0.0, 0.0)
    lat = py.offset_lattice(dx, dy, 3)
    # outer index walks dy, inner walks dx (camera.rs:437-447)
    assert lat[1] == py.add(lat[0], py.mul(py.div(dx, 3.0), 1.0))
    assert lat[3][0] > lat[0][0] and lat[3][1] == lat[0][1]
    assert orc.offset_lattice(dx, dy, 7) == py.offset_lattice(dx, dy, 7)


# ---- XorShift known answers ----
def test_xorshift_golden():
    g = load("xorshift")
    for st in g["streams"]:
        seed = int(st["seed"], 16)
        assert orc.next_int(seed, 64) == [int(v, 16) for v in st["next_int"]]
        assert orc.next_01(seed, 256) == [float.fromhex(v) for v in st["next_01"]]
        assert orc.copy_reset_chain(seed, 64) == [int(v, 16) for v in st["copy_reset"]]
        x = py.XorShift(seed)
        assert x.next_bound(-1.0, 1.0) == float.fromhex(st["next_bound_m1_1"])
    far = g["far_children"]
    chain = orc.copy_reset_chain(int(far["seed"], 16), far["pixels"][-1] + 1)
    assert [chain[p] for p in far["pixels"]] == [int(v, 16) for v in far["children"]]


def test_next_01_range_and_fold():
    vals = orc.next_01(12345, 20000)
    assert all(0.0 <= v < 1.0 for v in vals)  # random.rs:49 debug_assert
    # u128 % (2^32-1) edge: state whose value is a multiple of 2^32-1 folds to 0
    x = py.XorShift(1)
    assert py.XorShift(0).next_01() == 0.0
    assert x.next_int() == orc.next_int(1, 1)[0]


# ---- scene + camera fixtures ----
def test_scene_complex_golden():
    g = load("scene_complex")
    for sc in g["scenes"]:
        seed = int(sc["seed"], 16)
        objs = py.scene_complex(seed)
        assert len(objs) == sc["n"]
        for (c, r, m), f in zip(objs, sc["spheres"]):
            assert c == tuple(float.fromhex(v) for v in f["center"])
            assert r == float.fromhex(f["radius"])
            assert m[0] == f["kind"] and m[1] == tuple(float.fromhex(v) for v in f["albedo"])
            assert m[2] == float.fromhex(f["fuzz"]) and m[3] == float.fromhex(f["ir"])
        kinds = [m[0] for _, _, m in objs[1:-3]]
        # thresholds 0.34 / 0.67 (mod.rs:80-88): roughly a third each
        for k in range(3):
            assert 0.2 < kinds.count(k) / len(kinds) < 0.46


def test_cameras_golden():
    g = load("cameras")
    for name, fix in g.items():
        if name == "complex_1200x675":
            pc, _ = py.scene_builtin("complex", 1, 675, 1200, 50)
        else:
            pc, _ = py.scene_builtin(name, 1)
        cam = c_camera(pc)
        for k, v in fix.items():
            want = [float.fromhex(x) for x in v] if isinstance(v, list) else float.fromhex(v)
            got = list(getattr(cam, k)) if isinstance(v, list) else getattr(cam, k)
            assert got == want, (name, k)


# ---- renders ----
@pytest.mark.parametrize("fixture", renders())
def test_c_oracle_reproduces_golden_render(fixture):
    import ctypes as C
    fix = load(fixture)
    seed = int(fix["seed"], 16)
    pc, objs = py.scene_builtin(fix["scene"], seed, fix["height"], fix["width"], fix["max_depth"])
    cam = c_camera(pc)
    sph, mat = c_scene(objs)
    fb, seg = orc.render(cam, sph, len(objs), mat, len(objs), fix["samples_sqrt"], seed,
                         nthreads=4, scheduler=0)
    assert np.array_equal(fb, fb_of(fix))
    assert seg == fix["segments"]
    assert orc.format_ppm(fb).decode() == fix["ppm"]


def test_c_and_python_oracles_agree_on_rows_of_final_scene():
    seed = 7
    pc, objs = py.scene_builtin("complex", seed, 45, 80, 50)
    cam = c_camera(pc)
    sph, mat = c_scene(objs)
    rows = (3, 19, 3)  # rows 3, 22, 41
    fb, seg = orc.render(cam, sph, len(objs), mat, len(objs), 2, seed, rows=rows)
    img, pseg = py.render(pc, objs, 2, seed, rows=[3, 22, 41])
    for k, y in enumerate((3, 22, 41)):
        for x in range(80):
            assert tuple(fb[k, x]) == img[(x, y)]
    assert seg == pseg


@pytest.mark.parametrize("h,w,s", [(1, 1, 3), (1, 13, 2), (9, 1, 2)])
def test_c_and_python_oracles_agree_on_degenerate_images(h, w, s):
    """One pixel, one row, one column: the camera's pixel deltas and the RNG
    chain's pixel order (camera.rs:223-260) at the shapes the GPU parity tests
    also render."""
    seed = 11
    pc, objs = py.scene_builtin("complex", seed, h, w, 50)
    cam = c_camera(pc)
    sph, mat = c_scene(objs)
    fb, seg = orc.render(cam, sph, len(objs), mat, len(objs), s, seed)
    img, pseg = py.render(pc, objs, s, seed, rows=list(range(h)))
    for y in range(h):
        for x in range(w):
            assert tuple(fb[y, x]) == img[(x, y)]
    assert seg == pseg


def test_schedulers_agree():
    pc, objs = py.scene_builtin("complex", 99, 27, 48, 50)
    cam = c_camera(pc)
    sph, mat = c_scene(objs)
    a, sa = orc.render(cam, sph, len(objs), mat, len(objs), 2, 99, nthreads=3, scheduler=0)
    b, sb = orc.render(cam, sph, len(objs), mat, len(objs), 2, 99, nthreads=5, scheduler=1)
    c, sc = orc.render(cam, sph, len(objs), mat, len(objs), 2, 99, rows=(1, 2, 13), nthreads=2)
    assert np.array_equal(a, b) and sa == sb
    assert np.array_equal(a[1::2], c)


def test_ppm_edge_values():
    fb = np.array([[[0.0, 1.0, 0.5], [math.nan, -0.25, 4.0]], [[1e-300, INF, 0.999999]] * 2])
    ppm = orc.format_ppm(fb).decode()
    img = {(x, y): tuple(fb[y, x]) for y in range(2) for x in range(2)}
    assert ppm == py.format_ppm(img, 2, 2)
    lines = ppm.split("\n")
    assert lines[:3] == ["P3", "2 2", "255"]
    # gamma 1/2.2, scale 255 (not 255.999), saturating casts (NaN -> 0, inf -> u64::MAX)
    assert lines[3].split() == ["0", "255", str(int(math.pow(0.5, 1 / 2.2) * 255)), "0", "0",
                                str(int(math.pow(4.0, 1 / 2.2) * 255))]
    assert lines[4].split()[1] == str(2 ** 64 - 1)
