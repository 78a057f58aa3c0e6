"""Parity of the HIP path (through the C ABI) with the oracle and the golden
fixtures. Bar: bit-exact f64 framebuffers (hence identical PPM bytes) and equal
traced-segment counts. Full-size configs are checked through sampled rows
against the oracle plus size-independent properties (determinism, shard
invariance, filter on/off invariance)."""
import ctypes as C
import os

import numpy as np
import pytest

import raytracing_in_a_weekend_rust_amd as rtw
from raytracing_in_a_weekend_rust_amd import _capi as capi
from oracle import oracle_ctypes as orc
from tests.golden_io import fb_of, load, renders

pytestmark = pytest.mark.gpu
SEED = rtw.DEFAULT_SEED


@pytest.fixture(autouse=True)
def _ab_switch(monkeypatch):
    """The strategy / schedule knobs these tests set (RTW_ACCEL, RTW_BUDGET_X, ...)
    are read by the library only under RTW_AB=1 (rtw_internal.h Knobs); with no knob
    set the A/B path is the production path."""
    monkeypatch.setenv("RTW_AB", "1")
P = C.POINTER(C.c_double)


def oracle(cam, sph, n, mt, nm, s, seed, rows=None):
    return orc.render(cam.raw, sph, n, mt, nm, s, seed, rows=rows)


def gpu(cam, sph, n, mt, nm, s, seed, shard=None):
    return rtw.render_flat(cam.raw, sph, n, mt, nm, s, seed, shard=shard)


def assert_same(fb, ref, st=None, seg=None):
    diff = int((fb != ref).sum())
    assert diff == 0, f"{diff} channels differ, max |d| = {np.abs(fb - ref).max()}"
    assert rtw.format_ppm(fb) == orc.format_ppm(ref)
    if st is not None:
        assert st.segments == seg


def test_device_available():
    assert rtw.device_count() >= 1


def test_f64_sqrt_div_correctly_rounded():
    rng = np.random.default_rng(11)
    n = 1 << 20
    a = np.abs(rng.standard_normal(n)) * 10.0 ** rng.integers(-300, 300, n)
    b = rng.standard_normal(n) * 10.0 ** rng.integers(-300, 300, n)
    a[:8] = [0.0, -0.0, np.inf, 1e-310, 5e-324, 4.0, 2.0, 1.7976931348623157e308]
    b[:8] = [1.0, 3.0, 7.0, 1e-300, 3.0, 4294967295.0, 3.0, 0.1]
    osq, odiv = np.zeros(n), np.zeros(n)
    capi.check(capi.lib.rtw_probe_f64_ops(0, a.ctypes.data_as(P), b.ctypes.data_as(P), n,
                                          osq.ctypes.data_as(P), odiv.ctypes.data_as(P)))
    with np.errstate(all="ignore"):
        assert np.array_equal(osq, np.sqrt(a), equal_nan=True)
        assert np.array_equal(odiv, a / b, equal_nan=True)
    # next_01's divisor on every 32-bit-ish numerator pattern class
    m = np.concatenate([np.arange(0, 4096), 4294967295 - np.arange(1, 4096),
                        rng.integers(0, 4294967295, 1 << 16)]).astype(np.float64)
    d = np.full_like(m, 4294967295.0)
    osq, odiv = np.zeros(len(m)), np.zeros(len(m))
    capi.check(capi.lib.rtw_probe_f64_ops(0, m.ctypes.data_as(P), d.ctypes.data_as(P), len(m),
                                          osq.ctypes.data_as(P), odiv.ctypes.data_as(P)))
    assert np.array_equal(odiv, m / d)


def test_device_seed_jump_ahead():
    for seed, first in ((SEED, 0), (SEED, 809_000), (1, 123_456_789), ((1 << 128) - 1, 9_400_000)):
        out = (capi.U128 * 2048)()
        capi.check(capi.lib.rtw_probe_device_seeds(0, capi.U128.of(seed), first, 2048, out))
        assert [out[i].value() for i in range(2048)] == rtw.seed_children(seed, first, 2048)


@pytest.mark.parametrize("fixture", renders())
def test_golden_renders(fixture):
    fix = load(fixture)
    seed = int(fix["seed"], 16)
    cam, sph, n, mt, nm = rtw.builtin_scene(fix["scene"], seed, fix["height"], fix["width"],
                                            fix["max_depth"])
    fb, st = gpu(cam, sph, n, mt, nm, fix["samples_sqrt"], seed)
    assert np.array_equal(fb, fb_of(fix))
    assert rtw.format_ppm(fb).decode() == fix["ppm"]
    assert st.segments == fix["segments"]


def test_config2_three_lambertian_full_image():
    """BASELINE config 2: 400x225, spp 8 -> s=3, depth 8, 1x MI355X vs the CPU render."""
    cam, sph, n, mt, nm = rtw.builtin_scene("three_lambertian", SEED)
    assert (cam.raw.img_width, cam.raw.img_height, cam.raw.max_depth) == (400, 225, 8)
    fb, st = gpu(cam, sph, n, mt, nm, 3, SEED)
    ref, seg = oracle(cam, sph, n, mt, nm, 3, SEED)
    assert_same(fb, ref, st, seg)
    assert st.samples == 400 * 225 * 9


@pytest.mark.parametrize("scene,h,w,d,s", [
    ("complex", 36, 64, 50, 2),
    ("complex", 45, 80, 10, 3),     # the reference's own MAX_DEPTH
    ("complex", 20, 30, 1, 2),      # every bounce hits the depth cap
    ("complex", 20, 30, 0, 2),      # max_depth 0: black, RNG still consumed
    ("complex", 17, 29, 50, 0),     # samples_sqrt 0: one centre-offset sample
    ("complex", 17, 29, 50, 1),
    ("simple", 54, 96, 25, 2),      # the reference's simple(): dielectric + metal fuzz 0
    ("threads", 40, 40, 50, 2),
    ("three_lambertian", 23, 41, 8, 4),
    ("complex", 1, 1, 50, 3),       # one pixel: one lane of one wave, every other idle
    ("complex", 1, 37, 50, 2),      # one row
    ("complex", 23, 1, 50, 2),      # one column
])
def test_scenes_bit_exact(scene, h, w, d, s):
    cam, sph, n, mt, nm = rtw.builtin_scene(scene, SEED + 1, h, w, d)
    fb, st = gpu(cam, sph, n, mt, nm, s, SEED + 2)
    ref, seg = oracle(cam, sph, n, mt, nm, s, SEED + 2)
    assert_same(fb, ref, st, seg)


def test_empty_scene_and_pinhole_camera():
    world = rtw.SceneBuilder().build()  # `Empty`: every ray misses -> sky
    cam = rtw.Camera.new(19, 33, 50, 1.0, 90.0, (0., 0., 0.), (0., 0., -1.), (0., 1., 0.), 0.0, 1.0)
    fb, st = rtw.Camera.threaded_render(cam, world, 3, seed=5, ppm_path=None)
    sph, n, mt, nm = world.flatten()
    ref, seg = orc.render(cam.raw, sph, n, mt, nm, 3, 5)
    assert_same(fb, ref, st, seg)


def test_walk_scratch_overflow_falls_back_exactly():
    """A cluster of coincident spheres gives every ray through it more candidates
    than the walk scratch holds (rtw_accel.h kMaxCand = 8): the walk records the
    overflow without branching out, and the segment is redone by the scan -- same
    (t, index) first minimum as the reference, bit-for-bit."""
    world = rtw.SceneBuilder()
    lam = rtw.Lambertian((0.5, 0.6, 0.7))
    world.add(rtw.Sphere.new_world_obj(0., -100.5, -1., 100., rtw.Lambertian((0.8, 0.8, 0.))))
    for _ in range(24):  # identical spheres: the first index wins every tie
        world.add(rtw.Sphere.new_world_obj(0., 0., -1., 0.5, lam))
    world.add(rtw.Sphere.new_world_obj(1., 0., -1., 0.5, rtw.Metal((0.8, 0.6, 0.2), 0.3)))
    world.add(rtw.Sphere.new_world_obj(-1., 0., -1., 0.5, rtw.Dielectric(1.5)))
    sph, n, mt, nm = world.build().flatten()
    cam = rtw.Camera.new(24, 40, 12, 1.0, 60.0, (0., 0.3, 1.), (0., 0., -1.), (0., 1., 0.), 0.0, 1.0)
    fb, st = gpu(cam, sph, n, mt, nm, 2, 17)
    ref, seg = oracle(cam, sph, n, mt, nm, 2, 17)
    assert_same(fb, ref, st, seg)
    assert st.accel == 2 and st.brute_segments > 0


def test_custom_scene_through_trait_surface(tmp_path):
    world = rtw.SceneBuilder()
    world.add(rtw.Sphere.new_world_obj(0., -100.5, -1., 100., rtw.Lambertian((0.8, 0.8, 0.0))))
    world.add(rtw.Sphere.new_world_obj(0., 0., -1., 0.5, rtw.Metal((0.9, 0.9, 0.9), 1.0)))
    glass = rtw.Dielectric(1.5)
    world.add(rtw.Sphere.new_world_obj(-1., 0., -1., 0.5, glass))
    world.add(rtw.Sphere.new_world_obj(-1., 0., -1., -0.4, glass))  # hollow glass (negative radius)
    world.add(rtw.Sphere.new_world_obj(1., 0., -1., 0.5, rtw.Dielectric(1.0 / 1.33)))
    world.add(rtw.Sphere.new_world_obj(0., 0., -1., 0.5, rtw.Lambertian((0.2, 0.2, 0.2))))  # coincident: tie rule
    cam = rtw.Camera.new(36, 64, 30, 1.0, 60.0, (0., 0.5, 1.), (0., 0., -1.), (0., 1., 0.), 2.0, 2.0)
    os.chdir(tmp_path)
    fb, st = rtw.Camera.threaded_render(cam, world.build(), 3, seed=77)
    sph, n, mt, nm = world.build().flatten()
    ref, seg = orc.render(cam.raw, sph, n, mt, nm, 3, 77)
    assert_same(fb, ref, st, seg)
    assert (tmp_path / "img.ppm").read_bytes() == orc.format_ppm(ref)


def test_filter_stress_scenes():
    """Scenes aimed at the exact f32 pre-filter: huge and tiny spheres, spheres far
    outside the guard, near-tangent rays, coincident and nested spheres."""
    rng = np.random.default_rng(5)
    world = rtw.SceneBuilder()
    lam = rtw.Lambertian((0.7, 0.6, 0.5))
    world.add(rtw.Sphere.new_world_obj(0., -1e6, 0., 1e6 - 0.0, lam))        # giant ground
    world.add(rtw.Sphere.new_world_obj(0., 1e13, 0., 5e12, lam))              # outside the guard
    world.add(rtw.Sphere.new_world_obj(3e3, 2., -4e3, 1e-4, lam))             # tiny, far
    for _ in range(150):
        c = rng.uniform(-3, 3, 3)
        c[1] = abs(c[1]) * 0.3
        r = float(10 ** rng.uniform(-6, 0.3))
        kind = rng.integers(0, 3)
        m = (lam if kind == 0 else rtw.Metal(tuple(rng.random(3)), float(rng.random()))
             if kind == 1 else rtw.Dielectric(float(rng.uniform(1.0, 2.4))))
        world.add(rtw.Sphere.new_world_obj(*map(float, c), r, m))
    # spheres exactly tangent to the pinhole camera's central rays
    for z in (-2.0, -3.0, -5.0):
        world.add(rtw.Sphere.new_world_obj(0.5, 0., z, 0.5, lam))
        world.add(rtw.Sphere.new_world_obj(-0.25, 0.25, z, 0.25 * 2 ** 0.5 / 2, lam))
    scene = world.build()
    sph, n, mt, nm = scene.flatten()
    for cam in (rtw.Camera.new(40, 64, 20, 1.0, 70.0, (0., 0.4, 2.), (0., 0.2, -1.), (0., 1., 0.), 0.0, 3.0),
                rtw.Camera.new(33, 47, 20, 1.0, 30.0, (0., 0., 0.), (0., 0., -1.), (0., 1., 0.), 0.0, 1.0),
                rtw.Camera.new(25, 25, 20, 1.0, 179.0, (1e5, 1e5, 1e5), (0., 0., 0.), (0., 1., 0.), 1.0, 2e5)):
        fb, st = rtw.render_flat(cam.raw, sph, n, mt, nm, 2, 99)
        ref, seg = orc.render(cam.raw, sph, n, mt, nm, 2, 99)
        assert_same(fb, ref, st, seg)


STRATEGIES = [  # (RTW_ACCEL, RTW_BUDGET_X, variant): Scene::hit strategy x budget x schedule
    ("0", "0", "16"), ("1", "0", "16"), ("2", "0", "16"),  # f64 scan / filtered scan / BVH
    ("2", "0.01", "coopg16"), ("2", "0.01", "64"),  # park every pixel after its first sample
    ("2", "1.5", "16"), ("1", "2", "64"),      # park the heavier pixels
    ("2", "0.3", "heavy0"), ("2", "2", "heavy3"),  # persistent: drain by plain waves / 3 priority waves
    ("2", "0", "rate1"),                        # rate-based parking of nearly every pixel
    ("2", "0", "order0"), ("2", "0", "order1"),  # row-major / bottom-up hand-out (default: by cost)
    ("2", "0.3", "coopg16"), ("1", "0.3", "coopg16"),  # 16-lane drain groups (default: one wave)
    ("2", "0.3", "join5"), ("2", "1.5", "join50"),  # priority waves join the cursor (RTW_JOIN %)
    ("2", "0", "endgame"), ("2", "0.3", "endgame"),  # dry cursor: park everything (RTW_ENDGAME)
    ("2", "0", "endgame_coopg16"),
    ("2", "0", "probe2"), ("2", "0.3", "probe3"),  # cost probe on one pixel per 2x2 / 3x3 block
    ("2", "0", "prepark"), ("2", "0", "drainprio0"),  # probe-hot pixels parked at once; drain at prio 0
]


@pytest.mark.parametrize("accel,budget,coop", STRATEGIES)
def test_strategies_bit_exact(monkeypatch, accel, budget, coop):
    """Every Scene::hit strategy and every phase-1 budget (including parking all
    pixels into the cooperative kernel) gives the oracle's image bit-for-bit."""
    monkeypatch.setenv("RTW_ACCEL", accel)
    monkeypatch.setenv("RTW_BUDGET_X", budget)
    monkeypatch.setenv("RTW_HEAVY", {"heavy0": "0", "heavy3": "3"}.get(coop, "1"))
    monkeypatch.setenv("RTW_RATE_X", "1" if coop == "rate1" else "8")
    monkeypatch.setenv("RTW_RATE_K", "2" if coop == "rate1" else "16")
    monkeypatch.setenv("RTW_ORDER", {"order0": "0", "order1": "1"}.get(coop, "2"))
    monkeypatch.setenv("RTW_COOPG", "16" if coop == "coopg16" else "64")
    monkeypatch.setenv("RTW_JOIN", {"join5": "5", "join50": "50"}.get(coop, "0"))
    endgame = coop.startswith("endgame")
    monkeypatch.setenv("RTW_ENDGAME", "100000000" if endgame else "0")
    monkeypatch.setenv("RTW_PROBE_SUB", coop[5:] if coop.startswith("probe") else "1")
    monkeypatch.setenv("RTW_PREPARK", "4" if coop == "prepark" else "0")
    monkeypatch.setenv("RTW_DRAIN_PRIO", "0" if coop == "drainprio0" else "3")
    if coop == "endgame_coopg16":
        monkeypatch.setenv("RTW_COOPG", "16")
    cam, sph, n, mt, nm = rtw.builtin_scene("complex", SEED, 45, 80, 50)
    fb, st = gpu(cam, sph, n, mt, nm, 3, SEED)
    ref, seg = oracle(cam, sph, n, mt, nm, 3, SEED)
    assert_same(fb, ref, st, seg)
    assert st.accel == int(accel)
    if budget == "0.01":
        assert st.parked_pixels == 45 * 80
    if budget == "0" and coop not in ("rate1", "prepark") and not endgame:
        assert st.parked_pixels == 0
    if coop == "prepark":
        assert st.parked_pixels > 45 * 80 // 4
    if endgame:
        assert st.parked_pixels > 0
    if coop == "rate1":
        assert st.parked_pixels > 45 * 80 // 2
    if accel == "2" and budget == "0":
        assert st.node_visits > 0 and st.brute_segments < st.segments // 100


def test_knobs_ignored_without_ab_switch(monkeypatch):
    """Production renders take no tuning from the environment: without RTW_AB the
    strategy knobs are not read (the BVH stays on, nothing is parked)."""
    monkeypatch.delenv("RTW_AB")
    monkeypatch.setenv("RTW_ACCEL", "0")
    monkeypatch.setenv("RTW_BUDGET_X", "0.01")
    cam, sph, n, mt, nm = rtw.builtin_scene("complex", SEED, 45, 80, 50)
    fb, st = gpu(cam, sph, n, mt, nm, 3, SEED)
    assert st.accel == 2 and st.parked_pixels < 45 * 80
    monkeypatch.setenv("RTW_AB", "1")
    fb2, st2 = gpu(cam, sph, n, mt, nm, 3, SEED)
    assert st2.accel == 0 and st2.parked_pixels == 45 * 80
    assert np.array_equal(fb, fb2) and st.segments == st2.segments


@pytest.mark.parametrize("accel,budget,coop", [("2", "0.01", "16"), ("2", "0.7", "64")])
def test_strategies_on_stress_and_deep_scenes(monkeypatch, tmp_path, accel, budget, coop):
    monkeypatch.setenv("RTW_ACCEL", accel)
    monkeypatch.setenv("RTW_BUDGET_X", budget)
    monkeypatch.setenv("RTW_COOPG", coop)
    test_filter_stress_scenes()
    _deep_closed_sphere()
    _escaping_mirrors()
    test_custom_scene_through_trait_surface(tmp_path)


def test_shards_reassemble_bit_exact():
    cam, sph, n, mt, nm = rtw.builtin_scene("complex", SEED, 50, 70, 50)
    full, st = gpu(cam, sph, n, mt, nm, 2, SEED)
    for world in (2, 3, 8):
        img = np.zeros_like(full)
        segs = 0
        for r in range(world):
            nr = len(range(r, 50, world))
            tile, ts = gpu(cam, sph, n, mt, nm, 2, SEED, shard=(r, world, nr))
            img[r::world] = tile
            segs += ts.segments
        assert np.array_equal(img, full)
        assert segs == st.segments


def test_session_device_resident_matches_host_api():
    torch = pytest.importorskip("torch")
    cam, sph, n, mt, nm = rtw.builtin_scene("complex", SEED, 27, 48, 50)
    ref, _ = gpu(cam, sph, n, mt, nm, 2, SEED)
    sess = rtw.Session(0)
    sess.set_scene(sph, n, mt, nm)
    out = torch.zeros((27, 48, 3), dtype=torch.float64, device="cuda:0")
    stream = torch.cuda.current_stream()
    sess.render(cam.raw, 2, SEED, out.data_ptr(), stream=stream.cuda_stream)
    st = sess.stats()
    assert np.array_equal(out.cpu().numpy(), ref)
    assert st.kernel_ms > 0
    s2 = torch.cuda.Stream()
    out2 = torch.zeros_like(out)
    sess.render(cam.raw, 2, SEED, out2.data_ptr(), stream=s2.cuda_stream, shard=(1, 2, 13))
    s2.synchronize()
    assert np.array_equal(out2[:13].cpu().numpy(), ref[1::2])
    sess.close()


def test_final_scene_config3_sampled_rows():
    """BASELINE config 3 (1200x675, spp 100, depth 50): full image on the GPU,
    determinism, and 3 rows (top / middle / bottom) bit-exact vs the oracle."""
    cam, sph, n, mt, nm = rtw.builtin_scene("complex", SEED, 675, 1200, 50)
    fb, st = gpu(cam, sph, n, mt, nm, 10, SEED)
    fb2, st2 = gpu(cam, sph, n, mt, nm, 10, SEED)
    assert np.array_equal(fb, fb2) and st.segments == st2.segments
    assert np.isfinite(fb).all() and fb.min() >= 0.0 and fb.max() <= 1.0
    ref, seg = oracle(cam, sph, n, mt, nm, 10, SEED, rows=(0, 337, 3))
    assert np.array_equal(fb[0::337], ref)
    assert 2.5 < st.segments / st.samples < 3.5


def test_final_scene_config4_sampled_rows():
    """BASELINE config 4 workload (spp 500 -> s=23): two rows vs the oracle."""
    cam, sph, n, mt, nm = rtw.builtin_scene("complex", SEED, 675, 1200, 50)
    fb, st = gpu(cam, sph, n, mt, nm, 23, SEED, shard=(300, 74, 2))
    ref, seg = oracle(cam, sph, n, mt, nm, 23, SEED, rows=(300, 74, 2))
    assert_same(fb, ref, st, seg)


def test_stress_config5_sampled_rows():
    """BASELINE stress config (4096x2304, spp 2000 -> s=45, depth 50): the largest
    image -- 9.4M pixels, 24-bit jump-ahead -- on one sampled row, bit-exact vs
    the oracle."""
    cam, sph, n, mt, nm = rtw.builtin_scene("complex", SEED, 2304, 4096, 50)
    rows = (2047, 256, 1)  # image row 2047 (ground, near the bottom)
    fb, st = gpu(cam, sph, n, mt, nm, 45, SEED, shard=rows)
    assert st.samples == 4096 * 2025
    ref, seg = oracle(cam, sph, n, mt, nm, 45, SEED, rows=rows)
    assert_same(fb, ref, st, seg)


def _set_fold_black(monkeypatch, fold_black):
    if fold_black:
        monkeypatch.setenv("RTW_FOLD_BLACK", fold_black)
    else:
        monkeypatch.delenv("RTW_FOLD_BLACK", raising=False)


@pytest.mark.parametrize("fold_black", ["", "1"])
def test_deep_paths_use_spill_levels(monkeypatch, fold_black):
    """Camera inside a closed Lambertian sphere: every path bounces to the depth
    cap, so the path stack runs past its register slots into the HBM spill levels.
    By default a depth-capped sample skips the fold (its product is +-0);
    RTW_FOLD_BLACK=1 folds it through the spill levels as the recursion would."""
    _set_fold_black(monkeypatch, fold_black)
    _deep_closed_sphere()


def _deep_closed_sphere():
    world = rtw.SceneBuilder()
    world.add(rtw.Sphere.new_world_obj(0., 0., 0., 10., rtw.Lambertian((0.93, 0.91, 0.97))))
    world.add(rtw.Sphere.new_world_obj(0., -1., -3., 1., rtw.Metal((0.8, 0.85, 0.9), 0.2)))
    world.add(rtw.Sphere.new_world_obj(1.5, 0., -3., 0.7, rtw.Dielectric(1.5)))
    scene = world.build()
    sph, n, mt, nm = scene.flatten()
    for depth in (9, 40):
        cam = rtw.Camera.new(24, 32, depth, 1.0, 80.0, (0., 0., 2.), (0., 0., -1.), (0., 1., 0.), 0.5, 5.0)
        fb, st = rtw.render_flat(cam.raw, sph, n, mt, nm, 2, 31)
        ref, seg = orc.render(cam.raw, sph, n, mt, nm, 2, 31)
        assert_same(fb, ref, st, seg)
        assert st.segments == st.samples * depth  # nothing ever escapes


@pytest.mark.parametrize("fold_black", ["", "1"])
def test_long_escaping_paths_fold_spill_levels(monkeypatch, fold_black):
    """Two big facing mirrors (r = 1e4, fuzz 0 and 0.05, 2 apart) with the camera
    between them looking down at a slant: paths bounce ~20 times and most escape, so
    the fold of a sky leaf reads its deepest attenuation rows back from the HBM spill
    levels; the rest hit the depth cap (black leaf, fold skipped unless
    RTW_FOLD_BLACK=1)."""
    _set_fold_black(monkeypatch, fold_black)
    _escaping_mirrors()


def _escaping_mirrors():
    world = rtw.SceneBuilder()
    world.add(rtw.Sphere.new_world_obj(0., -10001., 0., 1e4, rtw.Metal((0.97, 0.95, 0.9), 0.)))
    world.add(rtw.Sphere.new_world_obj(0., 10001., 0., 1e4, rtw.Metal((0.9, 0.95, 0.97), 0.05)))
    world.add(rtw.Sphere.new_world_obj(0., 0., -4., 0.6, rtw.Lambertian((0.7, 0.3, 0.3))))
    scene = world.build()
    sph, n, mt, nm = scene.flatten()
    cam = rtw.Camera.new(24, 40, 40, 1.0, 70.0, (0., 0., 0.), (0., -1., -3.), (0., 0., -1.), 0.2, 4.0)
    fb, st = rtw.render_flat(cam.raw, sph, n, mt, nm, 3, 77)
    ref, seg = orc.render(cam.raw, sph, n, mt, nm, 3, 77)
    assert_same(fb, ref, st, seg)
    assert st.segments > 12 * st.samples  # deep paths (~20 segments/sample): past the 8 register levels
    assert float(ref.mean()) > 0.2  # most escape to the sky
    assert float((ref.sum(-1) == 0).mean()) > 0.01  # some pixels only ever reach the depth cap


@pytest.mark.parametrize("budget", ["0.01", "0"])
def test_trapped_paths_fast_forward(monkeypatch, budget):
    """Scenes that trap paths (rtw_accel.h "Trapped paths"): Lambertian spheres
    hovering within 0.01 of a big Lambertian ground (rays slip inside through the
    skipped near root), an overlapping Lambertian pair (neighbour half-space), a
    glass sphere (total internal reflection) and a small glass sphere inside a big
    one. With every pixel parked (budget 0.01) the drain groups fast-forward the
    trapped samples; the image, the segment count and the RNG streams after them
    must match the oracle bit-for-bit."""
    monkeypatch.setenv("RTW_BUDGET_X", budget)
    world = rtw.SceneBuilder()
    world.add(rtw.Sphere.new_world_obj(0., -100., 0., 100., rtw.Lambertian((0.6, 0.6, 0.5))))
    for i, gap in enumerate((0.001, 0.004, 0.0095, 0.02)):
        world.add(rtw.Sphere.new_world_obj(-1.5 + i, 0.3 + gap + (i * i) * 1e-3, -0.5, 0.3,
                                           rtw.Lambertian((0.3 + 0.1 * i, 0.5, 0.7))))
    world.add(rtw.Sphere.new_world_obj(-0.6, 0.45, -1.6, 0.45, rtw.Lambertian((0.8, 0.3, 0.2))))
    world.add(rtw.Sphere.new_world_obj(0.1, 0.45, -1.6, 0.45, rtw.Lambertian((0.2, 0.8, 0.3))))  # overlaps
    world.add(rtw.Sphere.new_world_obj(1.3, 0.6, -1.5, 0.6, rtw.Dielectric(1.5)))
    world.add(rtw.Sphere.new_world_obj(1.3, 0.6, -1.5, 0.2, rtw.Dielectric(2.4)))  # glass in glass
    world.add(rtw.Sphere.new_world_obj(-2.4, 0.5, -2.2, 0.5, rtw.Metal((0.8, 0.8, 0.8), 0.3)))
    scene = world.build()
    sph, n, mt, nm = scene.flatten()
    cam = rtw.Camera.new(40, 64, 50, 1.0, 40.0, (0., 1.2, 3.5), (0., 0.3, -1.), (0., 1., 0.), 0.3, 4.0)
    fb, st = rtw.render_flat(cam.raw, sph, n, mt, nm, 3, 1234)
    ref, seg = orc.render(cam.raw, sph, n, mt, nm, 3, 1234)
    assert_same(fb, ref, st, seg)
    if budget == "0.01":
        assert st.parked_pixels == 40 * 64
        assert st.trap_segments > 0


@pytest.mark.parametrize("coop", ["join5", "heavy0", "default"])
def test_no_progress_guard_and_leftover_launch(monkeypatch, coop):
    """A zero no-progress guard (RTW_SPIN_GUARD_MS=0): waiting waves of the
    persistent kernel leave as soon as two checks see nothing move, so claimed
    tickets can be left behind and parked pixels published after the drain
    waves left are finished by the follow-up launch (rtw_park_leftover). The
    image must still be complete and bit-exact."""
    monkeypatch.setenv("RTW_SPIN_GUARD_MS", "0")
    monkeypatch.setenv("RTW_BUDGET_X", "0.3")
    monkeypatch.setenv("RTW_JOIN", "5" if coop == "join5" else "0")
    if coop == "heavy0":
        monkeypatch.setenv("RTW_HEAVY", "0")
    cam, sph, n, mt, nm = rtw.builtin_scene("complex", SEED, 45, 80, 50)
    fb, st = gpu(cam, sph, n, mt, nm, 3, SEED)
    ref, seg = oracle(cam, sph, n, mt, nm, 3, SEED)
    assert_same(fb, ref, st, seg)
    assert st.parked_pixels > 0 and st.leftover_pixels <= st.parked_pixels
    print(f"guard exits {st.guard_exits}, leftover pixels {st.leftover_pixels}")


@pytest.mark.parametrize("budget", ["0.01", "0.3"])
def test_leftover_launch_finishes_every_parked_pixel(monkeypatch, budget):
    """The persistent kernel with its drain switched off (RTW_DRAIN_OFF=1, no
    priority waves): every parked pixel is published and left unclaimed, so the
    follow-up launch (rtw_park_leftover) finishes all of them -- its region-B spill
    columns by slot, the pass-1 records it stages and its published-flag filter.
    Budget 0.01 parks every pixel after its first sample."""
    monkeypatch.setenv("RTW_DRAIN_OFF", "1")
    monkeypatch.setenv("RTW_HEAVY", "0")
    monkeypatch.setenv("RTW_BUDGET_X", budget)
    cam, sph, n, mt, nm = rtw.builtin_scene("complex", SEED, 45, 80, 50)
    fb, st = gpu(cam, sph, n, mt, nm, 3, SEED)
    ref, seg = oracle(cam, sph, n, mt, nm, 3, SEED)
    assert_same(fb, ref, st, seg)
    assert st.parked_pixels > 0 and st.leftover_pixels == st.parked_pixels
    if budget == "0.01":
        assert st.parked_pixels == 45 * 80


def test_default_guard_leaves_nothing_behind():
    """On an exclusive device the default guard never fires: every parked pixel
    is finished inside the persistent kernel."""
    cam, sph, n, mt, nm = rtw.builtin_scene("complex", SEED, 90, 160, 50)
    fb, st = gpu(cam, sph, n, mt, nm, 4, SEED)
    assert st.guard_exits == 0 and st.leftover_pixels == 0


def test_session_renders_on_two_streams_are_serialized():
    """Renders of one session share its device buffers: a render enqueued on a
    second stream before the first finished must wait for it (both images exact)."""
    torch = pytest.importorskip("torch")
    cam, sph, n, mt, nm = rtw.builtin_scene("complex", SEED, 60, 96, 50)
    ref_a, _ = gpu(cam, sph, n, mt, nm, 3, SEED)
    ref_b, _ = gpu(cam, sph, n, mt, nm, 2, SEED + 7)
    sess = rtw.Session(0)
    sess.set_scene(sph, n, mt, nm)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    a = torch.zeros((60, 96, 3), dtype=torch.float64, device="cuda:0")
    b = torch.zeros_like(a)
    sess.render(cam.raw, 3, SEED, a.data_ptr(), stream=s1.cuda_stream)
    sess.render(cam.raw, 2, SEED + 7, b.data_ptr(), stream=s2.cuda_stream)
    st = sess.stats()  # the second render's stats; the latch covers the first
    s1.synchronize()
    s2.synchronize()
    assert np.array_equal(a.cpu().numpy(), ref_a)
    assert np.array_equal(b.cpu().numpy(), ref_b)
    assert st.pixels == 60 * 96
    sess.close()


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0], None])
def test_multi_device_abi_matches_single_device(devices):
    """rtw_threaded_render_multi (the multi-GPU Camera::threaded_render through the
    C ABI alone): one session + host thread per entry, rows dealt cyclically,
    gathered by strided device-to-host copies. Repeating device 0 exercises
    several sessions and streams on the one GPU of the test box; None = every
    visible device. Bit-exact against the single-device image."""
    cam, sph, n, mt, nm = rtw.builtin_scene("complex", SEED, 61, 96, 50)
    ref, st = gpu(cam, sph, n, mt, nm, 3, SEED)
    fb, mst = rtw.render_flat_multi(cam.raw, sph, n, mt, nm, 3, SEED, devices=devices)
    assert np.array_equal(fb, ref)
    assert mst.segments == st.segments and mst.pixels == 61 * 96 and mst.samples == st.samples
    # merged times: the slowest entry's main kernel and whole render
    assert 0 < mst.main_kernel_ms <= mst.kernel_ms


def test_multi_device_more_entries_than_rows():
    """Device entries beyond the image's rows get no rows (rows r = i mod n with
    n = min(entries, H)); the image is still the single-device one."""
    cam, sph, n, mt, nm = rtw.builtin_scene("complex", SEED, 3, 17, 50)
    ref, st = gpu(cam, sph, n, mt, nm, 2, SEED)
    fb, mst = rtw.render_flat_multi(cam.raw, sph, n, mt, nm, 2, SEED, devices=[0] * 5)
    assert np.array_equal(fb, ref)
    assert mst.segments == st.segments and mst.pixels == 3 * 17


def test_shutdown_frees_and_recreates_sessions():
    cam, sph, n, mt, nm = rtw.builtin_scene("complex", SEED, 30, 40, 50)
    ref, _ = gpu(cam, sph, n, mt, nm, 2, SEED)
    rtw.render_flat_multi(cam.raw, sph, n, mt, nm, 2, SEED, devices=[0, 0])
    rtw.shutdown()
    fb, _ = gpu(cam, sph, n, mt, nm, 2, SEED)  # the one-shot session is re-created
    assert np.array_equal(fb, ref)
    fb, _ = rtw.render_flat_multi(cam.raw, sph, n, mt, nm, 2, SEED, devices=[0, 0, 0, 0])
    assert np.array_equal(fb, ref)
    rtw.shutdown()


def test_camera_rays_on_frustum_edges():
    """Camera rays through a scene built on pixel-frustum edges: spheres tangent to
    pixel and tile frusta, grazing the defocus cone, straddling the focus plane,
    behind and around the camera, a camera inside a sphere, and a tight sphere
    cluster (once the bounds of the rejected per-tile camera-ray candidate lists,
    kept as a walk stress scene). Bit-exact."""
    rng = np.random.default_rng(23)
    world = rtw.SceneBuilder()
    lam = rtw.Lambertian((0.6, 0.5, 0.4))
    world.add(rtw.Sphere.new_world_obj(0., -1000., 0., 1000., lam))
    for _ in range(220):
        c = rng.uniform(-3, 3, 3)
        c[2] = -abs(c[2]) * 2 - 0.5
        r = float(10 ** rng.uniform(-3, -0.5))
        m = lam if rng.random() < 0.4 else rtw.Metal((0.9, 0.8, 0.7), 0.2) if rng.random() < 0.5 else rtw.Dielectric(1.5)
        world.add(rtw.Sphere.new_world_obj(*map(float, c), r, m))
    for k in range(12):  # a tight cluster: more candidates than a list holds
        world.add(rtw.Sphere.new_world_obj(0.01 * k, 0.2, -2.0, 0.05, lam))
    world.add(rtw.Sphere.new_world_obj(0., 0.3, 1.2, 0.3, lam))    # behind the camera
    world.add(rtw.Sphere.new_world_obj(0., 0.4, 1., 0.6, rtw.Dielectric(1.5)))  # the camera inside glass
    sph, n, mt, nm = world.build().flatten()
    for cam in (rtw.Camera.new(30, 48, 12, 1.0, 50.0, (0., 0.4, 1.), (0., 0.1, -2.), (0., 1., 0.), 4.0, 3.0),
                rtw.Camera.new(31, 29, 12, 1.0, 90.0, (0., 0.4, 1.), (0.3, 0.2, -2.), (0., 1., 0.), 0.0, 1.0)):
        fb, st = rtw.render_flat(cam.raw, sph, n, mt, nm, 2, 404)
        ref, seg = orc.render(cam.raw, sph, n, mt, nm, 2, 404)
        assert_same(fb, ref, st, seg)
