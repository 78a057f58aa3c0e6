"""f32 fast mode (rtw_session_render_fast / rtw_threaded_render_fast): the gate is
statistical, as SURVEY 8(c) sets it for fast mode -- on the 8-bit PPM values
(color.rs:196-247: (c^(1/2.2) * 255) as u64), per channel the image-mean
|mean(fast - ref)| <= 1.0, and >= 99% of pixels with every channel within
max(8, 4 sigma_MC) of the f64 reference render, sigma_MC being the per-pixel
spread of 8 more f64 renders at other seeds at the same spp (max over the 3x3
neighbourhood; tests/fast_gate.py, calibrated on the oracle against itself in
tests/test_fast_gate.py). The f64 references
are the oracle itself (config 1) or the parity path, which is bit-exact to the
oracle (test_gpu_parity.py). Exact properties: determinism, shard invariance,
black at max_depth 0, the sky of an empty scene."""
import numpy as np
import pytest

import raytracing_in_a_weekend_rust_amd as rtw
from oracle import oracle_ctypes as orc
from tests.fast_gate import BIAS_TOL, PIXEL_FRAC, gate

pytestmark = pytest.mark.gpu
SEED = rtw.DEFAULT_SEED
def fast(cam, sph, n, mt, nm, s, seed, shard=None):
    return rtw.render_flat_fast(cam.raw, sph, n, mt, nm, s, seed, shard=shard)


def test_fast_final_scene_statistical():
    cam, sph, n, mt, nm = rtw.builtin_scene("complex", SEED, 108, 192, 50)
    fb, st = fast(cam, sph, n, mt, nm, 16, SEED)
    assert fb.dtype == np.float32 and fb.shape == (108, 192, 3)
    assert st.samples == 108 * 192 * 256 and st.segments > 2 * st.samples
    ref, _ = rtw.render_flat(cam.raw, sph, n, mt, nm, 16, SEED + 100)
    others = [rtw.render_flat(cam.raw, sph, n, mt, nm, 16, SEED + 101 + i)[0] for i in range(8)]
    bias, within = gate(fb, ref, others)
    assert (bias <= BIAS_TOL).all(), bias
    assert within >= PIXEL_FRAC, within


def test_fast_config1_vs_oracle_statistical():
    """BASELINE config 1 (three_lambertian, 400x225, s=3, depth 8) against the C oracle."""
    cam, sph, n, mt, nm = rtw.builtin_scene("three_lambertian", SEED)
    fb, _ = fast(cam, sph, n, mt, nm, 3, SEED)
    ref, _ = orc.render(cam.raw, sph, n, mt, nm, 3, SEED + 100)
    others = [orc.render(cam.raw, sph, n, mt, nm, 3, SEED + 101 + i)[0] for i in range(8)]
    bias, within = gate(fb, ref, others)
    assert (bias <= BIAS_TOL).all(), bias
    assert within >= PIXEL_FRAC, within


@pytest.mark.parametrize("scene,h,w,d,s", [
    ("simple", 54, 96, 25, 6),       # dielectric + metal with fuzz 0
    ("threads", 40, 40, 50, 8),
])
def test_fast_other_scenes_statistical(scene, h, w, d, s):
    cam, sph, n, mt, nm = rtw.builtin_scene(scene, SEED + 1, h, w, d)
    fb, _ = fast(cam, sph, n, mt, nm, s, SEED)
    ref, _ = rtw.render_flat(cam.raw, sph, n, mt, nm, s, SEED + 100)
    others = [rtw.render_flat(cam.raw, sph, n, mt, nm, s, SEED + 101 + i)[0] for i in range(8)]
    bias, within = gate(fb, ref, others)
    assert (bias <= BIAS_TOL).all(), bias
    assert within >= PIXEL_FRAC, within


def test_fast_deterministic_and_shard_invariant():
    cam, sph, n, mt, nm = rtw.builtin_scene("complex", SEED, 90, 160, 50)
    a, sa = fast(cam, sph, n, mt, nm, 4, SEED)
    b, sb = fast(cam, sph, n, mt, nm, 4, SEED)
    assert np.array_equal(a, b) and sa.segments == sb.segments
    parts = [fast(cam, sph, n, mt, nm, 4, SEED, shard=(r, 3, 30))[0] for r in range(3)]
    assembled = np.zeros_like(a)
    for r in range(3):
        assembled[r::3] = parts[r]
    assert np.array_equal(assembled, a)
    c, _ = fast(cam, sph, n, mt, nm, 4, SEED + 1)
    assert not np.array_equal(a, c)  # the render seed reaches the streams


def test_fast_depth_zero_is_black_and_spp_one():
    cam, sph, n, mt, nm = rtw.builtin_scene("complex", SEED, 20, 30, 5)
    cam.raw.max_depth = 0  # ray_color at depth 0 >= max_depth: black (camera.rs:381-383)
    fb, st = fast(cam, sph, n, mt, nm, 2, SEED)
    assert not fb.any() and st.segments == 0
    cam, sph, n, mt, nm = rtw.builtin_scene("complex", SEED, 17, 29, 50)
    fb, st = fast(cam, sph, n, mt, nm, 0, SEED)
    assert st.samples == 17 * 29 and np.isfinite(fb).all() and fb.any()


def test_fast_empty_scene_sky():
    world = rtw.SceneBuilder().build()
    cam = rtw.Camera.new(19, 33, 50, 1.0, 90.0, (0., 0., 0.), (0., 0., -1.), (0., 1., 0.), 0.0, 1.0)
    sph, n, mt, nm = world.flatten()
    fb, st = fast(cam, sph, n, mt, nm, 3, 5)
    ref, seg = orc.render(cam.raw, sph, n, mt, nm, 3, 5)
    assert st.segments == seg
    assert np.abs(fb - ref).max() <= 1e-5


def test_fast_custom_scene_statistical():
    """Hollow glass (negative radius), a coincident pair, a refraction index < 1."""
    world = rtw.SceneBuilder()
    world.add(rtw.Sphere.new_world_obj(0., -100.5, -1., 100., rtw.Lambertian((0.8, 0.8, 0.0))))
    world.add(rtw.Sphere.new_world_obj(0., 0., -1., 0.5, rtw.Metal((0.9, 0.9, 0.9), 1.0)))
    glass = rtw.Dielectric(1.5)
    world.add(rtw.Sphere.new_world_obj(-1., 0., -1., 0.5, glass))
    world.add(rtw.Sphere.new_world_obj(-1., 0., -1., -0.4, glass))
    world.add(rtw.Sphere.new_world_obj(1., 0., -1., 0.5, rtw.Dielectric(1.0 / 1.33)))
    cam = rtw.Camera.new(72, 128, 30, 1.0, 60.0, (0., 0.5, 1.), (0., 0., -1.), (0., 1., 0.), 2.0, 2.0)
    sph, n, mt, nm = world.build().flatten()
    fb, _ = fast(cam, sph, n, mt, nm, 6, 77)
    ref, _ = rtw.render_flat(cam.raw, sph, n, mt, nm, 6, 177)
    others = [rtw.render_flat(cam.raw, sph, n, mt, nm, 6, 178 + i)[0] for i in range(8)]
    bias, within = gate(fb, ref, others)
    assert (bias <= BIAS_TOL).all(), bias
    assert within >= PIXEL_FRAC, within


def test_fast_errors_mirror_the_reference():
    cam, sph, n, mt, nm = rtw.builtin_scene("complex", SEED, 20, 30, 5)
    cam.raw.img_width = 0
    with pytest.raises(rtw.RtwError) as e:
        fast(cam, sph, n, mt, nm, 2, SEED)
    assert e.value.code == -2  # RTW_E_EMPTY_IMAGE (camera.rs:267)
