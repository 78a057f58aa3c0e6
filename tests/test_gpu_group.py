"""Device-resident multi-GPU groups (rtw_group_*, include/rtw_capi.h ABI 7) and the
f32 multi-device host call, on the one GPU of the test box.

A group renders image row r on entry r % n and gathers the row tiles on the root
device, then un-permutes them there (the node-level Camera::threaded_render,
camera.rs:223-352 with the pool of camera.rs:253 taking every GPU). With a
repeated device index the gather is device copies; `rccl_always` makes a
one-entry group gather through RCCL (ncclCommInitAll + ncclGather, one rank), so
the dlopen'ed RCCL path runs here too. Every image must be bit-identical to the
one-device one-shot render (the per-pixel RNG streams depend only on the global
pixel index, random.rs:61-69)."""
import numpy as np
import pytest

import raytracing_in_a_weekend_rust_amd as rtw
from oracle import oracle_ctypes as orc  # checker only

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

SEED = rtw.DEFAULT_SEED


def scene(h=27, w=48, depth=20):
    return rtw.builtin_scene("complex", SEED, h, w, depth)


def group_render(devices, cam, sph, n, mt, nm, s, fast=False, **kw):
    g = rtw.Group(devices, **kw)
    g.set_scene(sph, n, mt, nm)
    out = torch.full((cam.img_height, cam.img_width, 3), -1.0,
                     dtype=torch.float32 if fast else torch.float64, device="cuda:0")
    (g.render_fast if fast else g.render)(cam, s, SEED, out.data_ptr())
    total, per, info = g.stats()
    g.close()
    return out.cpu().numpy(), total, per, info


@pytest.mark.parametrize("devices,gather", [([0], "none"), ([0, 0], "copy"), ([0, 0, 0], "copy"),
                                            ([0] * 8, "copy")])
def test_group_matches_one_shot_and_oracle(devices, gather):
    cam, sph, n, mt, nm = scene()
    ref, seg = orc.render(cam.raw, sph, n, mt, nm, 2, SEED)
    fb, total, per, info = group_render(devices, cam.raw, sph, n, mt, nm, 2)
    assert info["gather"] == gather and info["n_entries"] == len(devices)
    assert np.array_equal(fb, ref), f"{int((fb != ref).sum())} channels differ"
    assert total.segments == seg == sum(p.segments for p in per)
    assert total.pixels == 27 * 48 and len(per) == len(devices)
    assert all(p.pixels == len(range(i, 27, len(devices))) * 48 for i, p in enumerate(per))
    assert 0 < total.main_kernel_ms <= total.kernel_ms
    assert info["wall_ms"] >= info["render_ms_max"] > 0


def test_group_rccl_gather_one_rank():
    cam, sph, n, mt, nm = scene()
    ref, seg = orc.render(cam.raw, sph, n, mt, nm, 2, SEED)
    fb, total, _, info = group_render([0], cam.raw, sph, n, mt, nm, 2, rccl_always=True)
    assert info["gather"] == "rccl"
    assert np.array_equal(fb, ref) and total.segments == seg


def test_group_more_entries_than_rows():
    cam, sph, n, mt, nm = scene(h=3, w=40, depth=10)
    ref, seg = orc.render(cam.raw, sph, n, mt, nm, 1, SEED)
    fb, total, per, info = group_render([0] * 5, cam.raw, sph, n, mt, nm, 1)
    assert info["n_entries"] == 3 and len(per) == 3
    assert np.array_equal(fb, ref) and total.segments == seg


def test_group_repeat_renders_and_scene_swap():
    cam, sph, n, mt, nm = scene()
    g = rtw.Group([0, 0])
    out = torch.zeros((27, 48, 3), dtype=torch.float64, device="cuda:0")
    g.set_scene(sph, n, mt, nm)
    g.render(cam.raw, 1, SEED, out.data_ptr())
    first = out.cpu().numpy().copy()
    cam2, sph2, n2, mt2, nm2 = rtw.builtin_scene("simple", SEED, 27, 48, 10)
    g.set_scene(sph2, n2, mt2, nm2)
    g.render(cam2.raw, 1, SEED, out.data_ptr())
    ref2, _ = orc.render(cam2.raw, sph2, n2, mt2, nm2, 1, SEED)
    assert np.array_equal(out.cpu().numpy(), ref2)
    g.set_scene(sph, n, mt, nm)
    g.render(cam.raw, 1, SEED, out.data_ptr())
    assert np.array_equal(out.cpu().numpy(), first)
    g.close()


def test_group_fast_matches_one_device_fast():
    cam, sph, n, mt, nm = scene()
    one, _ = rtw.render_flat_fast(cam.raw, sph, n, mt, nm, 2, SEED)
    fb, total, _, info = group_render([0, 0, 0], cam.raw, sph, n, mt, nm, 2, fast=True)
    assert info["gather"] == "copy" and info["fast"] == 1
    assert np.array_equal(fb, one), "fast mode is shard-invariant: the group must match bit for bit"
    assert total.pixels == 27 * 48


def test_multi_fast_matches_one_device_fast():
    cam, sph, n, mt, nm = scene()
    one, st1 = rtw.render_flat_fast(cam.raw, sph, n, mt, nm, 2, SEED)
    multi, st2 = rtw.render_flat_multi_fast(cam.raw, sph, n, mt, nm, 2, SEED, devices=[0, 0])
    assert np.array_equal(multi, one) and st1.segments == st2.segments


def test_camera_threaded_render_uses_every_device(tmp_path):
    """The Python mirror of camera.rs:223-227 goes through rtw_threaded_render_multi
    (every visible device) and still writes the reference's PPM."""
    cam, sph, n, mt, nm = scene(h=18, w=32, depth=10)
    world = rtw.SceneBuilder()
    mats = {}
    for i in range(n):
        k = sph[i].mat
        if k not in mats:
            m = mt[k]
            mats[k] = (rtw.Lambertian(tuple(m.albedo)) if m.kind == 0 else
                       rtw.Metal(tuple(m.albedo), m.fuzz) if m.kind == 1 else rtw.Dielectric(m.ir))
        world.add(rtw.Sphere.new_world_obj(*sph[i].center, sph[i].radius, mats[k]))
    ppm = tmp_path / "img.ppm"
    fb, st = rtw.Camera.threaded_render(cam, world.build(), 1, SEED, ppm_path=str(ppm))
    ref, seg = orc.render(cam.raw, sph, n, mt, nm, 1, SEED)
    assert np.array_equal(fb, ref) and st.segments == seg
    assert ppm.read_bytes() == orc.format_ppm(ref)


def test_group_orders_after_callers_null_stream():
    """The group's streams are non-blocking; its first write to `out` must still come
    after work the caller queued on the device's null stream (torch's default
    stream). A long spin then a fill of `out` precede the render: the render's
    image must be what is left."""
    cam, sph, n, mt, nm = scene()
    ref, _ = orc.render(cam.raw, sph, n, mt, nm, 2, SEED)
    assert torch.cuda.current_stream().cuda_stream == 0  # the null stream
    for devices in ([0], [0, 0]):
        g = rtw.Group(devices)
        g.set_scene(sph, n, mt, nm)
        out = torch.zeros((27, 48, 3), dtype=torch.float64, device="cuda:0")
        torch.cuda._sleep(200_000_000)  # ~0.1 s of spinning on the null stream
        out.fill_(-7.0)
        g.render(cam.raw, 2, SEED, out.data_ptr())
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), ref), devices
        g.close()


def test_group_orders_after_callers_stream():
    """Inside torch.cuda.stream(s) the caller's pending work is on s, not on the null
    stream: render(..., stream=s) orders the group's first write to `out` after it
    (ADVICE r05). A spin then a fill of `out` on s precede the render."""
    cam, sph, n, mt, nm = scene()
    ref, _ = orc.render(cam.raw, sph, n, mt, nm, 2, SEED)
    side = torch.cuda.Stream(device="cuda:0")
    for devices in ([0], [0, 0]):
        g = rtw.Group(devices)
        g.set_scene(sph, n, mt, nm)
        out = torch.zeros((27, 48, 3), dtype=torch.float64, device="cuda:0")
        torch.cuda.synchronize()
        with torch.cuda.stream(side):
            torch.cuda._sleep(200_000_000)  # ~0.1 s of spinning on the caller's stream
            out.fill_(-7.0)
            g.render(cam.raw, 2, SEED, out.data_ptr(), stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), ref), devices
        g.close()


_FALLBACK_CHILD = r"""
import sys, numpy as np, torch
import raytracing_in_a_weekend_rust_amd as rtw
SEED = rtw.DEFAULT_SEED
cam, sph, n, mt, nm = rtw.builtin_scene("complex", SEED, 27, 48, 20)
ref, st = rtw.render_flat(cam.raw, sph, n, mt, nm, 2, SEED)
ok, why = rtw.rccl_available()
assert not ok and "not loadable" in why, why
g = rtw.Group([0], rccl_try=True)
g.set_scene(sph, n, mt, nm)
out = torch.full((27, 48, 3), -1.0, dtype=torch.float64, device="cuda:0")
g.render(cam.raw, 2, SEED, out.data_ptr())
total, per, info = g.stats()
assert info["fallback"] == "rccl_unloadable" and info["gather"] == "none", info
assert "not loadable" in info["note"], info
assert np.array_equal(out.cpu().numpy(), ref) and total.segments == st.segments
g.close()
try:
    rtw.Group([0], rccl_always=True)
except rtw.RtwError as e:
    assert "not loadable" in str(e), e
else:
    raise AssertionError("rccl_always must fail without RCCL")
print("fallback ok")
"""


def test_group_falls_back_when_rccl_is_unloadable():
    """RCCL made unloadable (RTW_RCCL_SONAME under RTW_AB, in a child process: the
    library opens RCCL once per process): a group that would gather through RCCL
    falls back, says why, and renders the same image; RTW_GROUP_RCCL_ALWAYS fails
    loudly instead."""
    import os
    import subprocess
    import sys
    env = dict(os.environ, RTW_AB="1", RTW_RCCL_SONAME="librccl_missing_for_test.so")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", _FALLBACK_CHILD], cwd=root, env=env, capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0 and "fallback ok" in out.stdout, out.stdout + out.stderr


def test_group_rccl_try_uses_rccl_when_present():
    cam, sph, n, mt, nm = scene()
    ref, seg = orc.render(cam.raw, sph, n, mt, nm, 2, SEED)
    fb, total, _, info = group_render([0], cam.raw, sph, n, mt, nm, 2, rccl_try=True)
    assert info["gather"] == "rccl" and info["fallback"] == "none" and info["note"] == ""
    assert np.array_equal(fb, ref) and total.segments == seg


two_gpus = pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs 2 GPUs")


@two_gpus
@pytest.mark.parametrize("devices,kw,gather", [([0, 1], {}, "rccl"), ([0, 1], {"copy_gather": True}, "copy"),
                                               ([1, 0], {}, "rccl")])
def test_group_distinct_gpus(devices, kw, gather):
    """Distinct GPUs: the ncclGather over xGMI and the peer-copy gather, and a root
    that is not device 0 (the image lands on devices[0]); the caller's current
    device is restored."""
    cam, sph, n, mt, nm = scene()
    ref, seg = orc.render(cam.raw, sph, n, mt, nm, 2, SEED)
    torch.cuda.set_device(0)
    g = rtw.Group(devices, **kw)
    g.set_scene(sph, n, mt, nm)
    out = torch.full((27, 48, 3), -1.0, dtype=torch.float64, device=f"cuda:{devices[0]}")
    g.render(cam.raw, 2, SEED, out.data_ptr())
    assert torch.cuda.current_device() == 0
    total, per, info = g.stats()
    g.close()
    if gather == "rccl" and rtw.rccl_available()[0]:
        # RCCL is loadable here: a fallback would hide an RCCL regression
        assert info["gather"] == "rccl" and info["fallback"] == "none", info
    elif gather == "rccl":
        assert info["gather"] == "copy" and info["fallback"] != "none", info
    else:
        assert info["gather"] == "copy", info
    assert np.array_equal(out.cpu().numpy(), ref) and total.segments == seg
