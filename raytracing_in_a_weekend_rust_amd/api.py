"""Python mirror of the reference's trait surface for the sampling path, over the
C ABI (include/rtw_capi.h). Same names and argument order as the reference:

    cam = Camera.new(height, width, max_depth, focal_length, fov,
                     look_from, look_to, vup, defocus_angle, focus_dist)   # camera.rs:138-150
    world = SceneBuilder(); world.add(Sphere.new_world_obj(x, y, z, r, mat)); world.build()
    Camera.threaded_render(cam, world, samples_sqrt, seed=...)             # camera.rs:223-227

Rendering always runs the HIP megakernel in librtw.so; there is no Python/CPU
render path. Errors the reference raises by assert!/panic come back as RtwError
with the matching RTW_E_* code.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _capi as capi
from ._capi import RtwError, check, lib

DEFAULT_SEED = 1764892800000  # ms since epoch at 2025-12-05T00:00Z (XorShift::default stand-in)


def _v(t) -> capi.Vec3:
    return capi.Vec3(float(t[0]), float(t[1]), float(t[2]))


# ---------------------------------------------------------------- materials --
class Material:
    def flatten(self) -> capi.Material:
        raise NotImplementedError


@dataclass(eq=False)
class Lambertian(Material):  # materials.rs:11-20
    albedo: tuple

    def flatten(self):
        m = capi.Material()
        m.kind = capi.LAMBERTIAN
        m.albedo[:] = [float(a) for a in self.albedo]
        return m


@dataclass(eq=False)
class Metal(Material):  # materials.rs:39-50
    albedo: tuple
    fuzz: float

    def __post_init__(self):
        if not self.fuzz <= 1.0:  # assert!(fuzz <= 1.), materials.rs:47
            raise RtwError(-3, "Fuzz cannot be more than 1")

    def flatten(self):
        m = capi.Material()
        m.kind = capi.METAL
        m.albedo[:] = [float(a) for a in self.albedo]
        m.fuzz = float(self.fuzz)
        return m


@dataclass(eq=False)
class Dielectric(Material):  # materials.rs:65-73
    ir: float

    def flatten(self):
        m = capi.Material()
        m.kind = capi.DIELECTRIC
        m.ir = float(self.ir)
        return m


# ---------------------------------------------------------------- hittables --
@dataclass(eq=False)
class Sphere:  # sphere.rs:11-37
    center: tuple
    radius: float
    mat: Material

    @staticmethod
    def new_world_obj(x, y, z, radius, mat) -> "Sphere":
        return Sphere((x, y, z), radius, mat)


@dataclass(eq=False)
class Scene:  # hittable.rs:119-143
    objects: list = field(default_factory=list)

    def flatten(self):
        """Sphere and material tables in insertion order; materials are shared
        by identity like Arc<dyn Material>. An empty scene flattens to zero
        spheres (the reference's `Empty`, hittable.rs:98-106)."""
        mats, index = [], {}
        sph = (capi.Sphere * max(1, len(self.objects)))()
        for i, o in enumerate(self.objects):
            if id(o.mat) not in index:
                index[id(o.mat)] = len(mats)
                mats.append(o.mat.flatten())
            s = sph[i]
            s.center[:] = [float(c) for c in o.center]
            s.radius = float(o.radius)
            s.mat = index[id(o.mat)]
        mt = (capi.Material * max(1, len(mats)))(*mats)
        return sph, len(self.objects), mt, len(mats)


class SceneBuilder:  # hittable.rs:86-117
    def __init__(self):
        self.objects = []

    def add(self, obj):
        self.objects.append(obj)

    def build(self) -> Scene:
        return Scene(list(self.objects))


# ------------------------------------------------------------------- camera --
class Camera:
    """Wraps rtw_camera (the derived values of Camera::new)."""

    def __init__(self, raw: capi.Camera):
        self.raw = raw

    @staticmethod
    def new(img_height, img_width, max_depth, focal_length, fov, look_from, look_to, vup,
            defocus_angle, focus_dist) -> "Camera":
        raw = capi.Camera()
        check(lib.rtw_camera_new(img_height, img_width, max_depth, focal_length, fov,
                                 C.byref(_v(look_from)), C.byref(_v(look_to)), C.byref(_v(vup)),
                                 defocus_angle, focus_dist, C.byref(raw)))
        return Camera(raw)

    def width(self):
        return self.raw.img_width

    def height(self):
        return self.raw.img_height

    @staticmethod
    def offset_lattice(dx, dy, num_layers):  # camera.rs:422-450
        n = C.c_uint32()
        lib.rtw_offset_lattice(C.byref(_v(dx)), C.byref(_v(dy)), num_layers, None, 0, C.byref(n))
        out = (capi.Vec3 * max(1, n.value))()
        check(lib.rtw_offset_lattice(C.byref(_v(dx)), C.byref(_v(dy)), num_layers, out, n.value,
                                     C.byref(n)))
        return [out[i].tup() for i in range(n.value)]

    @staticmethod
    def threaded_render(cam: "Camera", world: Scene, samples_sqrt: int, seed: int = DEFAULT_SEED,
                        ppm_path: str | None = "img.ppm", shard=None, devices=None):
        """camera.rs:223-352 on the GPUs of this node: the reference's pool takes every
        core (camera.rs:253), this takes every visible GPU (`devices` None) or the
        listed ones (rtw_threaded_render_multi). `shard` renders only those rows, on
        one device (rtw_threaded_render). Returns (framebuffer HxWx3 f64, stats)."""
        sph, ns, mt, nm = world.flatten()
        if shard is not None:
            fb, st = render_flat(cam.raw, sph, ns, mt, nm, samples_sqrt, seed, shard)
        else:
            fb, st = render_flat_multi(cam.raw, sph, ns, mt, nm, samples_sqrt, seed, devices)
        if ppm_path is not None and shard is None:
            write_ppm(ppm_path, fb)
        return fb, st


# ---------------------------------------------------------------- functions --
def builtin_scene(name: str, seed: int = DEFAULT_SEED, height=0, width=0, max_depth=0):
    """Flattened built-in scene (raytracing/mod.rs): (Camera, spheres, n, mats, nm)."""
    ns, nm = C.c_uint32(), C.c_uint32()
    cam = capi.Camera()
    rc = lib.rtw_scene_builtin(name.encode(), capi.U128.of(seed), height, width, max_depth,
                               C.byref(cam), None, None, 0, C.byref(ns), C.byref(nm))
    if rc not in (0, -8):
        check(rc)
    cap = max(ns.value, nm.value, 1)
    sph, mt = (capi.Sphere * cap)(), (capi.Material * cap)()
    check(lib.rtw_scene_builtin(name.encode(), capi.U128.of(seed), height, width, max_depth,
                                C.byref(cam), sph, mt, cap, C.byref(ns), C.byref(nm)))
    return Camera(cam), sph, ns.value, mt, nm.value


def _shard(shard):
    if shard is None:
        return None
    if isinstance(shard, capi.Shard):
        return shard
    b, step, n = shard
    return capi.Shard(b, step, n, 0)


def render_flat(cam: capi.Camera, sph, n_sph, mats, n_mats, samples_sqrt, seed=DEFAULT_SEED,
                shard=None):
    """rtw_threaded_render: host buffers in, (n_rows x W x 3 f64, Stats) out."""
    sh = _shard(shard)
    n_rows = cam.img_height if sh is None else sh.n_rows
    fb = np.zeros((n_rows, cam.img_width, 3), dtype=np.float64)
    st = capi.Stats()
    check(lib.rtw_threaded_render(C.byref(cam), sph, n_sph, mats, n_mats, samples_sqrt,
                                  capi.U128.of(seed), C.byref(sh) if sh is not None else None,
                                  fb.ctypes.data_as(C.POINTER(C.c_double)), C.byref(st)))
    return fb, st


def render_flat_multi(cam: capi.Camera, sph, n_sph, mats, n_mats, samples_sqrt, seed=DEFAULT_SEED,
                      devices=None):
    """rtw_threaded_render_multi: the whole image over a list of GPUs (None = every
    visible device; an index may repeat), rows dealt cyclically, gathered by strided
    device-to-host copies into one host framebuffer. Returns (H x W x 3 f64, Stats)."""
    fb = np.zeros((cam.img_height, cam.img_width, 3), dtype=np.float64)
    st = capi.Stats()
    devs = list(devices or [])
    arr = (C.c_int * max(1, len(devs)))(*devs)
    check(lib.rtw_threaded_render_multi(C.byref(cam), sph, n_sph, mats, n_mats, samples_sqrt,
                                        capi.U128.of(seed), arr if devs else None, len(devs),
                                        fb.ctypes.data_as(C.POINTER(C.c_double)), C.byref(st)))
    return fb, st


def render_flat_multi_fast(cam: capi.Camera, sph, n_sph, mats, n_mats, samples_sqrt,
                           seed=DEFAULT_SEED, devices=None):
    """rtw_threaded_render_multi_fast: render_flat_multi in f32 fast mode."""
    fb = np.zeros((cam.img_height, cam.img_width, 3), dtype=np.float32)
    st = capi.Stats()
    devs = list(devices or [])
    arr = (C.c_int * max(1, len(devs)))(*devs)
    check(lib.rtw_threaded_render_multi_fast(C.byref(cam), sph, n_sph, mats, n_mats, samples_sqrt,
                                             capi.U128.of(seed), arr if devs else None, len(devs),
                                             fb.ctypes.data_as(C.POINTER(C.c_float)), C.byref(st)))
    return fb, st


def shutdown():
    """rtw_shutdown: frees the device resources of the one-shot and multi-GPU calls."""
    check(lib.rtw_shutdown())


def build_id() -> str:
    return lib.rtw_build_id().decode()


def render_flat_fast(cam: capi.Camera, sph, n_sph, mats, n_mats, samples_sqrt, seed=DEFAULT_SEED,
                     shard=None):
    """rtw_threaded_render_fast (f32 fast mode, statistical parity): host buffers in,
    (n_rows x W x 3 f32, Stats) out."""
    sh = _shard(shard)
    n_rows = cam.img_height if sh is None else sh.n_rows
    fb = np.zeros((n_rows, cam.img_width, 3), dtype=np.float32)
    st = capi.Stats()
    check(lib.rtw_threaded_render_fast(C.byref(cam), sph, n_sph, mats, n_mats, samples_sqrt,
                                       capi.U128.of(seed), C.byref(sh) if sh is not None else None,
                                       fb.ctypes.data_as(C.POINTER(C.c_float)), C.byref(st)))
    return fb, st


def format_ppm(fb: np.ndarray) -> bytes:
    fb = np.ascontiguousarray(fb, dtype=np.float64)
    h, w = fb.shape[0], fb.shape[1]
    p = fb.ctypes.data_as(C.POINTER(C.c_double))
    # one formatting pass in the common case: values in [0, 1] give <= 4 bytes a
    # channel; the size query + second call only when a brighter image overflows
    cap = 12 * w * h + h + 64
    buf = C.create_string_buffer(cap)
    n = check(lib.rtw_format_ppm(p, w, h, buf, cap))
    if n > cap:
        buf = C.create_string_buffer(n)
        check(lib.rtw_format_ppm(p, w, h, buf, n))
    return C.string_at(buf, n)


def write_ppm(path: str, fb: np.ndarray):
    fb = np.ascontiguousarray(fb, dtype=np.float64)
    check(lib.rtw_write_ppm(path.encode(), fb.ctypes.data_as(C.POINTER(C.c_double)),
                            fb.shape[1], fb.shape[0]))


def xorshift_next_int(seed: int, n: int):
    out = (capi.U128 * max(1, n))()
    check(lib.rtw_xorshift_next_int(capi.U128.of(seed), n, out))
    return [out[i].value() for i in range(n)]


def xorshift_next_01(seed: int, n: int):
    out = (C.c_double * max(1, n))()
    check(lib.rtw_xorshift_next_01(capi.U128.of(seed), n, out))
    return list(out[:n])


def seed_children(seed: int, first_pixel: int, count: int):
    out = (capi.U128 * max(1, count))()
    check(lib.rtw_seed_children(capi.U128.of(seed), first_pixel, count, out))
    return [out[i].value() for i in range(count)]


def device_count() -> int:
    n = C.c_int()
    check(lib.rtw_device_count(C.byref(n)))
    return n.value


class Session:
    """Device-resident rendering (rtw_session_*): the scene lives in HBM; renders
    are enqueued on a caller HIP stream into a caller device buffer."""

    def __init__(self, device: int = 0):
        self.h = C.c_void_p()
        check(lib.rtw_session_create(device, C.byref(self.h)))

    def set_scene(self, sph, n_sph, mats, n_mats):
        check(lib.rtw_session_set_scene(self.h, sph, n_sph, mats, n_mats))

    def render(self, cam: capi.Camera, samples_sqrt: int, seed: int, out_dev_ptr: int,
               stream: int | None = None, shard=None):
        sh = _shard(shard)
        check(lib.rtw_session_render(self.h, C.byref(cam), samples_sqrt, capi.U128.of(seed),
                                     C.byref(sh) if sh is not None else None,
                                     C.c_void_p(out_dev_ptr), C.c_void_p(stream or 0)))

    def render_fast(self, cam: capi.Camera, samples_sqrt: int, seed: int, out_dev_ptr: int,
                    stream: int | None = None, shard=None):
        """f32 fast mode into an n_rows x W x 3 f32 device buffer."""
        sh = _shard(shard)
        check(lib.rtw_session_render_fast(self.h, C.byref(cam), samples_sqrt, capi.U128.of(seed),
                                          C.byref(sh) if sh is not None else None,
                                          C.c_void_p(out_dev_ptr), C.c_void_p(stream or 0)))

    def stats(self) -> capi.Stats:
        st = capi.Stats()
        check(lib.rtw_session_stats(self.h, C.byref(st)))
        return st

    def diag(self, n_pixels: int):
        """RTW_DIAG=1 renders: per-pixel (segments, clock/1024 at completion)."""
        import numpy as np
        out = np.zeros(2 * n_pixels + 4, dtype=np.uint32)
        check(lib.rtw_session_diag(self.h, out.ctypes.data_as(C.POINTER(C.c_uint32)), out.size))
        return out[:2 * n_pixels].reshape(n_pixels, 2), int(out[2 * n_pixels])

    def diag_events(self, n_pixels: int):
        """RTW_DIAG=2 renders: per pixel (segments, completion, hand-out, first park,
        first drain claim) as raw 100 MHz clock words (0: never), and the launch start."""
        import numpy as np
        out = np.zeros(5 * n_pixels + 4, dtype=np.uint32)
        check(lib.rtw_session_diag(self.h, out.ctypes.data_as(C.POINTER(C.c_uint32)), out.size))
        rec = out[:2 * n_pixels].reshape(n_pixels, 2)
        ev = out[2 * n_pixels + 4:].reshape(n_pixels, 3)
        return np.concatenate([rec, ev], axis=1), int(out[2 * n_pixels])

    def close(self):
        if self.h:
            lib.rtw_session_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def rccl_available():
    """(True, "") if RCCL (librccl.so.1 with ncclGather) can be loaded, else (False,
    why). Needs no GPU."""
    buf = C.create_string_buffer(256)
    ok = lib.rtw_rccl_available(buf, len(buf))
    return bool(ok), buf.value.decode()


class Group:
    """Device-resident multi-GPU renders (rtw_group_*): one session per device entry
    (None = every visible device; an index may repeat), rows dealt cyclically, the
    row tiles gathered on the root device (entry 0) by ncclGather over xGMI when the
    entries are distinct GPUs (device copies otherwise, or when RCCL cannot be loaded
    or initialised: `stats()[2]["fallback"]` and `note()` say why) and un-permuted
    there into a caller device buffer. Blocking renders. rccl_always: RCCL even for
    one entry, an RCCL failure is an error; rccl_try: RCCL even for one entry, with
    the fallback."""

    def __init__(self, devices=None, copy_gather: bool = False, rccl_always: bool = False,
                 rccl_try: bool = False):
        self.h = C.c_void_p()
        devs = list(devices or [])
        arr = (C.c_int * max(1, len(devs)))(*devs)
        flags = ((capi.GROUP_COPY_GATHER if copy_gather else 0) | (capi.GROUP_RCCL_ALWAYS if rccl_always else 0)
                 | (capi.GROUP_RCCL_TRY if rccl_try else 0))
        check(lib.rtw_group_create(arr if devs else None, len(devs), flags, C.byref(self.h)))

    def set_scene(self, sph, n_sph, mats, n_mats):
        check(lib.rtw_group_set_scene(self.h, sph, n_sph, mats, n_mats))

    def render(self, cam: capi.Camera, samples_sqrt: int, seed: int, out_dev_ptr: int, stream: int = 0):
        """The whole image into an H x W x 3 f64 buffer on the root device, ordered after
        the work queued on `stream` (a hipStream_t handle of the root device, e.g.
        torch.cuda.current_stream().cuda_stream; 0 = the null stream)."""
        check(lib.rtw_group_render_on(self.h, C.byref(cam), samples_sqrt, capi.U128.of(seed),
                                      C.c_void_p(out_dev_ptr), C.c_void_p(stream or None)))

    def render_fast(self, cam: capi.Camera, samples_sqrt: int, seed: int, out_dev_ptr: int, stream: int = 0):
        """f32 fast mode into an H x W x 3 f32 buffer on the root device (`stream` as render)."""
        check(lib.rtw_group_render_fast_on(self.h, C.byref(cam), samples_sqrt, capi.U128.of(seed),
                                           C.c_void_p(out_dev_ptr), C.c_void_p(stream or None)))

    def stats(self):
        """(total Stats, [per-entry Stats], info dict) of the last render."""
        info = capi.GroupInfo()
        check(lib.rtw_group_stats(self.h, None, None, 0, C.byref(info)))
        total = capi.Stats()
        per = (capi.Stats * max(1, info.n_entries))()
        check(lib.rtw_group_stats(self.h, C.byref(total), per, max(1, info.n_entries), C.byref(info)))
        d = info.as_dict()
        d["gather"] = capi.GATHER_NAMES.get(info.gather, info.gather)
        d["fallback"] = capi.FALLBACK_NAMES.get(info.fallback, info.fallback)
        d["note"] = self.note()
        return total, [per[i] for i in range(info.n_entries)], d

    def note(self) -> str:
        """Why the group gathers by device copies although its entries are distinct
        GPUs ("" when it does not)."""
        return (lib.rtw_group_note(self.h) or b"").decode()

    def close(self):
        if self.h:
            lib.rtw_group_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
