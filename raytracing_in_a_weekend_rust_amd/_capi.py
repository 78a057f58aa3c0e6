"""ctypes binding of librtw.so (include/rtw_capi.h).

The library is the product: HIP kernels for gfx950 plus the C++ host mirror of
the reference types. There is no Python or CPU fallback for the render: if the
shared library is missing, importing this module raises.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RTW_LIB") or os.path.join(_HERE, "_lib", "librtw.so")


class Vec3(C.Structure):
    _fields_ = [("x", C.c_double), ("y", C.c_double), ("z", C.c_double)]

    def tup(self):
        return (self.x, self.y, self.z)


class U128(C.Structure):
    _fields_ = [("lo", C.c_uint64), ("hi", C.c_uint64)]

    @staticmethod
    def of(v: int) -> "U128":
        v &= (1 << 128) - 1
        return U128(v & 0xFFFFFFFFFFFFFFFF, v >> 64)

    def value(self) -> int:
        return self.lo | (self.hi << 64)


class Camera(C.Structure):
    _fields_ = [
        ("img_height", C.c_uint32), ("img_width", C.c_uint32), ("max_depth", C.c_uint32),
        ("_pad0", C.c_uint32),
        ("focal_length", C.c_double), ("fov", C.c_double),
        ("look_from", Vec3), ("look_to", Vec3), ("vup", Vec3),
        ("u", Vec3), ("v", Vec3), ("w", Vec3),
        ("viewport_height", C.c_double), ("viewport_width", C.c_double),
        ("pixel00", Vec3), ("pixel_delta_u", Vec3), ("pixel_delta_v", Vec3),
        ("defocus_angle", C.c_double), ("focus_dist", C.c_double),
        ("defocus_disk_u", Vec3), ("defocus_disk_v", Vec3),
    ]


LAMBERTIAN, METAL, DIELECTRIC = 0, 1, 2


class Material(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("_pad", C.c_uint32), ("albedo", C.c_double * 3),
                ("fuzz", C.c_double), ("ir", C.c_double)]


class Sphere(C.Structure):
    _fields_ = [("center", C.c_double * 3), ("radius", C.c_double), ("mat", C.c_uint32),
                ("_pad", C.c_uint32)]


class Shard(C.Structure):
    _fields_ = [("row_begin", C.c_uint32), ("row_step", C.c_uint32), ("n_rows", C.c_uint32),
                ("_pad", C.c_uint32)]


class Stats(C.Structure):
    _fields_ = [("pixels", C.c_uint64), ("samples", C.c_uint64), ("segments", C.c_uint64),
                ("sphere_tests", C.c_uint64), ("wave_iterations", C.c_uint64),
                ("exact_tests", C.c_uint64), ("exact_wave_iterations", C.c_uint64),
                ("kernel_ms", C.c_double), ("grid_blocks", C.c_uint32),
                ("block_threads", C.c_uint32), ("node_visits", C.c_uint64),
                ("brute_segments", C.c_uint64), ("accel", C.c_uint32), ("lds_bytes", C.c_uint32),
                ("parked_pixels", C.c_uint64), ("inside_segments", C.c_uint64),
                ("trap_segments", C.c_uint64), ("guard_exits", C.c_uint64),
                ("leftover_pixels", C.c_uint64), ("main_kernel_ms", C.c_double)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class GroupInfo(C.Structure):
    _fields_ = [("n_entries", C.c_uint32), ("gather", C.c_uint32), ("wall_ms", C.c_double),
                ("render_ms_max", C.c_double), ("root_gather_ms", C.c_double),
                ("fast", C.c_uint32), ("fallback", C.c_uint32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_ if not k.startswith("_")}


GATHER_NAMES = {0: "none", 1: "copy", 2: "rccl"}
FALLBACK_NAMES = {0: "none", 1: "rccl_unloadable", 2: "comm_init_failed"}
GROUP_COPY_GATHER = 1
GROUP_RCCL_ALWAYS = 2
GROUP_RCCL_TRY = 4

RTW_OK = 0
ERRORS = {-1: "RTW_E_ARG", -2: "RTW_E_EMPTY_IMAGE", -3: "RTW_E_FUZZ", -4: "RTW_E_MAT_INDEX",
          -5: "RTW_E_HIP", -6: "RTW_E_UNSUPPORTED", -7: "RTW_E_NO_DEVICE", -8: "RTW_E_CAPACITY"}

# name -> (restype, argtypes); every symbol include/rtw_capi.h declares.
_P = C.POINTER
SIGNATURES = {
    "rtw_version": (C.c_char_p, []),
    "rtw_abi_version": (C.c_int, []),
    "rtw_build_id": (C.c_char_p, []),
    "rtw_last_error": (C.c_char_p, []),
    "rtw_shutdown": (C.c_int, []),
    "rtw_device_count": (C.c_int, [_P(C.c_int)]),
    "rtw_camera_new": (C.c_int, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_double, C.c_double,
                                 _P(Vec3), _P(Vec3), _P(Vec3), C.c_double, C.c_double,
                                 _P(Camera)]),
    "rtw_offset_lattice": (C.c_int, [_P(Vec3), _P(Vec3), C.c_uint32, _P(Vec3), C.c_uint32,
                                     _P(C.c_uint32)]),
    "rtw_interval_contains_inc": (C.c_int, [C.c_double, C.c_double, C.c_double]),
    "rtw_interval_contains_ex": (C.c_int, [C.c_double, C.c_double, C.c_double]),
    "rtw_xorshift_next_int": (C.c_int, [U128, C.c_uint32, _P(U128)]),
    "rtw_xorshift_next_01": (C.c_int, [U128, C.c_uint32, _P(C.c_double)]),
    "rtw_seed_children": (C.c_int, [U128, C.c_uint64, C.c_uint64, _P(U128)]),
    "rtw_scene_builtin": (C.c_int, [C.c_char_p, U128, C.c_uint32, C.c_uint32, C.c_uint32,
                                    _P(Camera), _P(Sphere), _P(Material), C.c_uint32,
                                    _P(C.c_uint32), _P(C.c_uint32)]),
    "rtw_format_ppm": (C.c_int64, [_P(C.c_double), C.c_uint32, C.c_uint32, C.c_char_p,
                                   C.c_uint64]),
    "rtw_write_ppm": (C.c_int, [C.c_char_p, _P(C.c_double), C.c_uint32, C.c_uint32]),
    "rtw_threaded_render": (C.c_int, [_P(Camera), _P(Sphere), C.c_uint32, _P(Material),
                                      C.c_uint32, C.c_uint32, U128, _P(Shard),
                                      _P(C.c_double), _P(Stats)]),
    "rtw_threaded_render_multi": (C.c_int, [_P(Camera), _P(Sphere), C.c_uint32, _P(Material),
                                            C.c_uint32, C.c_uint32, U128, _P(C.c_int), C.c_uint32,
                                            _P(C.c_double), _P(Stats)]),
    "rtw_threaded_render_multi_fast": (C.c_int, [_P(Camera), _P(Sphere), C.c_uint32, _P(Material),
                                                 C.c_uint32, C.c_uint32, U128, _P(C.c_int),
                                                 C.c_uint32, _P(C.c_float), _P(Stats)]),
    "rtw_group_create": (C.c_int, [_P(C.c_int), C.c_uint32, C.c_uint32, _P(C.c_void_p)]),
    "rtw_group_destroy": (C.c_int, [C.c_void_p]),
    "rtw_group_set_scene": (C.c_int, [C.c_void_p, _P(Sphere), C.c_uint32, _P(Material),
                                      C.c_uint32]),
    "rtw_group_render": (C.c_int, [C.c_void_p, _P(Camera), C.c_uint32, U128, C.c_void_p]),
    "rtw_group_render_fast": (C.c_int, [C.c_void_p, _P(Camera), C.c_uint32, U128, C.c_void_p]),
    "rtw_group_render_on": (C.c_int, [C.c_void_p, _P(Camera), C.c_uint32, U128, C.c_void_p, C.c_void_p]),
    "rtw_group_render_fast_on": (C.c_int, [C.c_void_p, _P(Camera), C.c_uint32, U128, C.c_void_p,
                                           C.c_void_p]),
    "rtw_group_stats": (C.c_int, [C.c_void_p, _P(Stats), _P(Stats), C.c_uint32, _P(GroupInfo)]),
    "rtw_group_note": (C.c_char_p, [C.c_void_p]),
    "rtw_rccl_available": (C.c_int, [C.c_char_p, C.c_size_t]),
    "rtw_threaded_render_fast": (C.c_int, [_P(Camera), _P(Sphere), C.c_uint32, _P(Material),
                                           C.c_uint32, C.c_uint32, U128, _P(Shard),
                                           _P(C.c_float), _P(Stats)]),
    "rtw_session_create": (C.c_int, [C.c_int, _P(C.c_void_p)]),
    "rtw_session_destroy": (C.c_int, [C.c_void_p]),
    "rtw_session_set_scene": (C.c_int, [C.c_void_p, _P(Sphere), C.c_uint32, _P(Material),
                                        C.c_uint32]),
    "rtw_session_render": (C.c_int, [C.c_void_p, _P(Camera), C.c_uint32, U128, _P(Shard),
                                     C.c_void_p, C.c_void_p]),
    "rtw_session_render_fast": (C.c_int, [C.c_void_p, _P(Camera), C.c_uint32, U128, _P(Shard),
                                          C.c_void_p, C.c_void_p]),
    "rtw_session_stats": (C.c_int, [C.c_void_p, _P(Stats)]),
    "rtw_session_diag": (C.c_int, [C.c_void_p, _P(C.c_uint32), C.c_uint64]),
    "rtw_probe_device_seeds": (C.c_int, [C.c_int, U128, C.c_uint64, C.c_uint64, _P(U128)]),
    "rtw_probe_f64_ops": (C.c_int, [C.c_int, _P(C.c_double), _P(C.c_double), C.c_uint64,
                                    _P(C.c_double), _P(C.c_double)]),
}


class RtwError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


def _load():
    # One HIP runtime per process. torch ships its own libamdhip64 (soname
    # libamdhip64.so.7, requested by torch as "libamdhip64.so"). If librtw.so
    # loaded /opt/rocm's copy first, torch would map a second runtime and find no
    # GPU; loading torch first makes librtw.so bind to torch's copy (same soname),
    # so torch streams and tensors are valid handles for the C ABI.
    if os.environ.get("RTW_NO_TORCH", "0") != "1":
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"librtw.so not built at {LIB_PATH}: run `make` (or __graft_entry__.build()). "
            "There is no fallback render path.")
    lib = C.CDLL(LIB_PATH)
    # the ABI check comes before any other symbol is bound: a stale library that
    # predates a symbol is reported as such, not as an AttributeError
    if not hasattr(lib, "rtw_abi_version"):
        raise ImportError(f"{LIB_PATH} predates rtw_abi_version (ABI < 6): rebuild with `make`")
    lib.rtw_abi_version.restype = C.c_int
    lib.rtw_abi_version.argtypes = []
    if lib.rtw_abi_version() != ABI_VERSION:
        raise ImportError(f"{LIB_PATH} has ABI {lib.rtw_abi_version()}, this binding expects "
                          f"{ABI_VERSION}: rebuild with `make`")
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


ABI_VERSION = 7  # include/rtw_capi.h RTW_ABI_VERSION this binding's structs follow
lib = _load()


def check(rc: int) -> int:
    if rc < 0:
        raise RtwError(rc, lib.rtw_last_error().decode())
    return rc
