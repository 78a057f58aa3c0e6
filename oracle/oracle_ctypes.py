"""TEST INFRASTRUCTURE ONLY: ctypes binding of the C oracle (oracle/rtw_oracle.c).

Used as the parity checker (tests/, __graft_entry__.smoke()) and as bench.py's
cpu_baseline leg. Struct layouts match include/rtw_capi.h byte for byte, so the
product's ctypes structs are passed straight through.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "librtw_oracle.so")

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"oracle not built: {LIB_PATH} (run `make -C oracle`)")
        L = C.CDLL(LIB_PATH)
        P = C.POINTER
        L.orc_xs_next_int.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32, P(C.c_uint64)]
        L.orc_xs_next_01.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32, P(C.c_double)]
        L.orc_xs_copy_reset_chain.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, P(C.c_uint64)]
        L.orc_interval_contains_inc.argtypes = [C.c_double] * 3
        L.orc_interval_contains_ex.argtypes = [C.c_double] * 3
        L.orc_camera_new.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, C.c_double, C.c_double,
                                     P(C.c_double), P(C.c_double), P(C.c_double), C.c_double,
                                     C.c_double, C.c_void_p]
        L.orc_offset_lattice.restype = C.c_uint32
        L.orc_offset_lattice.argtypes = [P(C.c_double), P(C.c_double), C.c_uint32, P(C.c_double)]
        L.orc_scene_complex.restype = C.c_uint32
        L.orc_scene_complex.argtypes = [C.c_uint64, C.c_uint64, C.c_void_p, C.c_void_p, C.c_uint32]
        L.orc_render.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32,
                                 C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32,
                                 C.c_uint32, C.c_uint32, C.c_int, P(C.c_double), P(C.c_uint64)]
        L.orc_render_rows.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32,
                                      C.c_uint32, C.c_uint64, C.c_uint64, P(C.c_uint32), C.c_uint32,
                                      C.c_uint32, C.c_int, P(C.c_double), P(C.c_uint64),
                                      P(C.c_uint64)]
        L.orc_format_ppm.restype = C.c_uint64
        L.orc_format_ppm.argtypes = [P(C.c_double), C.c_uint32, C.c_uint32, C.c_char_p, C.c_uint64]
        _lib = L
    return _lib


def split(v: int):
    v &= (1 << 128) - 1
    return v & 0xFFFFFFFFFFFFFFFF, v >> 64


def next_int(seed: int, n: int):
    out = (C.c_uint64 * (2 * n))()
    lib().orc_xs_next_int(*split(seed), n, out)
    return [out[2 * i] | (out[2 * i + 1] << 64) for i in range(n)]


def next_01(seed: int, n: int):
    out = (C.c_double * n)()
    lib().orc_xs_next_01(*split(seed), n, out)
    return list(out)


def copy_reset_chain(seed: int, n: int):
    out = (C.c_uint64 * (2 * n))()
    lib().orc_xs_copy_reset_chain(*split(seed), n, out)
    return [out[2 * i] | (out[2 * i + 1] << 64) for i in range(n)]


def camera_new(h, w, max_depth, focal_length, fov, look_from, look_to, vup, defocus_angle,
               focus_dist, cam_struct):
    a3 = C.c_double * 3
    lib().orc_camera_new(h, w, max_depth, focal_length, fov, a3(*look_from), a3(*look_to),
                         a3(*vup), defocus_angle, focus_dist, C.byref(cam_struct))
    return cam_struct


def offset_lattice(dx, dy, s):
    a3 = C.c_double * 3
    n = lib().orc_offset_lattice(a3(*dx), a3(*dy), s, None)
    out = (C.c_double * (3 * n))()
    lib().orc_offset_lattice(a3(*dx), a3(*dy), s, out)
    return [tuple(out[3 * i:3 * i + 3]) for i in range(n)]


def scene_complex(seed: int, sph_array, mat_array, cap: int) -> int:
    return lib().orc_scene_complex(*split(seed), C.byref(sph_array), C.byref(mat_array), cap)


def render(cam, sph, n_sph, mats, n_mats, samples_sqrt, seed, rows=None, nthreads=None,
           scheduler=1):
    """rows: None (all) or (row_begin, row_step, n_rows). Returns (fb, segments)."""
    if rows is None:
        rows = (0, 1, cam.img_height)
    b, step, n = rows
    nthreads = nthreads or min(16, os.cpu_count() or 1)
    out = np.zeros((n, cam.img_width, 3), dtype=np.float64)
    seg = C.c_uint64()
    rc = lib().orc_render(C.byref(cam), C.byref(sph), n_sph, C.byref(mats), n_mats, samples_sqrt,
                          *split(seed), b, step, n, nthreads, scheduler,
                          out.ctypes.data_as(C.POINTER(C.c_double)), C.byref(seg))
    if rc != 0:
        raise ValueError(f"orc_render failed: {rc}")
    return out, seg.value


def render_rows(cam, sph, n_sph, mats, n_mats, samples_sqrt, seed, rows, nthreads=None,
                scheduler=1):
    """rows: ascending image-row indices. Returns (fb [len(rows), W, 3], segments,
    per-row segments)."""
    rows = np.ascontiguousarray(rows, dtype=np.uint32)
    nthreads = nthreads or min(16, os.cpu_count() or 1)
    out = np.zeros((len(rows), cam.img_width, 3), dtype=np.float64)
    row_seg = np.zeros(len(rows), dtype=np.uint64)
    seg = C.c_uint64()
    rc = lib().orc_render_rows(C.byref(cam), C.byref(sph), n_sph, C.byref(mats), n_mats,
                               samples_sqrt, *split(seed),
                               rows.ctypes.data_as(C.POINTER(C.c_uint32)), len(rows), nthreads,
                               scheduler, out.ctypes.data_as(C.POINTER(C.c_double)), C.byref(seg),
                               row_seg.ctypes.data_as(C.POINTER(C.c_uint64)))
    if rc != 0:
        raise ValueError(f"orc_render_rows failed: {rc}")
    return out, seg.value, row_seg


def format_ppm(fb: np.ndarray) -> bytes:
    fb = np.ascontiguousarray(fb, dtype=np.float64)
    h, w = fb.shape[0], fb.shape[1]
    p = fb.ctypes.data_as(C.POINTER(C.c_double))
    n = lib().orc_format_ppm(p, w, h, None, 0)
    buf = C.create_string_buffer(n)
    lib().orc_format_ppm(p, w, h, buf, n)
    return buf.raw[:n]
