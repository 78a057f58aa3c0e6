"""Generates the committed golden fixtures in tests/golden/ from the pure-Python
restatement (oracle/pyoracle.py), cross-checking every value against the C
restatement (oracle/rtw_oracle.c) before writing. The reference itself (Rust)
cannot be built or run in this image (no cargo/rustc), and its own tests pin no
pixel/RNG values, so these fixtures are restatement-generated ("parity unpinned"
by the reference). Run from the repo root:

    python tests/golden/make_golden.py
"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import oracle_ctypes as orc  # noqa: E402
from oracle import pyoracle as py  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")
SEEDS = [1764892800000, 1, 0xDEADBEEFCAFEBABE0123456789ABCDEF, (1 << 127) + 12345]


class OCam(C.Structure):  # same layout as orc_camera / rtw_camera
    _fields_ = [("img_height", C.c_uint32), ("img_width", C.c_uint32), ("max_depth", C.c_uint32),
                ("_pad0", C.c_uint32), ("focal_length", C.c_double), ("fov", C.c_double)] + \
               [(n, C.c_double * 3) for n in ("look_from", "look_to", "vup", "u", "v", "w")] + \
               [("viewport_height", C.c_double), ("viewport_width", C.c_double)] + \
               [(n, C.c_double * 3) for n in ("pixel00", "pixel_delta_u", "pixel_delta_v")] + \
               [("defocus_angle", C.c_double), ("focus_dist", C.c_double)] + \
               [(n, C.c_double * 3) for n in ("defocus_disk_u", "defocus_disk_v")]


class OSph(C.Structure):
    _fields_ = [("center", C.c_double * 3), ("radius", C.c_double), ("mat", C.c_uint32),
                ("_pad", C.c_uint32)]


class OMat(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("_pad", C.c_uint32), ("albedo", C.c_double * 3),
                ("fuzz", C.c_double), ("ir", C.c_double)]


def hx(v):
    return float(v).hex()


def hv(t):
    return [hx(x) for x in t]


def c_camera(pc):
    cam = OCam()
    orc.camera_new(pc.height, pc.width, pc.max_depth, pc.focal_length, pc.fov, pc.look_from,
                   pc.look_to, pc.vup, pc.defocus_angle, pc.focus_dist, cam)
    return cam


def c_scene(objs):
    sph, mat = (OSph * len(objs))(), (OMat * len(objs))()
    for i, (c, r, m) in enumerate(objs):
        sph[i].center[:] = list(c)
        sph[i].radius = r
        sph[i].mat = i
        mat[i].kind = m[0]
        mat[i].albedo[:] = list(m[1])
        mat[i].fuzz = m[2]
        mat[i].ir = m[3]
    return sph, mat


def xorshift():
    out = []
    for seed in SEEDS:
        x = py.XorShift(seed)
        ints = [x.next_int() for _ in range(64)]
        x = py.XorShift(seed)
        f01 = [x.next_01() for _ in range(256)]
        x = py.XorShift(seed)
        kids = [x.copy_reset().state for _ in range(64)]
        assert ints == orc.next_int(seed, 64)
        assert f01 == orc.next_01(seed, 256)
        assert kids == orc.copy_reset_chain(seed, 64)
        x = py.XorShift(seed)
        b = x.next_bound(-1.0, 1.0)
        out.append({"seed": hex(seed), "next_int": [hex(v) for v in ints],
                    "next_01": [hx(v) for v in f01], "copy_reset": [hex(v) for v in kids],
                    "next_bound_m1_1": hx(b)})
    # far children of the copy_reset chain (pixel indices of a 1200x675 image)
    seed = SEEDS[0]
    far = [0, 1, 1199, 1200, 405_000, 809_999]
    chain = orc.copy_reset_chain(seed, far[-1] + 1)
    x = py.XorShift(seed)
    pyk = []
    for p in range(far[-1] + 1):
        k = x.copy_reset().state
        if p in far:
            pyk.append(k)
    assert pyk == [chain[p] for p in far]
    return {"streams": out, "far_children": {"seed": hex(seed), "pixels": far,
                                             "children": [hex(v) for v in pyk]}}


def scene_json(seed):
    objs = py.scene_complex(seed)
    sph, mat = (OSph * 600)(), (OMat * 600)()
    n = orc.scene_complex(seed, sph, mat, 600)
    assert n == len(objs)
    for i, (c, r, m) in enumerate(objs):
        assert tuple(sph[i].center) == c and sph[i].radius == r
        assert (mat[i].kind, tuple(mat[i].albedo), mat[i].fuzz, mat[i].ir) == m
    return {"seed": hex(seed), "n": len(objs),
            "spheres": [{"center": hv(c), "radius": hx(r), "kind": m[0], "albedo": hv(m[1]),
                         "fuzz": hx(m[2]), "ir": hx(m[3])} for c, r, m in objs]}


def camera_json(pc):
    cam = c_camera(pc)
    d = {}
    for name, val in (("pixel00", pc.pixel00), ("pixel_delta_u", pc.pixel_delta_u),
                      ("pixel_delta_v", pc.pixel_delta_v), ("u", pc.u), ("v", pc.v), ("w", pc.w),
                      ("defocus_disk_u", pc.defocus_disk_u), ("defocus_disk_v", pc.defocus_disk_v)):
        assert tuple(getattr(cam, name)) == val, name
        d[name] = hv(val)
    assert cam.viewport_height == pc.viewport_height and cam.viewport_width == pc.viewport_width
    d["viewport_height"] = hx(pc.viewport_height)
    d["viewport_width"] = hx(pc.viewport_width)
    return d


RENDERS = [  # (file, scene, seed, h, w, max_depth, samples_sqrt)
    ("render_three_lambertian_40x23_s2_d8", "three_lambertian", SEEDS[0], 23, 40, 8, 2),
    ("render_complex_16x9_s1_d10", "complex", SEEDS[0], 9, 16, 10, 1),
    ("render_complex_24x14_s0_d50", "complex", SEEDS[1], 14, 24, 50, 0),
    ("render_simple_32x18_s2_d25", "simple", SEEDS[0], 18, 32, 25, 2),
    ("render_super_simple_12x12_s3_d50", "super_simple", SEEDS[2], 12, 12, 50, 3),
]


def render_json(scene, seed, h, w, d, s):
    import numpy as np

    pc, objs = py.scene_builtin(scene, seed, h, w, d)
    img, seg = py.render(pc, objs, s, seed)
    cam = c_camera(pc)
    sph, mat = c_scene(objs)
    fb = np.zeros((h, w, 3))
    segc = C.c_uint64()
    rc = orc.lib().orc_render(C.byref(cam), C.byref(sph), len(objs), C.byref(mat), len(objs), s,
                              *orc.split(seed), 0, 1, h, 4, 1,
                              fb.ctypes.data_as(C.POINTER(C.c_double)), C.byref(segc))
    assert rc == 0
    for (x, y), col in img.items():
        assert tuple(fb[y, x]) == col, (x, y)
    assert seg == segc.value
    ppm = py.format_ppm(img, w, h)
    assert ppm.encode() == orc.format_ppm(fb)
    return {"scene": scene, "seed": hex(seed), "height": h, "width": w, "max_depth": d,
            "samples_sqrt": s, "segments": seg,
            "framebuffer": [hx(v) for y in range(h) for x in range(w) for v in img[(x, y)]],
            "ppm": ppm}


def main():
    def dump(name, obj):
        with open(os.path.join(OUT, name + ".json"), "w") as f:
            json.dump(obj, f, indent=0)
            f.write("\n")

    dump("xorshift", xorshift())
    dump("scene_complex", {"scenes": [scene_json(SEEDS[0]), scene_json(SEEDS[3])]})
    cams = {}
    for scene in ("complex", "simple", "three_lambertian", "super_simple"):
        pc, _ = py.scene_builtin(scene, SEEDS[0])
        cams[scene] = camera_json(pc)
    pc, _ = py.scene_builtin("complex", SEEDS[0], 675, 1200, 50)
    cams["complex_1200x675"] = camera_json(pc)
    dump("cameras", cams)
    for fname, scene, seed, h, w, d, s in RENDERS:
        dump(fname, render_json(scene, seed, h, w, d, s))
        print("wrote", fname)


if __name__ == "__main__":
    main()
