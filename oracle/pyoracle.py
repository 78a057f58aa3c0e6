"""TEST INFRASTRUCTURE ONLY -- second, independent CPU restatement of the
reference's sampling path, in pure Python (big-int u128, IEEE f64 floats).

Used only by tests/ and tests/golden/make_golden.py to cross-check the C oracle
(oracle/rtw_oracle.c) bit-for-bit on small cases. Python floats are IEEE
binary64 with correctly rounded + - * / and math.sqrt, and Python never fuses
a*b+c, so evaluating the reference's expressions in the reference's order gives
the reference's bits. Parity status: see oracle/rtw_oracle.h (render values are
parity-unpinned by reference fixtures; none exist).

Citations are to /root/reference/src/... of NicoElbers/Raytracing_in_a_weekend_rust.
"""
from __future__ import annotations

import math

MASK128 = (1 << 128) - 1
INF = float("inf")


# ---------------------------------------------------------------- XorShift --
class XorShift:
    """src/util/random.rs:3-70 (u128 state, shifts drop bits >= 128)."""

    def __init__(self, seed: int):
        self.state = seed & MASK128

    def next_int(self) -> int:  # random.rs:33-38
        s = self.state
        s ^= (s << 23) & MASK128
        s ^= s >> 17
        s ^= (s << 26) & MASK128
        self.state = s
        return s

    def next_01(self) -> float:  # random.rs:40-52
        n = self.next_int() % 0xFFFFFFFF
        return float(n) / 4294967295.0

    def next_bound(self, lo: float, hi: float) -> float:  # random.rs:54-59
        diff = hi - lo
        nxt = self.next_01()
        return lo + diff * nxt

    def copy_reset(self) -> "XorShift":  # random.rs:61-69
        st = self.state
        r = st ^ self.next_int()
        r ^= r >> 13
        r ^= (r << 5) & MASK128
        r ^= r >> 11
        return XorShift(r)


# -------------------------------------------------------------------- vec3 --
# tuples (x, y, z); each helper restates one operator of src/space/vec3.rs
def add(a, b):
    return (a[0] + b[0], a[1] + b[1], a[2] + b[2])


def sub(a, b):
    return (a[0] - b[0], a[1] - b[1], a[2] - b[2])


def neg(a):
    return (-a[0], -a[1], -a[2])


def mul(a, s):  # Vec3 * f64 (vec3.rs:72-82); f64 * Vec3 is vec * self
    return (a[0] * s, a[1] * s, a[2] * s)


def div(a, s):  # vec3.rs:110-120
    return (a[0] / s, a[1] / s, a[2] / s)


def mulv(a, b):  # Color * Color (color.rs:60-70)
    return (a[0] * b[0], a[1] * b[1], a[2] * b[2])


def len_sq(a):  # vec3.rs:150-152
    return a[0] * a[0] + a[1] * a[1] + a[2] * a[2]


def dot(a, b):  # vec3.rs:160-167
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]


def cross(a, b):  # vec3.rs:170-180
    return (a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0])


def unit(a):  # vec3.rs:183-185
    return div(a, math.sqrt(len_sq(a)))


def random_bounded(r: XorShift, lo, hi):  # vec3.rs:207-216
    diff = hi - lo
    x = lo + r.next_01() * diff
    y = lo + r.next_01() * diff
    z = lo + r.next_01() * diff
    return (x, y, z)


def random_in_unit_sphere(r):  # vec3.rs:218-227
    while True:
        p = random_bounded(r, -1.0, 1.0)
        if len_sq(p) <= 1.0:
            return p


def random_unit_vec(r):  # vec3.rs:229-232
    return unit(random_in_unit_sphere(r))


def random_vec_in_unit_disk(r):  # vec3.rs:270-277
    while True:
        x = r.next_bound(-1.0, 1.0)
        y = r.next_bound(-1.0, 1.0)
        v = (x, y, 0.0)
        if len_sq(v) < 1.0:
            return v


def near_zero(a):  # vec3.rs:246-250
    d = 1e-8
    return a[0] < d and a[1] < d and a[2] < d


def reflect(v, n):  # vec3.rs:252-257
    b = mul(n, dot(v, n))
    return sub(v, mul(b, 2.0))


def fmin(a, b):  # Rust f64::min: NaN-ignoring
    if a != a:
        return b
    if b != b:
        return a
    return a if a < b else b


def refract(v, n, ratio):  # vec3.rs:259-268
    cos_theta = fmin(dot(neg(v), n), 1.0)
    out_perp = mul(add(v, mul(n, cos_theta)), ratio)
    out_par = mul(n, -math.sqrt(abs(1.0 - len_sq(out_perp))))
    return add(out_perp, out_par)


def contains_inc(lo, hi, x):  # interval.rs:55-57
    return lo <= x <= hi


def contains_ex(lo, hi, x):  # interval.rs:60-62
    return lo < x < hi


# ------------------------------------------------------------------ camera --
RADS_PER_DEG = math.pi / 180.0


class Camera:
    """camera.rs:138-221 (argument order: height first)."""

    def __init__(self, h, w, max_depth, focal_length, fov, look_from, look_to, vup,
                 defocus_angle, focus_dist):
        theta = fov * RADS_PER_DEG
        hh = math.tan(theta / 2.0)
        self.viewport_height = 2.0 * hh * focus_dist
        self.viewport_width = self.viewport_height * (float(w) / float(h))
        self.w = unit(sub(look_from, look_to))
        self.u = unit(cross(vup, self.w))
        self.v = cross(self.w, self.u)
        viewport_u = mul(self.u, self.viewport_width)
        viewport_v = mul(neg(self.v), self.viewport_height)
        self.pixel_delta_u = div(viewport_u, float(w))
        self.pixel_delta_v = div(viewport_v, float(h))
        self.pixel00 = sub(sub(sub(look_from, mul(self.w, focus_dist)), div(viewport_u, 2.0)),
                           div(viewport_v, 2.0))
        r = focus_dist * math.tan((defocus_angle / 2.0) * RADS_PER_DEG)
        self.defocus_disk_u = mul(self.u, r)
        self.defocus_disk_v = mul(self.v, r)
        self.height, self.width, self.max_depth = h, w, max_depth
        self.look_from, self.look_to, self.vup = look_from, look_to, vup
        self.defocus_angle, self.focus_dist = defocus_angle, focus_dist
        self.focal_length, self.fov = focal_length, fov


def offset_lattice(dx, dy, s):  # camera.rs:422-450
    if s == 0:
        return [add(div(dx, 2.0), div(dy, 2.0))]
    sf = float(s)
    dx = div(dx, sf)
    dy = div(dy, sf)
    pos0 = add(div(dx, 2.0), div(dy, 2.0))
    out = []
    for y in range(s):
        pos = add(pos0, mul(dy, float(y)))
        for x in range(s):
            out.append(add(pos, mul(dx, float(x))))
    return out


# -------------------------------------------------------------------- scene --
LAMBERTIAN, METAL, DIELECTRIC = 0, 1, 2


def scene_complex(seed: int):
    """raytracing/mod.rs:62-103 with an explicit seed. Returns a list of
    (center, radius, (kind, albedo, fuzz, ir)) in insertion order."""
    objs = [((0.0, -1000.0, 0.0), 1000.0, (LAMBERTIAN, (0.5, 0.5, 0.5), 0.0, 0.0))]
    rnd = XorShift(seed)
    for a in range(-11, 11):
        for b in range(-11, 11):
            choose = rnd.next_01()
            cx = float(a) + 0.9 * rnd.next_01()
            cz = float(b) + 0.9 * rnd.next_01()
            center = (cx, 0.2, cz)
            if math.sqrt(len_sq(sub(center, (4.0, 0.2, 0.0)))) > 0.9:
                if choose < 0.34:
                    c1 = (rnd.next_01(), rnd.next_01(), rnd.next_01())
                    c2 = (rnd.next_01(), rnd.next_01(), rnd.next_01())
                    m = (LAMBERTIAN, mulv(c1, c2), 0.0, 0.0)
                elif choose < 0.67:
                    c1 = (rnd.next_01(), rnd.next_01(), rnd.next_01())
                    c2 = (rnd.next_01(), rnd.next_01(), rnd.next_01())
                    fuzz = rnd.next_bound(0.0, 1.0)
                    m = (METAL, mulv(c1, c2), fuzz, 0.0)
                else:
                    m = (DIELECTRIC, (0.0, 0.0, 0.0), 0.0, 1.5)
                objs.append((center, 0.2, m))
    objs.append(((0.0, 1.0, 0.0), 1.0, (DIELECTRIC, (0.0, 0.0, 0.0), 0.0, 1.5)))
    objs.append(((-4.0, 1.0, 0.0), 1.0, (LAMBERTIAN, (0.4, 0.2, 0.1), 0.0, 0.0)))
    objs.append(((4.0, 1.0, 0.0), 1.0, (METAL, (0.7, 0.6, 0.5), 0.0, 0.0)))
    return objs


# ------------------------------------------------------------------- render --
def sphere_hit(center, radius, orig, d):  # sphere.rs:39-71 + hittable.rs:27-37, 64-81
    oc = sub(orig, center)
    a = len_sq(d)
    half_b = dot(oc, d)
    c = len_sq(oc) - radius * radius
    disc = half_b * half_b - (a * c)
    if disc < 0.0:
        return None
    sq = math.sqrt(disc)
    root = None
    for x in (-sq, sq):
        t = (x - half_b) / a
        if contains_inc(0.01, INF, t):
            root = t
            break
    if root is None:
        return None
    p = add(mul(d, root), orig)
    outward = div(sub(p, center), radius)
    front = dot(d, outward) < 0.0
    return (root, p, outward if front else neg(outward), front)


def scene_hit(objs, orig, d):  # hittable.rs:131-143, first minimum wins
    best = None
    for obj in objs:
        h = sphere_hit(obj[0], obj[1], orig, d)
        if h is not None and (best is None or h[0] < best[0][0]):
            best = (h, obj[2])
    return best


def reflectance(ir, cos):  # materials.rs:75-80, powi(5) = x * ((x*x) * (x*x))
    r0 = (1.0 - ir) / (1.0 + ir)
    r0 = r0 * r0
    x = 1.0 - cos
    return r0 + (1.0 - r0) * (x * ((x * x) * (x * x)))


def scatter(m, d, rec, rnd):  # materials.rs:22-37, 52-63, 83-111
    kind, albedo, fuzz, ir = m
    _, p, normal, front = rec
    if kind == LAMBERTIAN:
        sd = add(normal, random_unit_vec(rnd))
        if near_zero(sd):
            sd = normal
        return p, sd, albedo
    if kind == METAL:
        refl = reflect(unit(d), normal)
        return p, add(refl, mul(random_unit_vec(rnd), fuzz)), albedo
    ratio = 1.0 / ir if front else ir
    ud = unit(d)
    cos_t = fmin(dot(neg(ud), normal), 1.0)
    sin_t = math.sqrt(1.0 - cos_t * cos_t)
    cant = ratio * sin_t > 1.0
    if cant or reflectance(ir, cos_t) > rnd.next_01():
        nd = reflect(ud, normal)
    else:
        nd = refract(ud, normal, ratio)
    return p, nd, (1.0, 1.0, 1.0)


def ray_color(cam, objs, orig, d, rnd, depth, stats):  # camera.rs:376-398
    if depth >= cam.max_depth:
        return (0.0, 0.0, 0.0)
    stats[0] += 1
    hit = scene_hit(objs, orig, d)
    if hit is not None:
        rec, m = hit
        o2, d2, att = scatter(m, d, rec, rnd)
        return mulv(att, ray_color(cam, objs, o2, d2, rnd, depth + 1, stats))
    ud = unit(d)
    a = 0.5 * (ud[1] + 1.0)
    return add(mul((1.0, 1.0, 1.0), 1.0 - a), mul((0.5, 0.7, 1.0), a))


def get_ray(cam, i, j, offset, rnd):  # camera.rs:400-420, 452-456
    loc = add(add(cam.pixel00, mul(cam.pixel_delta_u, float(i))), mul(cam.pixel_delta_v, float(j)))
    sample = add(loc, offset)
    if cam.defocus_angle <= 0.0:
        origin = cam.look_from
    else:
        p = random_vec_in_unit_disk(rnd)
        origin = add(add(cam.look_from, mul(cam.defocus_disk_u, p[0])), mul(cam.defocus_disk_v, p[1]))
    return origin, sub(sample, origin)


def render(cam, objs, samples_sqrt, seed, rows=None):
    """camera.rs:223-374 without the thread pool: returns {(x, y): (r, g, b)} for
    the requested rows (default: all) and the traced-segment count."""
    offsets = offset_lattice(cam.pixel_delta_v, cam.pixel_delta_u, samples_sqrt)
    rows = set(range(cam.height)) if rows is None else set(rows)
    parent = XorShift(seed)
    out = {}
    stats = [0]
    for y in range(max(rows) + 1):
        for x in range(cam.width):
            rnd = parent.copy_reset()
            if y not in rows:
                continue
            acc = (0.0, 0.0, 0.0)
            for off in offsets:
                o, d = get_ray(cam, x, y, off, rnd)
                acc = add(acc, ray_color(cam, objs, o, d, rnd, 0, stats))
            out[(x, y)] = div(acc, float(len(offsets)))
    return out, stats[0]


def cpow(x, y):
    """libm pow (Rust f64::powf): NaN for a negative base with a fractional exponent."""
    try:
        return math.pow(x, y)
    except ValueError:
        return math.nan


def format_ppm(img, w, h) -> str:  # color.rs:196-247
    def sat(v):
        if not (v > 0.0):
            return 0
        if v >= 18446744073709551616.0:
            return (1 << 64) - 1
        return int(v)

    lines = [f"P3\n{w} {h}\n255\n"]
    for y in range(h):
        vals = []
        for x in range(w):
            for c in img[(x, y)]:
                vals.append(str(sat(cpow(c, 1.0 / 2.2) * 255.0)))
        if vals:
            lines.append(" ".join(vals) + "\n")
    return "".join(lines)


# ----------------------------------------------------------- scene presets --
def scene_builtin(name: str, seed: int, h=0, w=0, max_depth=0):
    """raytracing/mod.rs builders (+ BASELINE config 1 'three_lambertian').
    Returns (Camera, objs). Zero h/w/max_depth take the builder's own values."""
    def pick(v, d):
        return v if v else d

    L = LAMBERTIAN
    if name == "complex":  # mod.rs:54-126, Config defaults 1080x1920 (main.rs:20-29)
        cam = Camera(pick(h, 1080), pick(w, 1920), pick(max_depth, 10), 1.0, 20.0,
                     (13.0, 2.0, 3.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 0.6, 10.0)
        return cam, scene_complex(seed)
    if name in ("simple", "three_lambertian"):  # mod.rs:129-173
        three = name == "three_lambertian"
        cam = Camera(pick(h, 225 if three else 1080), pick(w, 400 if three else 1920),
                     pick(max_depth, 8 if three else 25), 1.0, 20.0, (-2.0, 2.0, 1.0),
                     (0.0, 0.0, -1.0), (0.0, 1.0, 0.0), 10.0, 3.4)
        objs = [((0.0, -100.5, -1.0), 100.0, (L, (0.8, 0.8, 0.0), 0.0, 0.0)),
                ((0.0, 0.0, -1.0), 0.5, (L, (0.1, 0.2, 0.5), 0.0, 0.0))]
        if three:
            objs.append(((1.0, 0.0, -1.0), 0.5, (L, (0.8, 0.6, 0.2), 0.0, 0.0)))
        else:
            objs.append(((-1.0, 0.0, -1.0), 0.5, (DIELECTRIC, (0.0, 0.0, 0.0), 0.0, 1.5)))
            objs.append(((1.0, 0.0, -1.0), 0.5, (METAL, (0.8, 0.6, 0.2), 0.0, 0.0)))
        return cam, objs
    if name in ("threads", "super_simple"):  # mod.rs:176-238
        cam = Camera(pick(h, 1000), pick(w, 1000), pick(max_depth, 50), 1.0, 50.0,
                     (0.0, 0.0, 0.0), (0.0, 0.0, -0.3), (0.0, 1.0, 0.0), 0.6, 10.0)
        return cam, [((0.0, -100.5, -1.0), 100.0, (L, (0.8, 0.8, 0.0), 0.0, 0.0))]
    raise ValueError(name)
