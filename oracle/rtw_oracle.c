/*
 * rtw_oracle.c -- TEST INFRASTRUCTURE ONLY. CPU restatement of the reference's
 * per-pixel sampling path, used as the parity checker (tests/, smoke()) and as
 * the CPU baseline (bench.py cpu_baseline, kind "port"). See rtw_oracle.h for
 * the parity status ("render values parity-unpinned by reference fixtures").
 *
 * Build: gcc -O2 -ffp-contract=off -fno-fast-math (oracle/Makefile). No FMA
 * contraction, generic x86-64 -- matching the reference's default release
 * profile (Cargo.toml:8-13), which never contracts a*b+c.
 *
 * All arithmetic is f64 in the reference's exact operation order. Reference
 * paths are relative to the reference repo root (src/...).
 */
#include "rtw_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

typedef unsigned __int128 u128;
typedef orc_vec3 V3;

static inline u128 mk128(uint64_t lo, uint64_t hi) { return ((u128)hi << 64) | lo; }

/* ---------------------------------------------------------------- vec3 --- */
/* src/space/vec3.rs:28-120 (Add/Sub/Neg/Mul<f64>/Div<f64>), 150-185 (len, dot,
 * cross, unit). `f64 * Vec3` is defined as `vec * self` (vec3.rs:84-90) and
 * f64 multiplication commutes bitwise, so one helper serves both. */
static inline V3 v3(double x, double y, double z) { V3 r = {x, y, z}; return r; }
static inline V3 vadd(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline V3 vsub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline V3 vneg(V3 a) { return v3(-a.x, -a.y, -a.z); }
static inline V3 vmul(V3 a, double s) { return v3(a.x * s, a.y * s, a.z * s); }
static inline V3 vdiv(V3 a, double s) { return v3(a.x / s, a.y / s, a.z / s); }
static inline V3 vmulv(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); } /* color.rs:60-70 */
static inline double len_sq(V3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }   /* vec3.rs:150-152 */
static inline double vdot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; } /* vec3.rs:160-167 */
static inline V3 vcross(V3 a, V3 b) {                                             /* vec3.rs:170-180 */
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline V3 vunit(V3 a) { return vdiv(a, sqrt(len_sq(a))); } /* vec3.rs:154-157, 183-185 */
static inline V3 ld3(const double *p) { return v3(p[0], p[1], p[2]); }

/* ------------------------------------------------------------- XorShift --- */
/* src/util/random.rs:33-38 */
static inline u128 xs_next_int(u128 *s) {
    *s ^= *s << 23;
    *s ^= *s >> 17;
    *s ^= *s << 26;
    return *s;
}
/* random.rs:40-52: (next % u32::MAX) as u32 as f64 / u32::MAX as f64 */
static inline double xs_next_01(u128 *s) {
    u128 n = xs_next_int(s);
    uint32_t b = (uint32_t)(n % (u128)0xFFFFFFFFu);
    return (double)b / 4294967295.0;
}
/* random.rs:54-59 */
static inline double xs_next_bound(u128 *s, double min, double max) {
    double diff = max - min;
    double next = xs_next_01(s);
    return min + diff * next;
}
/* random.rs:61-69: child = mix(parent ^ parent.next_int()) */
static inline u128 xs_copy_reset(u128 *s) {
    u128 self_state = *s;
    u128 r = self_state ^ xs_next_int(s);
    r ^= r >> 13;
    r ^= r << 5;
    r ^= r >> 11;
    return r;
}

void orc_xs_next_int(uint64_t lo, uint64_t hi, uint32_t n, uint64_t *out) {
    u128 s = mk128(lo, hi);
    for (uint32_t i = 0; i < n; ++i) {
        u128 v = xs_next_int(&s);
        out[2 * i] = (uint64_t)v;
        out[2 * i + 1] = (uint64_t)(v >> 64);
    }
}
void orc_xs_next_01(uint64_t lo, uint64_t hi, uint32_t n, double *out) {
    u128 s = mk128(lo, hi);
    for (uint32_t i = 0; i < n; ++i) out[i] = xs_next_01(&s);
}
void orc_xs_copy_reset_chain(uint64_t lo, uint64_t hi, uint64_t n, uint64_t *out) {
    u128 s = mk128(lo, hi);
    for (uint64_t i = 0; i < n; ++i) {
        u128 c = xs_copy_reset(&s);
        out[2 * i] = (uint64_t)c;
        out[2 * i + 1] = (uint64_t)(c >> 64);
    }
}

/* color.rs:249-255 Color::random: r, g, b in field order */
static inline V3 random_color(u128 *s) {
    double r = xs_next_01(s);
    double g = xs_next_01(s);
    double b = xs_next_01(s);
    return v3(r, g, b);
}

/* vec3.rs:207-216 random_bounded: min + next_01 * diff, fields x,y,z in order */
static inline V3 random_bounded(u128 *s, double min, double max) {
    double diff = max - min;
    double x = min + xs_next_01(s) * diff;
    double y = min + xs_next_01(s) * diff;
    double z = min + xs_next_01(s) * diff;
    return v3(x, y, z);
}
/* vec3.rs:218-227: rejection with inclusive len^2 <= 1 */
static inline V3 random_in_unit_sphere(u128 *s) {
    for (;;) {
        V3 p = random_bounded(s, -1., 1.);
        if (len_sq(p) <= 1.) return p;
    }
}
/* vec3.rs:229-232 */
static inline V3 random_unit_vec(u128 *s) { return vunit(random_in_unit_sphere(s)); }
/* vec3.rs:270-277: rejection with strict len^2 < 1 */
static inline V3 random_vec_in_unit_disk(u128 *s) {
    for (;;) {
        double x = xs_next_bound(s, -1., 1.);
        double y = xs_next_bound(s, -1., 1.);
        V3 v = v3(x, y, 0.);
        if (len_sq(v) < 1.) return v;
    }
}
/* vec3.rs:246-250 (no abs: reference quirk) */
static inline int near_zero(V3 a) {
    const double d = 1e-8;
    return (a.x < d) && (a.y < d) && (a.z < d);
}
/* vec3.rs:252-257 */
static inline V3 reflect(V3 v, V3 n) {
    V3 b = vmul(n, vdot(v, n));
    return vsub(v, vmul(b, 2.));
}
/* vec3.rs:259-268 */
static inline V3 refract(V3 self, V3 n, double ratio) {
    double cos_theta = fmin(vdot(vneg(self), n), 1.);
    V3 out_perp = vmul(vadd(self, vmul(n, cos_theta)), ratio);
    V3 out_par = vmul(n, -sqrt(fabs(1. - len_sq(out_perp))));
    return vadd(out_perp, out_par);
}

/* ------------------------------------------------------------- Interval --- */
/* interval.rs:55-62 */
int orc_interval_contains_inc(double min, double max, double x) { return min <= x && x <= max; }
int orc_interval_contains_ex(double min, double max, double x) { return min < x && x < max; }

/* --------------------------------------------------------------- Camera --- */
/* Rust f64::to_radians = self * (PI / 180.0) */
static inline double to_radians(double d) { return d * (M_PI / 180.0); }

/* camera.rs:138-221 */
void orc_camera_new(uint32_t h, uint32_t w, uint32_t max_depth, double focal_length,
                    double fov, const double from[3], const double to[3], const double vup_[3],
                    double defocus_angle, double focus_dist, orc_camera *c) {
    memset(c, 0, sizeof *c);
    double theta = to_radians(fov);
    double hh = tan(theta / 2.);
    double viewport_height = 2. * hh * focus_dist;
    double viewport_width = viewport_height * ((double)w / (double)h);
    V3 look_from = ld3(from), look_to = ld3(to), vup = ld3(vup_);
    V3 W = vunit(vsub(look_from, look_to));
    V3 U = vunit(vcross(vup, W));
    V3 Vv = vcross(W, U);
    V3 viewport_u = vmul(U, viewport_width);
    V3 viewport_v = vmul(vneg(Vv), viewport_height);
    V3 pdu = vdiv(viewport_u, (double)w);
    V3 pdv = vdiv(viewport_v, (double)h);
    V3 p00 = vsub(vsub(vsub(look_from, vmul(W, focus_dist)), vdiv(viewport_u, 2.)),
                  vdiv(viewport_v, 2.));
    double defocus_radius = focus_dist * tan(to_radians(defocus_angle / 2.));
    c->img_height = h;
    c->img_width = w;
    c->max_depth = max_depth;
    c->focal_length = focal_length;
    c->fov = fov;
    c->look_from = look_from;
    c->look_to = look_to;
    c->vup = vup;
    c->u = U;
    c->v = Vv;
    c->w = W;
    c->viewport_height = viewport_height;
    c->viewport_width = viewport_width;
    c->pixel00 = p00;
    c->pixel_delta_u = pdu;
    c->pixel_delta_v = pdv;
    c->defocus_angle = defocus_angle;
    c->focus_dist = focus_dist;
    c->defocus_disk_u = vmul(U, defocus_radius);
    c->defocus_disk_v = vmul(Vv, defocus_radius);
}

/* camera.rs:422-450 */
uint32_t orc_offset_lattice(const double dx_[3], const double dy_[3], uint32_t s, double *out) {
    V3 dx = ld3(dx_), dy = ld3(dy_);
    if (s == 0) {
        V3 p = vadd(vdiv(dx, 2.), vdiv(dy, 2.));
        if (out) { out[0] = p.x; out[1] = p.y; out[2] = p.z; }
        return 1;
    }
    double sf = (double)s;
    dx = vdiv(dx, sf);
    dy = vdiv(dy, sf);
    V3 pos0 = vadd(vdiv(dx, 2.), vdiv(dy, 2.));
    uint32_t k = 0;
    for (uint32_t y = 0; y < s; ++y) {
        V3 pos = vadd(pos0, vmul(dy, (double)y));
        for (uint32_t x = 0; x < s; ++x, ++k) {
            V3 p = vadd(pos, vmul(dx, (double)x));
            if (out) { out[3 * k] = p.x; out[3 * k + 1] = p.y; out[3 * k + 2] = p.z; }
        }
    }
    return k;
}

/* ---------------------------------------------------------------- Scene --- */
/* raytracing/mod.rs:62-103, XorShift seeded explicitly instead of wall-clock
 * (mod.rs:67 -> random.rs:16-22; XorShift::new, random.rs:29-31). */
uint32_t orc_scene_complex(uint64_t lo, uint64_t hi, orc_sphere *sph, orc_material *mat,
                           uint32_t cap) {
    uint32_t n = 0;
#define ADD(cx, cy, cz, r, K, ar, ag, ab, fz, irr)                                   \
    do {                                                                             \
        if (n < cap) {                                                               \
            orc_sphere *S = &sph[n];                                                 \
            orc_material *M = &mat[n];                                               \
            memset(S, 0, sizeof *S);                                                 \
            memset(M, 0, sizeof *M);                                                 \
            S->center[0] = (cx); S->center[1] = (cy); S->center[2] = (cz);           \
            S->radius = (r); S->mat = n;                                             \
            M->kind = (K); M->albedo[0] = (ar); M->albedo[1] = (ag);                 \
            M->albedo[2] = (ab); M->fuzz = (fz); M->ir = (irr);                      \
        }                                                                            \
        ++n;                                                                         \
    } while (0)
    ADD(0., -1000., 0., 1000., ORC_LAMBERTIAN, 0.5, 0.5, 0.5, 0., 0.);
    u128 s = mk128(lo, hi);
    for (int a = -11; a < 11; ++a) {
        for (int b = -11; b < 11; ++b) {
            double choose_mat = xs_next_01(&s);
            double cx = (double)a + 0.9 * xs_next_01(&s);
            double cy = 0.2;
            double cz = (double)b + 0.9 * xs_next_01(&s);
            V3 pv = vsub(v3(cx, cy, cz), v3(4., 0.2, 0.));
            if (sqrt(len_sq(pv)) > 0.9) {
                if (choose_mat < 0.34) {
                    V3 c1 = random_color(&s);
                    V3 c2 = random_color(&s);
                    V3 al = vmulv(c1, c2);
                    ADD(cx, cy, cz, 0.2, ORC_LAMBERTIAN, al.x, al.y, al.z, 0., 0.);
                } else if (choose_mat < 0.67) {
                    V3 c1 = random_color(&s);
                    V3 c2 = random_color(&s);
                    V3 al = vmulv(c1, c2);
                    double fuzz = xs_next_bound(&s, 0., 1.);
                    ADD(cx, cy, cz, 0.2, ORC_METAL, al.x, al.y, al.z, fuzz, 0.);
                } else {
                    ADD(cx, cy, cz, 0.2, ORC_DIELECTRIC, 0., 0., 0., 0., 1.5);
                }
            }
        }
    }
    ADD(0., 1., 0., 1., ORC_DIELECTRIC, 0., 0., 0., 0., 1.5);
    ADD(-4., 1., 0., 1., ORC_LAMBERTIAN, 0.4, 0.2, 0.1, 0., 0.);
    ADD(4., 1., 0., 1., ORC_METAL, 0.7, 0.6, 0.5, 0.0, 0.);
#undef ADD
    return n;
}

/* --------------------------------------------------------------- Render --- */
typedef struct { V3 orig, dir; } Ray; /* ray.rs:6-42 */

struct Obj;
struct Mat;
typedef struct {                       /* hittable.rs:16-23 */
    V3 point, normal;
    const struct Mat *mat;
    double t;
    int front;
} HitRec;

/* dyn Material stand-in (materials.rs:7-9); rc mimics Arc<dyn Material> clones. */
typedef int (*scatter_fn)(const struct Mat *, const Ray *, const HitRec *, u128 *, Ray *, V3 *);
typedef struct Mat {
    scatter_fn scatter;
    V3 albedo;
    double fuzz, ir;
    _Atomic long rc;
    char _pad[64]; /* keep refcounts of different materials on different lines */
} Mat;

/* dyn Hittable stand-in (hittable.rs:12-14) */
typedef int (*hit_fn)(const struct Obj *, const Ray *, double, double, HitRec *);
typedef struct Obj {
    hit_fn hit;
    V3 center;
    double radius;
    Mat *mat;
} Obj;

/* sphere.rs:39-71 + HitRecord::new / face_normal hittable.rs:27-37, 64-81 */
static inline int sphere_hit(V3 center, double radius, const Ray *r, double tmin, double tmax,
                             HitRec *rec) {
    V3 oc = vsub(r->orig, center);
    double a = len_sq(r->dir);
    double half_b = vdot(oc, r->dir);
    double c = len_sq(oc) - radius * radius;
    double d = half_b * half_b - (a * c); /* powi(2) == one multiply */
    if (d < 0.0) return 0;
    double sqrtd = sqrt(d);
    double root = (-sqrtd - half_b) / a;
    if (!(tmin <= root && root <= tmax)) { /* Interval::contains_inc, near root first */
        root = (sqrtd - half_b) / a;
        if (!(tmin <= root && root <= tmax)) return 0;
    }
    V3 point = vadd(vmul(r->dir, root), r->orig); /* Ray::at, ray.rs:28-31 */
    V3 outward = vdiv(vsub(point, center), radius);
    int front = vdot(r->dir, outward) < 0.0;
    rec->point = point;
    rec->normal = front ? outward : vneg(outward);
    rec->t = root;
    rec->front = front;
    return 1;
}

static int obj_sphere_hit(const Obj *o, const Ray *r, double tmin, double tmax, HitRec *rec) {
    if (!sphere_hit(o->center, o->radius, r, tmin, tmax, rec)) return 0;
    rec->mat = o->mat;
    atomic_fetch_add_explicit(&o->mat->rc, 1, memory_order_relaxed); /* self.mat.clone() */
    return 1;
}
static inline void rec_drop(const HitRec *rec) {
    atomic_fetch_sub_explicit(&((Mat *)rec->mat)->rc, 1, memory_order_release);
}

/* materials.rs:22-37 */
static int scatter_lambertian(const Mat *m, const Ray *r, const HitRec *rec, u128 *rng, Ray *out,
                              V3 *att) {
    (void)r;
    V3 sd = vadd(rec->normal, random_unit_vec(rng));
    if (near_zero(sd)) sd = rec->normal;
    out->orig = rec->point;
    out->dir = sd;
    *att = m->albedo;
    return 1;
}
/* materials.rs:52-63 */
static int scatter_metal(const Mat *m, const Ray *r, const HitRec *rec, u128 *rng, Ray *out,
                         V3 *att) {
    V3 reflected = reflect(vunit(r->dir), rec->normal);
    V3 ru = random_unit_vec(rng);
    out->orig = rec->point;
    out->dir = vadd(reflected, vmul(ru, m->fuzz));
    *att = m->albedo;
    return 1;
}
/* materials.rs:75-80, powi(5) lowers to x * ((x*x) * (x*x)) */
static inline double reflectance(double ir, double cos) {
    double r0 = (1. - ir) / (1. + ir);
    r0 = r0 * r0;
    double x = 1. - cos;
    return r0 + (1. - r0) * (x * ((x * x) * (x * x)));
}
/* materials.rs:83-111 (RNG drawn only when refraction is possible: `||` short-circuit) */
static int scatter_dielectric(const Mat *m, const Ray *r, const HitRec *rec, u128 *rng, Ray *out,
                              V3 *att) {
    double ratio = rec->front ? 1. / m->ir : m->ir;
    V3 ud = vunit(r->dir);
    double cos_theta = fmin(vdot(vneg(ud), rec->normal), 1.);
    double sin_theta = sqrt(1.0 - cos_theta * cos_theta);
    int cant = ratio * sin_theta > 1.;
    V3 dir;
    if (cant || reflectance(m->ir, cos_theta) > xs_next_01(rng))
        dir = reflect(ud, rec->normal);
    else
        dir = refract(ud, rec->normal, ratio);
    out->orig = rec->point;
    out->dir = dir;
    *att = v3(1., 1., 1.);
    return 1;
}

typedef struct {
    const orc_camera *cam;
    Obj *objs;
    uint32_t n_obj;
    uint32_t n_off;
    V3 *offsets;
    const u128 *children; /* per rendered pixel */
    const uint32_t *rows; /* image row of each rendered row, ascending */
    uint32_t n_rows, W;
    int faithful;
    double *out;
    _Atomic uint64_t *row_segments; /* per rendered row (nullable) */
    _Atomic uint64_t next_job;
    _Atomic uint64_t segments;
} Ctx;

/* Scene::hit hittable.rs:131-143: all objects, first minimum wins (min_by keeps
 * the earlier element unless the later one compares Less). */
static int scene_hit(const Ctx *c, const Ray *r, HitRec *best) {
    int found = 0;
    HitRec cand;
    for (uint32_t i = 0; i < c->n_obj; ++i) {
        const Obj *o = &c->objs[i];
        if (c->faithful) {
            if (!o->hit(o, r, 0.01, INFINITY, &cand)) continue;
            if (!found || cand.t < best->t) {
                if (found) rec_drop(best);
                *best = cand;
                found = 1;
            } else {
                rec_drop(&cand);
            }
        } else {
            if (!sphere_hit(o->center, o->radius, r, 0.01, INFINITY, &cand)) continue;
            if (!found || cand.t < best->t) {
                cand.mat = o->mat;
                *best = cand;
                found = 1;
            }
        }
    }
    return found;
}

static int mat_scatter(const Ctx *c, const Mat *m, const Ray *r, const HitRec *rec, u128 *rng,
                       Ray *out, V3 *att) {
    if (c->faithful) return m->scatter(m, r, rec, rng, out, att);
    if (m->scatter == scatter_lambertian) return scatter_lambertian(m, r, rec, rng, out, att);
    if (m->scatter == scatter_metal) return scatter_metal(m, r, rec, rng, out, att);
    return scatter_dielectric(m, r, rec, rng, out, att);
}

/* camera.rs:376-398 (recursive, exactly as the reference associates the product) */
static V3 ray_color(const Ctx *c, Ray r, u128 *rng, uint32_t depth, uint64_t *seg) {
    if (depth >= c->cam->max_depth) return v3(0., 0., 0.);
    HitRec rec;
    ++*seg;
    if (scene_hit(c, &r, &rec)) {
        Ray sc;
        V3 att;
        const Mat *m = rec.mat;
        if (c->faithful) atomic_fetch_add_explicit(&((Mat *)m)->rc, 1, memory_order_relaxed);
        int ok = mat_scatter(c, m, &r, &rec, rng, &sc, &att);
        if (c->faithful) { rec_drop(&rec); atomic_fetch_sub_explicit(&((Mat *)m)->rc, 1, memory_order_release); }
        if (ok) return vmulv(att, ray_color(c, sc, rng, depth + 1, seg));
        return v3(0., 0., 0.);
    }
    V3 ud = vunit(r.dir);
    double a = 0.5 * (ud.y + 1.0);
    return vadd(vmul(v3(1.0, 1.0, 1.0), 1.0 - a), vmul(v3(0.5, 0.7, 1.0), a));
}

/* camera.rs:452-456 */
static inline V3 defocus_disk_sample(const orc_camera *cam, u128 *rng) {
    V3 p = random_vec_in_unit_disk(rng);
    return vadd(vadd(cam->look_from, vmul(cam->defocus_disk_u, p.x)), vmul(cam->defocus_disk_v, p.y));
}

/* camera.rs:400-420 */
static inline Ray get_ray(const orc_camera *cam, uint32_t i, uint32_t j, V3 offset, u128 *rng) {
    V3 pixel_loc = vadd(vadd(cam->pixel00, vmul(cam->pixel_delta_u, (double)i)),
                        vmul(cam->pixel_delta_v, (double)j));
    V3 pixel_sample = vadd(pixel_loc, offset);
    V3 origin = cam->defocus_angle <= 0. ? cam->look_from : defocus_disk_sample(cam, rng);
    Ray r = {origin, vsub(pixel_sample, origin)};
    return r;
}

/* camera.rs:354-374 */
static void render_pixel(Ctx *c, uint64_t local_idx) {
    uint32_t lr = (uint32_t)(local_idx / c->W), x = (uint32_t)(local_idx % c->W);
    uint32_t y = c->rows[lr];
    u128 rng = c->children[local_idx];
    uint64_t seg = 0;
    V3 acc = v3(0., 0., 0.);
    for (uint32_t k = 0; k < c->n_off; ++k) {
        Ray r = get_ray(c->cam, x, y, c->offsets[k], &rng);
        acc = vadd(acc, ray_color(c, r, &rng, 0, &seg));
    }
    V3 col = vdiv(acc, (double)c->n_off);
    double *o = c->out + 3 * local_idx;
    o[0] = col.x;
    o[1] = col.y;
    o[2] = col.z;
    atomic_fetch_add_explicit(&c->segments, seg, memory_order_relaxed);
    if (c->row_segments) atomic_fetch_add_explicit(&c->row_segments[lr], seg, memory_order_relaxed);
}

static void *worker(void *arg) {
    Ctx *c = (Ctx *)arg;
    uint64_t npx = (uint64_t)c->n_rows * c->W;
    if (c->faithful) { /* one job per pixel (camera.rs:269-292) */
        for (;;) {
            uint64_t j = atomic_fetch_add_explicit(&c->next_job, 1, memory_order_relaxed);
            if (j >= npx) break;
            render_pixel(c, j);
        }
    } else { /* one job per row */
        for (;;) {
            uint64_t row = atomic_fetch_add_explicit(&c->next_job, 1, memory_order_relaxed);
            if (row >= c->n_rows) break;
            for (uint64_t x = 0; x < c->W; ++x) render_pixel(c, row * c->W + x);
        }
    }
    return NULL;
}

static int render_rows(const orc_camera *cam, const orc_sphere *sph, uint32_t n_sph,
                       const orc_material *mat, uint32_t n_mat, uint32_t samples_sqrt,
                       uint64_t seed_lo, uint64_t seed_hi, const uint32_t *rows,
                       uint32_t n_rows, uint32_t nthreads, int scheduler, double *out,
                       uint64_t *segments, uint64_t *row_segments) {
    uint32_t W = cam->img_width, H = cam->img_height;
    if (W == 0 || H == 0) return -1; /* camera.rs:267 */
    if (n_rows == 0) return 0;
    for (uint32_t k = 0; k < n_rows; ++k)
        if (rows[k] >= H || (k && rows[k] <= rows[k - 1])) return -2;
    for (uint32_t i = 0; i < n_sph; ++i)
        if (sph[i].mat >= n_mat) return -3;
    for (uint32_t i = 0; i < n_mat; ++i)
        if (mat[i].kind == ORC_METAL && !(mat[i].fuzz <= 1.)) return -4; /* materials.rs:47 */
    if (nthreads == 0) nthreads = 1;

    Ctx c;
    memset(&c, 0, sizeof c);
    c.cam = cam;
    c.W = W;
    c.rows = rows;
    c.n_rows = n_rows;
    if (row_segments) {
        memset(row_segments, 0, sizeof(uint64_t) * n_rows);
        c.row_segments = (_Atomic uint64_t *)row_segments;
    }
    c.faithful = scheduler == 0;
    c.out = out;

    /* offsets: called as offset_lattice(&pixel_delta_v, &pixel_delta_u, s) (camera.rs:243-244) */
    const double dv[3] = {cam->pixel_delta_v.x, cam->pixel_delta_v.y, cam->pixel_delta_v.z};
    const double du[3] = {cam->pixel_delta_u.x, cam->pixel_delta_u.y, cam->pixel_delta_u.z};
    c.n_off = orc_offset_lattice(dv, du, samples_sqrt, NULL);
    c.offsets = (V3 *)malloc(sizeof(V3) * c.n_off);
    orc_offset_lattice(dv, du, samples_sqrt, (double *)c.offsets);

    Mat *mats = (Mat *)aligned_alloc(64, sizeof(Mat) * (n_mat ? n_mat : 1));
    for (uint32_t i = 0; i < n_mat; ++i) {
        memset(&mats[i], 0, sizeof(Mat));
        mats[i].scatter = mat[i].kind == ORC_LAMBERTIAN ? scatter_lambertian
                          : mat[i].kind == ORC_METAL    ? scatter_metal
                                                        : scatter_dielectric;
        mats[i].albedo = ld3(mat[i].albedo);
        mats[i].fuzz = mat[i].fuzz;
        mats[i].ir = mat[i].ir;
        atomic_init(&mats[i].rc, 1);
    }
    c.objs = (Obj *)malloc(sizeof(Obj) * (n_sph ? n_sph : 1));
    for (uint32_t i = 0; i < n_sph; ++i) {
        c.objs[i].hit = obj_sphere_hit;
        c.objs[i].center = ld3(sph[i].center);
        c.objs[i].radius = sph[i].radius;
        c.objs[i].mat = &mats[sph[i].mat];
    }
    c.n_obj = n_sph;

    /* per-pixel children: copy_reset once per pixel in row-major order over the
     * whole image (camera.rs:255, 269-272), kept for the rendered rows only */
    u128 *children = (u128 *)malloc(sizeof(u128) * (uint64_t)n_rows * W);
    u128 parent = mk128(seed_lo, seed_hi);
    uint32_t last_row = rows[n_rows - 1];
    uint32_t next_lr = 0;
    for (uint32_t y = 0; y <= last_row; ++y) {
        int keep = next_lr < n_rows && y == rows[next_lr];
        for (uint32_t x = 0; x < W; ++x) {
            u128 ch = xs_copy_reset(&parent);
            if (keep) children[(uint64_t)next_lr * W + x] = ch;
        }
        if (keep) ++next_lr;
    }
    c.children = children;

    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * nthreads);
    for (uint32_t t = 1; t < nthreads; ++t) pthread_create(&th[t], NULL, worker, &c);
    worker(&c);
    for (uint32_t t = 1; t < nthreads; ++t) pthread_join(th[t], NULL);
    if (segments) *segments = atomic_load(&c.segments);

    free(th);
    free(children);
    free(c.objs);
    free(mats);
    free(c.offsets);
    return 0;
}

int orc_render(const orc_camera *cam, const orc_sphere *sph, uint32_t n_sph,
               const orc_material *mat, uint32_t n_mat, uint32_t samples_sqrt,
               uint64_t seed_lo, uint64_t seed_hi, uint32_t row_begin, uint32_t row_step,
               uint32_t n_rows, uint32_t nthreads, int scheduler, double *out,
               uint64_t *segments) {
    if (cam->img_width == 0 || cam->img_height == 0) return -1; /* camera.rs:267 */
    if (row_step == 0) row_step = 1;
    if (n_rows == 0) return 0;
    if ((uint64_t)row_begin + (uint64_t)(n_rows - 1) * row_step >= cam->img_height) return -2;
    uint32_t *rows = (uint32_t *)malloc(sizeof(uint32_t) * n_rows);
    for (uint32_t k = 0; k < n_rows; ++k) rows[k] = row_begin + k * row_step;
    int rc = render_rows(cam, sph, n_sph, mat, n_mat, samples_sqrt, seed_lo, seed_hi, rows, n_rows,
                         nthreads, scheduler, out, segments, NULL);
    free(rows);
    return rc;
}

int orc_render_rows(const orc_camera *cam, const orc_sphere *sph, uint32_t n_sph,
                    const orc_material *mat, uint32_t n_mat, uint32_t samples_sqrt,
                    uint64_t seed_lo, uint64_t seed_hi, const uint32_t *rows, uint32_t n_rows,
                    uint32_t nthreads, int scheduler, double *out, uint64_t *segments,
                    uint64_t *row_segments) {
    return render_rows(cam, sph, n_sph, mat, n_mat, samples_sqrt, seed_lo, seed_hi, rows, n_rows,
                       nthreads, scheduler, out, segments, row_segments);
}

/* ------------------------------------------------------------------ PPM --- */
/* Rust `f as u64`: saturating, NaN -> 0 */
static inline uint64_t sat_u64(double v) {
    if (!(v > 0.)) return 0; /* NaN, negatives, zeros */
    if (v >= 18446744073709551616.0) return UINT64_MAX;
    return (uint64_t)v;
}

/* color.rs:196-247: "P3\n{W} {H}\n255\n", then per image row the gamma-corrected
 * (powf(1/2.2)) channel values * 255 as u64, space separated, '\n' terminated. */
uint64_t orc_format_ppm(const double *rgb, uint32_t w, uint32_t h, char *buf, uint64_t cap) {
    char tmp[32];
    uint64_t n = 0;
#define PUT(str, len)                                                     \
    do {                                                                  \
        if (buf && n + (len) <= cap) memcpy(buf + n, (str), (len));       \
        n += (len);                                                       \
    } while (0)
    int l = snprintf(tmp, sizeof tmp, "P3\n%u %u\n255\n", w, h);
    PUT(tmp, (uint64_t)l);
    for (uint32_t y = 0; y < h; ++y) {
        for (uint64_t i = 0; i < 3ull * w; ++i) {
            double g = pow(rgb[(uint64_t)y * w * 3 + i], 1. / 2.2);
            l = snprintf(tmp, sizeof tmp, "%llu", (unsigned long long)sat_u64(g * 255.));
            PUT(tmp, (uint64_t)l);
            PUT(i + 1 == 3ull * w ? "\n" : " ", 1);
        }
    }
#undef PUT
    return n;
}
