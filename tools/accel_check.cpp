// accel_check.cpp -- host self-check of the exact-result BVH walk (csrc/rtw_accel.h).
//
// Test infrastructure (built by tests/test_accel.py, never shipped): for every ray
// it compares Scene::hit by the reference's brute-force scan (hittable.rs:131-143:
// every sphere, f64 Sphere::hit, first minimum in index order) with the kernel's
// accelerated path (always-spheres exactly, f32 BVH walk, f64 candidates, U check,
// brute-force fallback) -- the SAME walk code the device compiles. Rays: camera
// rays plus multi-bounce path rays (diffuse / mirror / glass-like continuations
// from the exact hits, so origins sit on surfaces and inside glass), random rays,
// and near-tangent rays aimed at sphere silhouettes.
//
//   accel_check SCENE SEED N_PATHS   (SCENE: a builtin name, or "random:K")
// Prints one JSON line of counts; exit 1 on any mismatch.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "rtw_accel.h"
#include "rtw_capi.h"

using namespace rtw_accel;

// 1: mirror a -DRTW_SELF_SKIP device build (candidate list without the sphere a
// segment leaves); 0 (default): the default device build's candidate list
static bool g_self_skip = false;

struct F4 {
    float x, y, z, w;
};

struct Rng {
    uint64_t s;
    uint64_t next() {
        uint64_t z = (s += 0x9e3779b97f4a7c15ull);
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
        return z ^ (z >> 31);
    }
    double u01() { return static_cast<double>(next() >> 11) * (1.0 / 9007199254740992.0); }
    double sym() { return 2. * u01() - 1.; }
};

struct Scene {
    std::vector<double> c, r, rr;
    std::vector<float> r2p;
    uint32_t n = 0;
    Bvh bvh;
    bool bvh_ok = false;
    std::vector<uint32_t> nbr_info;  // inside-cut lists (build_inside)
    std::vector<uint16_t> nbr_ids;
};

struct Hit {
    int idx = -1;
    double t = 0.;
};

// the reference's scan with the plain Sphere::hit
static Hit brute(const Scene &S, const double o[3], const double d[3]) {
    const double a = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
    Hit h;
    for (uint32_t i = 0; i < S.n; ++i) {
        double t;
        if (sphere_hit_f64_plain(o[0], o[1], o[2], d[0], d[1], d[2], a, S.c[3 * i], S.c[3 * i + 1],
                           S.c[3 * i + 2], S.rr[i], t) &&
            (h.idx < 0 || t < h.t))
            h.idx = static_cast<int>(i), h.t = t;
    }
    return h;
}

struct Counts {
    uint64_t rays = 0, walked = 0, visits = 0, max_visits = 0, cands = 0, fallbacks = 0,
             overflows = 0, not_walkable = 0, mismatches = 0, hits = 0, inside = 0, early = 0, early_tests = 0, self_skips = 0;
};

// The kernel's accelerated Scene::hit, host-side. `prev` = the sphere the path
// last hit (-1: none): the inside cut is tried first, as on the device.
static Hit accel(const Scene &S, const double o[3], const double d[3], Counts &k, int prev) {
    const double a = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
    Hit h;
    if (prev >= 0 && S.nbr_info[prev] != kNbrNone) {
        const uint32_t s = static_cast<uint32_t>(prev);
        double t;
        if (inside_far(o[0], o[1], o[2], d[0], d[1], d[2], a, S.c[3 * s], S.c[3 * s + 1], S.c[3 * s + 2],
                       S.rr[s], t)) {
            ++k.inside;
            h.idx = prev, h.t = t;
            const uint32_t info = S.nbr_info[s];
            for (uint32_t j = 0; j < (info & 0xffu); ++j) {
                const uint32_t i = S.nbr_ids[(info >> 8) + j];
                if (sphere_hit_f64(o[0], o[1], o[2], d[0], d[1], d[2], a, S.c[3 * i], S.c[3 * i + 1],
                                   S.c[3 * i + 2], S.rr[i], t) &&
                    better(t, i, h.t, h.idx))
                    h.idx = static_cast<int>(i), h.t = t;
            }
            return h;
        }
    }
    for (uint32_t i : S.bvh.always) {
        double t;
        if (sphere_hit_f64(o[0], o[1], o[2], d[0], d[1], d[2], a, S.c[3 * i], S.c[3 * i + 1],
                           S.c[3 * i + 2], S.rr[i], t) &&
            better(t, i, h.t, h.idx))
            h.idx = static_cast<int>(i), h.t = t;
    }
    if (S.bvh.n_node == 0) return h;
    const double mo = std::fmax(std::fmax(std::fabs(o[0]), std::fabs(o[1])), std::fabs(o[2]));
    const double sa = std::sqrt(a);
    WalkRay wr;
    const double inv = 1.0 / sa;
    if (!walk_setup(static_cast<float>(o[0]), static_cast<float>(o[1]), static_cast<float>(o[2]),
                    static_cast<float>(d[0] * inv), static_cast<float>(d[1] * inv),
                    static_cast<float>(d[2] * inv), mo, sa, filter_neg_g(mo), wr)) {
        ++k.not_walkable;
        return brute(S, o, d);
    }
    ++k.walked;
    if (prev >= 0 && g_self_skip) {  // opt-in device builds (-DRTW_SELF_SKIP) drop the sphere a
                                     // segment leaves (rtw_accel.h self_skip); default builds keep it
        const uint32_t p = static_cast<uint32_t>(prev);
        wr.skip = self_skip(prev, o[0], o[1], o[2], d[0], d[1], d[2], a, S.c[3 * p], S.c[3 * p + 1], S.c[3 * p + 2],
                            S.rr[p]);
        k.self_skips += wr.skip != 0xffffu ? 1u : 0u;
    }
    float U = INFINITY;
    if (h.idx >= 0) U = seed_cut(h.t, sa);
    uint32_t visits = 0;
    ArrayScratch ws;
    const bool ok = walk(reinterpret_cast<const F4 *>(S.bvh.nodes.data()),
                         reinterpret_cast<const F4 *>(S.bvh.leaves.data()), wr, U, visits, ws);
    const uint32_t nc = ws.nc;
    k.visits += visits;
    if (visits > k.max_visits) k.max_visits = visits;
    k.cands += nc;
    if (!ok) {
        ++k.overflows;
        return brute(S, o, d);
    }
    for (uint32_t j = 0; j < nc; ++j) {
        const uint32_t leaf = ws.cand_at(j);
        const uint32_t i = leaf;  // leaf id = sphere index
        double t;
        if (sphere_hit_f64(o[0], o[1], o[2], d[0], d[1], d[2], a, S.c[3 * i], S.c[3 * i + 1],
                           S.c[3 * i + 2], S.rr[i], t) &&
            better(t, i, h.t, h.idx))
            h.idx = static_cast<int>(i), h.t = t;
    }
    if (!cut_ok(U, h.idx, h.t, sa)) {
        ++k.fallbacks;
        return brute(S, o, d);
    }
    return h;
}

static void check(const Scene &S, const double o[3], const double d[3], Counts &k, Hit *out,
                  int prev = -1) {
    ++k.rays;
    const Hit b = brute(S, o, d);
    const Hit x = accel(S, o, d, k, prev);
    if (b.idx != x.idx || (b.idx >= 0 && std::memcmp(&b.t, &x.t, 8) != 0)) {
        if (k.mismatches < 10)
            fprintf(stderr, "MISMATCH o=(%.17g,%.17g,%.17g) d=(%.17g,%.17g,%.17g) brute=%d/%.17g accel=%d/%.17g\n",
                    o[0], o[1], o[2], d[0], d[1], d[2], b.idx, b.t, x.idx, x.t);
        ++k.mismatches;
    }
    if (b.idx >= 0) ++k.hits;
    if (out) *out = b;
}

static void finish_scene(Scene &S) {
    S.n = static_cast<uint32_t>(S.r.size());
    S.rr.resize(S.n);
    S.r2p.resize(S.n);
    for (uint32_t i = 0; i < S.n; ++i) {
        S.rr[i] = S.r[i] * S.r[i];
        S.r2p[i] = filter_r2p(&S.c[3 * i], S.rr[i]);
    }
    S.bvh_ok = build(S.c.data(), S.r.data(), S.r2p.data(), S.n, S.bvh);
    build_inside(S.c.data(), S.r.data(), S.n, S.nbr_info, S.nbr_ids);
}

int main(int argc, char **argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: accel_check SCENE SEED N_PATHS [SELF_SKIP 0|1]\n");
        return 2;
    }
    g_self_skip = argc > 4 ? std::atoi(argv[4]) != 0 : false;  // default: the default device build
    const std::string name = argv[1];
    const uint64_t seed = std::strtoull(argv[2], nullptr, 10);
    const uint64_t npaths = std::strtoull(argv[3], nullptr, 10);
    Rng rng{seed * 7919 + 17};
    Scene S;
    double from[3] = {13, 2, 3}, to[3] = {0, 0, 0};
    if (name.rfind("random:", 0) == 0) {
        // adversarial: clustered, coincident, nested, negative and tiny/huge radii
        const uint32_t K = static_cast<uint32_t>(std::atoi(name.c_str() + 7));
        for (uint32_t i = 0; i < K; ++i) {
            const double u = rng.u01();
            double cx = 6 * rng.sym(), cy = 2 * rng.sym(), cz = 6 * rng.sym();
            double r = 0.05 + 0.6 * rng.u01();
            if (u < 0.05 && i > 0) {  // coincident copy of an earlier sphere
                const uint32_t j = static_cast<uint32_t>(rng.next() % i);
                cx = S.c[3 * j], cy = S.c[3 * j + 1], cz = S.c[3 * j + 2], r = S.r[j];
            } else if (u < 0.10) {
                r = -r;  // hollow glass shell
            } else if (u < 0.13) {
                r = 1e-4 * rng.u01();
            } else if (u < 0.15) {
                r = 50 + 500 * rng.u01();  // huge -> always
            }
            S.c.insert(S.c.end(), {cx, cy, cz});
            S.r.push_back(r);
        }
        from[0] = 9, from[1] = 3, from[2] = 7;
    } else if (name.rfind("touch:", 0) == 0) {
        // near-tangent clusters: each sphere placed against an earlier one with a
        // gap of +-2^-k of the radii (k up to 60: overlapping, touching, just
        // apart), some nested, at a random offset up to 1e4 (inside-cut margins)
        const uint32_t K = static_cast<uint32_t>(std::atoi(name.c_str() + 6));
        const double off = std::ldexp(1., static_cast<int>(seed % 14));
        for (uint32_t i = 0; i < K; ++i) {
            double r = 0.05 + 0.5 * rng.u01();
            double cc[3] = {off + 4 * rng.sym(), 2 * rng.sym(), off + 4 * rng.sym()};
            if (i > 0 && rng.u01() < 0.8) {
                const uint32_t j = static_cast<uint32_t>(rng.next() % i);
                double v[3], vl;
                do {
                    v[0] = rng.sym(), v[1] = rng.sym(), v[2] = rng.sym();
                    vl = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
                } while (vl > 1. || vl < 1e-3);
                const double rj = std::fabs(S.r[j]);
                const double gap = std::ldexp(rng.sym(), -static_cast<int>(rng.next() % 61)) * (r + rj);
                const double dist = rng.u01() < 0.1 ? std::fabs(rj - r) * rng.u01() : rj + r + gap;
                for (int k2 = 0; k2 < 3; ++k2) cc[k2] = S.c[3 * j + k2] + v[k2] / vl * dist;
            }
            S.c.insert(S.c.end(), {cc[0], cc[1], cc[2]});
            S.r.push_back(r);
        }
        from[0] = off + 9, from[1] = 3, from[2] = off + 7;
        to[0] = off, to[2] = off;
    } else {
        rtw_camera cam;
        std::vector<rtw_sphere> sp(4096);
        std::vector<rtw_material> mt(4096);
        uint32_t ns = 0, nm = 0;
        if (rtw_scene_builtin(name.c_str(), rtw_u128{seed, 0}, 90, 160, 50, &cam, sp.data(), mt.data(),
                              4096, &ns, &nm) != 0) {
            fprintf(stderr, "scene: %s\n", rtw_last_error());
            return 2;
        }
        for (uint32_t i = 0; i < ns; ++i) {
            S.c.insert(S.c.end(), {sp[i].center[0], sp[i].center[1], sp[i].center[2]});
            S.r.push_back(sp[i].radius);
        }
        from[0] = cam.look_from.x, from[1] = cam.look_from.y, from[2] = cam.look_from.z;
        to[0] = cam.look_to.x, to[1] = cam.look_to.y, to[2] = cam.look_to.z;
    }
    finish_scene(S);
    Counts k;
    if (!S.bvh_ok) {
        printf("{\"scene\": \"%s\", \"bvh\": false}\n", name.c_str());
        return 0;
    }
    // 1. camera paths with bounces
    for (uint64_t p = 0; p < npaths; ++p) {
        double o[3] = {from[0] + 0.05 * rng.sym(), from[1] + 0.05 * rng.sym(), from[2] + 0.05 * rng.sym()};
        double d[3];
        for (int j = 0; j < 3; ++j) d[j] = (to[j] - from[j]) + 3.0 * rng.sym() * (j == 1 ? 0.6 : 1.0);
        int prev = -1;
        for (int depth = 0; depth < 50; ++depth) {
            Hit h;
            check(S, o, d, k, &h, prev);
            if (h.idx < 0) break;
            prev = h.idx;
            const uint32_t i = static_cast<uint32_t>(h.idx);
            double pnt[3], n[3];
            for (int j = 0; j < 3; ++j) pnt[j] = d[j] * h.t + o[j];
            for (int j = 0; j < 3; ++j) n[j] = (pnt[j] - S.c[3 * i + j]) / S.r[i];
            const double dn = d[0] * n[0] + d[1] * n[1] + d[2] * n[2];
            const double kind = rng.u01();
            double nd[3];
            if (kind < 0.4) {  // diffuse
                double u[3], l2;
                do {
                    u[0] = rng.sym(), u[1] = rng.sym(), u[2] = rng.sym();
                    l2 = u[0] * u[0] + u[1] * u[1] + u[2] * u[2];
                } while (l2 > 1. || l2 == 0.);
                const double s = dn < 0 ? 1. : -1.;
                for (int j = 0; j < 3; ++j) nd[j] = s * n[j] + u[j] / std::sqrt(l2);
            } else if (kind < 0.7) {  // mirror (sometimes grazing)
                for (int j = 0; j < 3; ++j) nd[j] = d[j] - 2. * dn * n[j];
            } else {  // continue straight (glass-like transmission: origin goes inside)
                for (int j = 0; j < 3; ++j) nd[j] = d[j] * (1. + 0.01 * rng.sym());
            }
            for (int j = 0; j < 3; ++j) o[j] = pnt[j], d[j] = nd[j];
        }
    }
    // 2. random rays
    for (uint64_t p = 0; p < npaths; ++p) {
        double o[3] = {8 * rng.sym(), 3 * rng.sym() + 1, 8 * rng.sym()};
        double d[3] = {rng.sym(), rng.sym(), rng.sym()};
        const double sc = std::exp(12 * rng.sym());  // unnormalised directions, many scales
        for (double &x : d) x *= sc;
        check(S, o, d, k, nullptr, S.n ? static_cast<int>(rng.next() % S.n) : -1);
    }
    // 3. near-tangent rays to random spheres (silhouettes), from outside and on-surface
    for (uint64_t p = 0; p < npaths && S.n; ++p) {
        const uint32_t i = static_cast<uint32_t>(rng.next() % S.n);
        const double R = std::fabs(S.r[i]);
        if (!(R < 1e6)) continue;
        double v[3] = {rng.sym(), rng.sym(), rng.sym()};
        const double vl = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
        double w[3] = {rng.sym(), rng.sym(), rng.sym()};  // direction
        const double wl = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
        for (int j = 0; j < 3; ++j) v[j] /= vl, w[j] /= wl;
        const double vw = v[0] * w[0] + v[1] * w[1] + v[2] * w[2];
        double q[3];  // q perpendicular to w
        for (int j = 0; j < 3; ++j) q[j] = v[j] - vw * w[j];
        const double ql = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2]);
        const double off = R * (1. + std::ldexp(rng.sym(), -static_cast<int>(rng.next() % 50)));
        const double back = rng.u01() < 0.5 ? 5. * R + 1. : 0.;
        double o[3], d[3];
        for (int j = 0; j < 3; ++j) {
            o[j] = S.c[3 * i + j] + q[j] / ql * off - w[j] * back;
            d[j] = w[j] * std::exp(4 * rng.sym());
        }
        check(S, o, d, k, nullptr, static_cast<int>(i));
    }
    // 4. rays from inside a sphere (interior points, and surface points with an
    // inward direction: trapped-ray bounces), hinted with that sphere
    for (uint64_t p = 0; p < npaths && S.n; ++p) {
        const uint32_t i = static_cast<uint32_t>(rng.next() % S.n);
        const double R = std::fabs(S.r[i]);
        if (!(R < 1e6)) continue;
        double v[3], vl;
        do {
            v[0] = rng.sym(), v[1] = rng.sym(), v[2] = rng.sym();
            vl = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
        } while (vl > 1. || vl < 1e-3);
        const double u = rng.u01();
        const double rad = u < 0.5 ? R : R * (u < 0.75 ? vl : 1. + std::ldexp(rng.sym(), -30));
        double o[3], d[3];
        for (int j = 0; j < 3; ++j) o[j] = S.c[3 * i + j] + v[j] / vl * rad;
        double w[3], wl;
        do {
            w[0] = rng.sym(), w[1] = rng.sym(), w[2] = rng.sym();
            wl = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
        } while (wl > 1. || wl < 1e-3);
        // inward: -n + unit (Lambertian from the inner face), or any direction
        const double in = rng.u01() < 0.7 ? -1. : 0.;
        const double sc = std::exp(3 * rng.sym());
        for (int j = 0; j < 3; ++j) d[j] = (in * v[j] / vl + w[j] / wl) * sc;
        check(S, o, d, k, nullptr, static_cast<int>(i));
    }
    // 5. sphere_early_miss (rtw_accel.h, opt-in): one sphere, origins on its surface
    // (rounded, plus offsets of +-2^-k radii; odd p: inside by |c| ~ 2 R^2 delta with
    // |d|^2 ~ |c| / 1.6e-5, the c < 0 bound's edge), directions outward / tangent /
    // inward at scales 2^-60 .. 2^60: every early miss is a miss of the plain Sphere::hit
    for (uint64_t p = 0; p < 4 * npaths && S.n; ++p) {
        const uint32_t i = static_cast<uint32_t>(rng.next() % S.n);
        const double R = std::fabs(S.r[i]);
        double v[3], vl;
        do {
            v[0] = rng.sym(), v[1] = rng.sym(), v[2] = rng.sym();
            vl = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
        } while (vl > 1. || vl < 1e-3);
        const double rad = R * (1. + (rng.u01() < 0.5 ? 0. : std::ldexp(rng.sym(), -static_cast<int>(rng.next() % 60))));
        double o[3], d[3], w[3];
        for (int j = 0; j < 3; ++j) o[j] = S.c[3 * i + j] + v[j] / vl * rad;
        for (int j = 0; j < 3; ++j) w[j] = rng.sym();
        const double mix = rng.u01() < 0.5 ? 1. : std::ldexp(rng.sym(), -static_cast<int>(rng.next() % 40));
        double sc = std::ldexp(1., static_cast<int>(rng.next() % 121) - 60);
        if (p & 1u) {
            const double delta = std::ldexp(1., -1 - static_cast<int>(rng.next() % 50));
            for (int j = 0; j < 3; ++j) o[j] = S.c[3 * i + j] + v[j] / vl * R * (1. - delta);
            double l2 = 0.;
            for (int j = 0; j < 3; ++j) l2 += (v[j] / vl * mix + w[j]) * (v[j] / vl * mix + w[j]);
            sc = std::sqrt(2. * R * R * delta / 1.6e-5 * std::exp(2. * rng.sym()) / l2);
        }
        for (int j = 0; j < 3; ++j) d[j] = (v[j] / vl * mix + w[j]) * sc;
        const double a = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
        const double ocx = o[0] - S.c[3 * i], ocy = o[1] - S.c[3 * i + 1], ocz = o[2] - S.c[3 * i + 2];
        const double hb = ocx * d[0] + ocy * d[1] + ocz * d[2];
        const double c = (ocx * ocx + ocy * ocy + ocz * ocz) - S.rr[i];
        ++k.early_tests;
        const bool early = sphere_early_miss(hb, c, a);
        k.early += early ? 1u : 0u;
        double t2 = 0.;
        const bool h2 = sphere_hit_f64_plain(o[0], o[1], o[2], d[0], d[1], d[2], a, S.c[3 * i], S.c[3 * i + 1],
                                             S.c[3 * i + 2], S.rr[i], t2);
        if (early && h2) {
            if (k.mismatches < 10)
                fprintf(stderr, "EARLY-MISS MISMATCH sphere %u hb=%.17g c=%.17g a=%.17g t=%.17g\n", i, hb, c, a, t2);
            ++k.mismatches;
        }
    }
    printf("{\"scene\": \"%s\", \"bvh\": true, \"n\": %u, \"always\": %zu, \"inner\": %u, \"depth\": %u, "
           "\"rays\": %llu, \"hits\": %llu, \"walked\": %llu, \"visits_per_walk\": %.3f, \"max_visits\": %llu, "
           "\"cands_per_walk\": %.3f, \"fallbacks\": %llu, \"overflows\": %llu, \"not_walkable\": %llu, "
           "\"inside_cuts\": %llu, \"self_skips\": %llu, \"early_miss\": %llu, \"early_tests\": %llu, \"mismatches\": %llu}\n",
           name.c_str(), S.n, S.bvh.always.size(), S.bvh.n_node, S.bvh.depth, (unsigned long long)k.rays,
           (unsigned long long)k.hits, (unsigned long long)k.walked,
           k.walked ? double(k.visits) / k.walked : 0., (unsigned long long)k.max_visits,
           k.walked ? double(k.cands) / k.walked : 0., (unsigned long long)k.fallbacks,
           (unsigned long long)k.overflows, (unsigned long long)k.not_walkable,
           (unsigned long long)k.inside, (unsigned long long)k.self_skips, (unsigned long long)k.early, (unsigned long long)k.early_tests,
           (unsigned long long)k.mismatches);
    return k.mismatches ? 1 : 0;
}
