// defer_model.cpp -- host model of the lane-compacted leaf pass.
//
// Developer tool (test infrastructure, never shipped). 64 lanes trace paths in lockstep
// through the final scene (camera rays, then Lambertian / metal / glass bounces by the
// scene's own materials, a new path when one ends), and every segment's Scene::hit runs
// the SAME walk the device compiles (rtw_accel.h) twice:
//   inline  -- the default walk: each visit runs its hit leaf children's filter test at
//              once (a wave pays max over lanes of the leaf children per visit) and the
//              sure hits shrink U;
//   defer   -- walk<true>: hit leaf children are only listed; after the walk one
//              wave-wide compacted pass filters all of them (ceil(total / lanes) trips).
// Per wave step it counts the wave-level trips of each loop (visit iterations = max
// visits, leaf trips, exact-test trips = max candidates) and, per lane, visits, leaf
// tests and candidates. Prints one JSON line.
//   defer_model SEED WAVE_STEPS
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "rtw_accel.h"
#include "rtw_capi.h"

using namespace rtw_accel;

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

// ArrayScratch that records the leaf children tested per visit (inline walk)
struct CountScratch : ArrayScratch {
    uint32_t cur = 0;
    std::vector<uint32_t> per_visit;
    void add_cand(uint32_t k, bool keep) {
        ++cur;
        ArrayScratch::add_cand(k, keep);
    }
    bool next(uint32_t &id) {
        per_visit.push_back(cur);
        cur = 0;
        return ArrayScratch::next(id);
    }
    void add_pending(uint64_t refs, uint32_t lmask, const F4 *, const WalkRay &, float &) {
        for (uint32_t j = 0; j < 4u; ++j)
            if ((lmask >> j) & 1u) add_cand(static_cast<uint32_t>(refs >> (16u * j)) & 0xffffu, true);
    }
};


// Lockstep model of the deferred walk with a mid-walk flush: every wave iteration
// each walking lane visits one node (hit leaf children listed, not tested); when
// the wave's listed leaves reach F (or a lane's list could overflow on its next
// visit), one compacted pass filters them all -- sure hits shrink their owner's U
// from then on -- in ceil(listed / walking lanes) trips. The host copy of walk()'s
// visit (rtw_accel.h), stepped one node at a time.
struct StepLane {
    WalkRay r;
    float U;
    uint32_t stk[64];
    uint32_t sp = 0, cur = 0, visits = 0, ncand = 0;
    std::vector<uint32_t> pend;
    bool done = false, bad = false;
};
static void step_visit(const F4 *nodes, StepLane &L) {
    const WalkRay &r = L.r;
    const uint32_t sx = r.neg & 1u, sy = (r.neg >> 1) & 1u, sz = r.neg >> 2;
    const uint32_t oct_shift = 8u * (r.neg & 3u);
    const bool oct_hi = r.neg >= 4u;
    ++L.visits;
    const F4 *N = nodes + kNodeF4 * L.cur;
    const F4 nX = N[sx], fX = N[sx ^ 1u], nY = N[2u + sy], fY = N[3u - sy], nZ = N[4u + sz], fZ = N[5u - sz],
             qc = N[6], qo = N[7];
    uint32_t hit = slab_hit4(nX, nY, nZ, fX, fY, fZ, r, L.U);
    const uint32_t r01 = as_u32(qc.x), r23 = as_u32(qc.y), masks = as_u32(qc.z);
    hit &= masks;
    const uint32_t lmask = hit & (masks >> 4);
    const uint32_t inner = hit & ~lmask & 15u;
    const uint64_t refs = (static_cast<uint64_t>(r23) << 32) | r01;
    for (uint32_t j = 0; j < 4; ++j)
        if ((lmask >> j) & 1u) L.pend.push_back(static_cast<uint32_t>(refs >> (16u * j)) & 0xffffu);
    const uint32_t ord = ((oct_hi ? as_u32(qo.y) : as_u32(qo.x)) >> oct_shift) & 0xffu;
    for (int t = 3; t >= 0; --t) {
        const uint32_t j = (ord >> (2 * t)) & 3u;
        if ((inner >> j) & 1u) L.stk[L.sp++] = static_cast<uint32_t>(refs >> (16u * j)) & 0xffffu;
    }
    if (L.sp == 0) L.done = true;
    else L.cur = L.stk[--L.sp];
}
struct FlushCounts {
    double iters = 0, trips = 0, flushes = 0, visits = 0, cands = 0, cand_trips = 0, walks = 0, waves = 0, tests = 0;
};
static void lockstep(const F4 *nodes, const F4 *leaves, std::vector<StepLane> &W, uint32_t F, FlushCounts &fc) {
    if (W.empty()) return;
    auto flush = [&](uint32_t lanes) {
        uint32_t total = 0;
        for (auto &L : W) total += static_cast<uint32_t>(L.pend.size());
        if (!total) return;
        fc.trips += (total + lanes - 1) / lanes;
        fc.flushes += 1;
        for (auto &L : W) {
            for (uint32_t k : L.pend) {
                ArrayScratch one;
                leaf_test(leaves, k, L.r, L.U, one);  // the filter + the sure-hit U
                L.ncand += one.nc;
                fc.tests += 1;
            }
            L.pend.clear();
        }
    };
    uint32_t it = 0;
    for (;;) {
        uint32_t walking = 0;
        for (auto &L : W)
            if (!L.done) ++walking;
        if (!walking) break;
        ++it;
        for (auto &L : W)
            if (!L.done) step_visit(nodes, L);
        uint32_t total = 0;
        bool full = false;
        for (auto &L : W) {
            total += static_cast<uint32_t>(L.pend.size());
            full = full || (!L.done && L.pend.size() + L.ncand + 4 > kMaxCand);
        }
        if (F && (total >= F || full)) flush(walking);
    }
    flush(static_cast<uint32_t>(W.size()));
    uint32_t cmax = 0;
    for (auto &L : W) fc.visits += L.visits, fc.cands += L.ncand, cmax = std::max(cmax, L.ncand);
    fc.iters += it, fc.cand_trips += cmax, fc.walks += W.size(), fc.waves += 1;
}

struct Lane {
    double o[3], d[3];
    int prev = -1;
    uint32_t depth = 0;
    bool live = false;
};

int main(int argc, char **argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: defer_model SEED WAVE_STEPS\n");
        return 2;
    }
    const uint64_t seed = std::strtoull(argv[1], nullptr, 10);
    const uint64_t steps = std::strtoull(argv[2], nullptr, 10);
    Rng rng{seed * 7919 + 17};
    rtw_camera cam;
    std::vector<rtw_sphere> sp(4096);
    std::vector<rtw_material> mt(4096);
    uint32_t ns = 0, nm = 0;
    if (rtw_scene_builtin("complex", rtw_u128{1764892800000ull, 0}, 675, 1200, 50, &cam, sp.data(), mt.data(), 4096,
                          &ns, &nm) != 0) {
        fprintf(stderr, "scene: %s\n", rtw_last_error());
        return 2;
    }
    std::vector<double> c, r, rr;
    std::vector<float> r2p;
    for (uint32_t i = 0; i < ns; ++i) {
        c.insert(c.end(), {sp[i].center[0], sp[i].center[1], sp[i].center[2]});
        r.push_back(sp[i].radius);
        rr.push_back(sp[i].radius * sp[i].radius);
        r2p.push_back(filter_r2p(&c[3 * i], rr[i]));
    }
    Bvh bvh;
    if (!build(c.data(), r.data(), r2p.data(), ns, bvh)) {
        fprintf(stderr, "no bvh\n");
        return 2;
    }
    std::vector<uint32_t> nbr_info;
    std::vector<uint16_t> nbr_ids;
    build_inside(c.data(), r.data(), ns, nbr_info, nbr_ids);
    const F4 *nodes = reinterpret_cast<const F4 *>(bvh.nodes.data());
    const F4 *leaves = reinterpret_cast<const F4 *>(bvh.leaves.data());
    const double from[3] = {cam.look_from.x, cam.look_from.y, cam.look_from.z};
    const double to[3] = {cam.look_to.x, cam.look_to.y, cam.look_to.z};

    struct Tot {
        double iters = 0, leaf_trips = 0, cand_trips = 0, visits = 0, leaf_tests = 0, cands = 0, overflow = 0,
               fallback = 0, pass_trips = 0, walks = 0, max_pending = 0, waves = 0, wave_overflow = 0;
    } in, df;
    Lane L[64];
    static constexpr uint32_t kFs[] = {0u, 8u, 16u, 32u, 64u, 128u};
    constexpr size_t kNF = sizeof(kFs) / sizeof(kFs[0]);
    FlushCounts fcs[kNF];
    auto restart = [&](Lane &l) {
        for (int j = 0; j < 3; ++j) l.o[j] = from[j] + 0.02 * rng.sym();
        for (int j = 0; j < 3; ++j) l.d[j] = (to[j] - from[j]) + 2.2 * rng.sym() * (j == 1 ? 0.6 : 1.0);
        l.prev = -1, l.depth = 0, l.live = true;
    };
    for (auto &l : L) restart(l);
    for (uint64_t s = 0; s < steps; ++s) {
        uint32_t in_it = 0, df_it = 0, in_cmax = 0, df_cmax = 0, df_total = 0, wave_walks = 0;
        bool in_of = false, df_of = false;
        std::vector<std::vector<uint32_t>> pv(64);
        std::vector<StepLane> W;
        for (int li = 0; li < 64; ++li) {
            Lane &l = L[li];
            const double a = l.d[0] * l.d[0] + l.d[1] * l.d[1] + l.d[2] * l.d[2];
            // the exact first hit (the scan) decides the path; the walks are only counted
            int best = -1;
            double bt = 0.;
            for (uint32_t i = 0; i < ns; ++i) {
                double t;
                if (sphere_hit_f64(l.o[0], l.o[1], l.o[2], l.d[0], l.d[1], l.d[2], a, c[3 * i], c[3 * i + 1],
                                   c[3 * i + 2], rr[i], t) &&
                    better(t, i, bt, best))
                    best = static_cast<int>(i), bt = t;
            }
            // inside cut first, as on the device: such segments do not walk
            bool walked = false;
            double tin;
            const bool inside = l.prev >= 0 && nbr_info[l.prev] != kNbrNone &&
                                inside_far(l.o[0], l.o[1], l.o[2], l.d[0], l.d[1], l.d[2], a, c[3 * l.prev],
                                           c[3 * l.prev + 1], c[3 * l.prev + 2], rr[l.prev], tin);
            if (!inside) {
                const double mo = std::fmax(std::fmax(std::fabs(l.o[0]), std::fabs(l.o[1])), std::fabs(l.o[2]));
                const double sa = std::sqrt(a), inv = 1.0 / sa;
                WalkRay wr;
                if (walk_setup(static_cast<float>(l.o[0]), static_cast<float>(l.o[1]), static_cast<float>(l.o[2]),
                               static_cast<float>(l.d[0] * inv), static_cast<float>(l.d[1] * inv),
                               static_cast<float>(l.d[2] * inv), mo, sa, filter_neg_g(mo), wr)) {
                    walked = true;
                    float U0 = INFINITY;
                    int ab = -1;
                    double at = 0.;
                    for (uint32_t i : bvh.always) {
                        double t;
                        if (sphere_hit_f64(l.o[0], l.o[1], l.o[2], l.d[0], l.d[1], l.d[2], a, c[3 * i], c[3 * i + 1],
                                           c[3 * i + 2], rr[i], t) &&
                            better(t, i, at, ab))
                            ab = static_cast<int>(i), at = t;
                    }
                    if (ab >= 0) U0 = seed_cut(at, sa);
                    {
                        StepLane sl;
                        sl.r = wr, sl.U = U0;
                        W.push_back(sl);
                    }
                    // inline
                    {
                        float U = U0;
                        uint32_t v = 0;
                        CountScratch ws;
                        const bool ok = walk<false>(nodes, leaves, wr, U, v, ws);
                        in.visits += v, in.cands += ws.nc, in.walks += 1;
                        in_it = std::max(in_it, v);
                        in_cmax = std::max(in_cmax, ws.nc);
                        for (uint32_t x : ws.per_visit) in.leaf_tests += x;
                        pv[li] = ws.per_visit;
                        if (!ok) in.overflow += 1, in_of = true;
                        else if (!cut_ok(U, best, bt, sa)) in.fallback += 1;
                    }
                    // deferred
                    {
                        float U = U0;
                        uint32_t v = 0;
                        CountScratch ws;
                        const bool ok = walk<true>(nodes, leaves, wr, U, v, ws);
                        df.visits += v, df.walks += 1, df.leaf_tests += ws.nc;
                        df.max_pending = std::max(df.max_pending, static_cast<double>(ws.nc));
                        df_it = std::max(df_it, v);
                        df_total += ws.nc;
                        uint32_t kept = 0;
                        for (uint32_t j = 0; j < ws.nc; ++j) {
                            const uint32_t k = ws.cand_at(j);
                            const F4 S = leaves[2 * k];
                            const float ocx = wr.ox - S.x, ocy = wr.oy - S.y, ocz = wr.oz - S.z;
                            const float hb = fmaf(ocx, wr.ex, fmaf(ocy, wr.ey, ocz * wr.ez));
                            const float cc = fmaf(ocx, ocx, fmaf(ocy, ocy, fmaf(ocz, ocz, -S.w)));
                            kept += !(fmaf(hb, hb, -cc) < wr.negG) ? 1u : 0u;
                        }
                        df.cands += kept;
                        df_cmax = std::max(df_cmax, kept);
                        if (!ok) df.overflow += 1, df_of = true;
                    }
                    ++wave_walks;
                }
            }
            (void)walked;
            // continue the path by the material
            if (best < 0 || ++l.depth >= 50) {
                restart(l);
                continue;
            }
            const uint32_t i = static_cast<uint32_t>(best);
            double p[3], n[3];
            for (int j = 0; j < 3; ++j) p[j] = l.d[j] * bt + l.o[j];
            for (int j = 0; j < 3; ++j) n[j] = (p[j] - c[3 * i + j]) / r[i];
            const double dn = l.d[0] * n[0] + l.d[1] * n[1] + l.d[2] * n[2];
            const bool front = dn < 0.;
            if (!front)
                for (double &x : n) x = -x;
            const rtw_material &M = mt[sp[i].mat];
            double u[3], l2;
            do {
                u[0] = rng.sym(), u[1] = rng.sym(), u[2] = rng.sym();
                l2 = u[0] * u[0] + u[1] * u[1] + u[2] * u[2];
            } while (l2 > 1. || l2 == 0.);
            for (double &x : u) x /= std::sqrt(l2);
            double nd[3];
            const double len = std::sqrt(a);
            double v[3] = {l.d[0] / len, l.d[1] / len, l.d[2] / len};
            if (M.kind == RTW_LAMBERTIAN) {
                for (int j = 0; j < 3; ++j) nd[j] = n[j] + u[j];
            } else if (M.kind == RTW_METAL) {
                const double dt = v[0] * n[0] + v[1] * n[1] + v[2] * n[2];
                for (int j = 0; j < 3; ++j) nd[j] = v[j] - 2. * dt * n[j] + M.fuzz * u[j];
            } else {
                const double ratio = front ? 1. / M.ir : M.ir;
                const double ct = std::fmin(-(v[0] * n[0] + v[1] * n[1] + v[2] * n[2]), 1.);
                const double st = std::sqrt(1. - ct * ct);
                const double r0 = (1. - M.ir) / (1. + M.ir);
                const double sch = r0 * r0 + (1. - r0 * r0) * std::pow(1. - ct, 5.);
                if (ratio * st > 1. || sch > rng.u01()) {
                    const double dt = v[0] * n[0] + v[1] * n[1] + v[2] * n[2];
                    for (int j = 0; j < 3; ++j) nd[j] = v[j] - 2. * dt * n[j];
                } else {
                    double q[3];
                    for (int j = 0; j < 3; ++j) q[j] = (v[j] + ct * n[j]) * ratio;
                    const double w = -std::sqrt(std::fabs(1. - (q[0] * q[0] + q[1] * q[1] + q[2] * q[2])));
                    for (int j = 0; j < 3; ++j) nd[j] = q[j] + w * n[j];
                }
            }
            for (int j = 0; j < 3; ++j) l.o[j] = p[j], l.d[j] = nd[j];
            l.prev = best;
        }
        if (!wave_walks) continue;
        for (size_t f = 0; f < kNF; ++f) {
            std::vector<StepLane> Wc = W;
            lockstep(nodes, leaves, Wc, kFs[f], fcs[f]);
        }
        // wave-level leaf trips of the inline walk: per visit iteration, max over lanes
        uint32_t trips = 0;
        for (uint32_t it = 0; it < in_it; ++it) {
            uint32_t m = 0;
            for (int li = 0; li < 64; ++li)
                if (it < pv[li].size()) m = std::max(m, pv[li][it]);
            trips += m;
        }
        in.waves += 1, df.waves += 1;
        in.iters += in_it, df.iters += df_it;
        in.leaf_trips += trips;
        df.pass_trips += (df_total + wave_walks - 1) / wave_walks;
        in.cand_trips += in_cmax, df.cand_trips += df_cmax;
        in.wave_overflow += in_of, df.wave_overflow += df_of;
    }
    auto dump = [](const char *name, const Tot &t) {
        printf("\"%s\": {\"visit_iters_per_wave\": %.3f, \"leaf_trips_per_wave\": %.3f, \"pass_trips_per_wave\": %.3f, "
               "\"cand_trips_per_wave\": %.3f, \"visits_per_walk\": %.3f, \"leaf_tests_per_walk\": %.3f, "
               "\"cands_per_walk\": %.3f, \"overflow_per_walk\": %.5f, \"waves_with_overflow\": %.4f, "
               "\"fallback_per_walk\": %.5f, \"max_pending\": %.0f}",
               name, t.iters / t.waves, t.leaf_trips / t.waves, t.pass_trips / t.waves, t.cand_trips / t.waves,
               t.visits / t.walks, t.leaf_tests / t.walks, t.cands / t.walks, t.overflow / t.walks,
               t.wave_overflow / t.waves, t.fallback / t.walks, t.max_pending);
    };
    printf("{\"waves\": %.0f, ", in.waves);
    dump("inline", in);
    printf(", ");
    dump("defer", df);
    for (size_t f = 0; f < kNF; ++f) {
        const FlushCounts &q = fcs[f];
        printf(", \"flush_at_%u\": {\"visit_iters_per_wave\": %.3f, \"pass_trips_per_wave\": %.3f, \"flushes_per_wave\": %.3f, "
               "\"cand_trips_per_wave\": %.3f, \"visits_per_walk\": %.3f, \"leaf_tests_per_walk\": %.3f, \"cands_per_walk\": %.3f}",
               kFs[f], q.iters / q.waves, q.trips / q.waves, q.flushes / q.waves, q.cand_trips / q.waves,
               q.visits / q.walks, q.tests / q.walks, q.cands / q.walks);
    }
    printf("}\n");
    return 0;
}
