// rtw_accel.h -- exact-result sphere BVH for Scene::hit (hittable.rs:131-143).
//
// The reference tests every object and keeps the first minimum (`min_by` over
// partial_cmp in insertion order). This header replaces the O(n) scan with a
// conservative f32 BVH walk that provably returns the SAME (t, index) as the scan:
//
//   1. "always" spheres (huge radius, or outside the f32 guard) are tested exactly
//      first, in index order;
//   2. the BVH walk (f32) only collects candidate spheres; a node is skipped only
//      if (a) the padded ray/box slab test proves the ray misses it, (b) its far
//      end lies before t = 0.01 (Interval::from(0.01), camera.rs:387), or (c) its
//      near end lies beyond U, a running estimate of the closest hit distance;
//      a leaf is skipped only if the exact-conservative f32 discriminant filter
//      proves the f64 discriminant negative (DESIGN.md "Exact pre-filter");
//   3. candidates get the reference's own f64 Sphere::hit (sphere.rs:39-71) and
//      the lexicographic (t, index) minimum -- the scan's first-minimum rule;
//   4. verification: a cut by (c) is safe iff the final t <= U. U is only an
//      estimate, so if the final hit is farther than U (or missing) the lane
//      redoes the segment by brute force. Correctness rests on (a), (b), the leaf
//      filter and this check, never on the quality of U.
//
// Padding (a): with o32 = fl32(o), e32 = fl32(d/|d|), the computed ray deviates
// from the exact one by <= 5 u32 (|o|_max + M_b) at any point of a box whose
// coordinates are bounded by M_b; f32 slab arithmetic adds ~3 u32 of the same
// scale and the f64 root's tangent error is ~2^-26 |oc|. Every box is inflated by
// kPadK * M_b on the host and every lane widens its slabs by kPadK * |o|_max, with
// kPadK = 2^-16 (> 30x the bound).
//
// Shared by the device kernel (rtw_render.hip) and the host self-check
// (tools/accel_check.cpp): one definition of the walk for both.
#pragma once

#include <cstdint>
#include <cstring>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define RTW_HD __host__ __device__ __forceinline__
#else
#define RTW_HD inline
#endif
#include <cmath>
#include <vector>

namespace rtw_accel {

constexpr float kPadK = 1.52587890625e-05f;  // 2^-16
constexpr double kPadKd = 1.52587890625e-05;
constexpr float kDirFloor = 9.094947017729282e-13f;  // 2^-40: |e_i| clamp before 1/e_i
constexpr float kGuardBvh = 1e8f;       // |origin| beyond -> brute force for the segment
constexpr uint32_t kMaxSpheres = 32768;  // 16-bit leaf / node ids
constexpr uint32_t kEmpty = 0xffffffffu;  // "no node"
// Node stride 9 float4 (144 B): with 8 (128 B) every node starts on one of 2 of
// the 16 four-bank slots and ds_read_b128 gathers of different nodes conflict
// 8-way; an odd stride spreads them over all 16.
constexpr uint32_t kNodeF4 = 9;
constexpr uint32_t kNodeFloats = 4 * kNodeF4;
constexpr uint32_t kMaxAlways = 16;
constexpr uint32_t kMaxCand = 8;        // candidate list entries (walk scratch)
constexpr double kHugeRatio = 16.0;     // radius > kHugeRatio x median radius -> "always"

// Node (128 B, eight float4; 4-wide, children in the parent):
//   q0..q5 = lo.x[4], hi.x[4], lo.y[4], hi.y[4], lo.z[4], hi.z[4] (padded boxes
//   of the 4 children; an empty slot has every plane at +inf and is never hit),
//   q6.x/.y = child refs, 16 bits each (slot j in bits 16 (j & 1) of q6[j >> 1]):
//   inner node id or leaf k; q6.z = slot masks: bits 0-3 occupied, bits 4-7 leaf,
//   q7.x/.y = near-to-far child order per ray octant: byte o (octant bit k set
//   = direction k negative) holds 4 2-bit slot indices, nearest first.
// Leaf (32 B, two float4), leaf id = sphere index: {cx, cy, cz, R2'} (the pass-1
// filter record) and {d2, sphere index, 0, 0} with d2 >= 2 (R2' - r*r) (the
// filter's inflation, x2).

RTW_HD uint32_t as_u32(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
}
RTW_HD float as_f32(uint32_t u) {
    float f;
    memcpy(&f, &u, 4);
    return f;
}

RTW_HD float rcp32(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_rcpf(x);
#else
    return 1.0f / x;
#endif
}
RTW_HD float fmin3(float a, float b, float c) { return fminf(fminf(a, b), c); }
RTW_HD float fmax3(float a, float b, float c) { return fmaxf(fmaxf(a, b), c); }

// The reference's Sphere::hit (sphere.rs:39-71) in f64 with its operation order:
// a = d.d (hoisted), hb = oc.d, c = oc.oc - r*r, disc = hb*hb - a*c; roots
// (-sq - hb)/a then (sq - hb)/a, the first inside [0.01, inf] (interval.rs:55-57).
//
// Exact early miss (no sqrt, no division; host analysis only -- on the device it
// measured +0.3 %, a wave rarely skips as a whole, ab_early_miss_REJECTED.log): a ray
// leaving a sphere it starts on or outside of (hb >= 0, c >= -1.6e-5 a). With
// c >= 0, disc = RN(RN(hb^2) - RN(a c)) <= RN(hb^2) so sq <= hb and both roots
// are <= 0. With -1.6e-5 a <= c < 0 (origin on the surface up to rounding) the
// far root the reference computes is <= 1.0001 (sqrt(|c|/a) + 3u hb/a) < 0.0044
// for hb <= 1e12 a; both rejected by t >= 0.01. The magnitude guards keep every
// product finite and normal. Bounds in DESIGN.md 3.4; the plain form below stays
// the host checks' brute-force reference (tests/test_accel.py compares the two).
RTW_HD bool sphere_early_miss(double hb, double c, double a) {
    return hb >= 0. && c >= -1.6e-5 * a && hb <= 1e12 * a && a >= 1e-100 && a <= 1e100;
}
RTW_HD bool sphere_hit_f64_plain(double ox, double oy, double oz, double dx, double dy, double dz,
                                 double a, double cx, double cy, double cz, double rr, double &t) {
    const double ocx = ox - cx, ocy = oy - cy, ocz = oz - cz;
    const double hb = ocx * dx + ocy * dy + ocz * dz;
    const double c = (ocx * ocx + ocy * ocy + ocz * ocz) - rr;
    const double disc = hb * hb - a * c;
    if (disc < 0.) return false;
    const double sq = __builtin_sqrt(disc);
    t = (-sq - hb) / a;
    if (!(t >= 0.01)) t = (sq - hb) / a;
    return t >= 0.01;
}
RTW_HD bool sphere_hit_f64(double ox, double oy, double oz, double dx, double dy, double dz,
                           double a, double cx, double cy, double cz, double rr, double &t) {
    const double ocx = ox - cx, ocy = oy - cy, ocz = oz - cz;
    const double hb = ocx * dx + ocy * dy + ocz * dz;
    const double c = (ocx * ocx + ocy * ocy + ocz * ocz) - rr;
    const double disc = hb * hb - a * c;
    if (disc < 0.) return false;
    const double sq = __builtin_sqrt(disc);
    t = (-sq - hb) / a;
    if (!(t >= 0.01)) t = (sq - hb) / a;
    return t >= 0.01;
}

// The sphere a segment starts on, as a leaf the walk may drop: a ray leaving it
// (sphere_early_miss on the exact hb and c that sphere_hit_f64 computes, same
// operations) cannot hit it at t >= 0.01, so the scan's minimum is the same
// without it. Every bounce off a BVH sphere used to carry it as a candidate and an
// exact f64 test (sqrt and both divisions). Returns the leaf id or 0xffff. Host
// analysis only: on the device, 37 % fewer candidates, but the wave's candidate
// loop runs for its busiest lane's real candidates and the f64 check costs more
// (+0.8 %, profiles/r02_misc/ab_self_skip_REJECTED.log).
RTW_HD uint32_t self_skip(int prev, double ox, double oy, double oz, double dx, double dy, double dz,
                          double a, double cx, double cy, double cz, double rr) {
    const double ocx = ox - cx, ocy = oy - cy, ocz = oz - cz;
    const double hb = ocx * dx + ocy * dy + ocz * dz;
    const double c = (ocx * ocx + ocy * ocy + ocz * ocz) - rr;
    return prev >= 0 && sphere_early_miss(hb, c, a) ? static_cast<uint32_t>(prev) : 0xffffu;
}

// Exact-conservative f32 pre-filter of the discriminant (DESIGN.md "Exact
// pre-filter"): records carry R2' >= r*r + K (m_c^2 + r*r/2) (host, rounded up)
// and a lane with origin magnitude m_o keeps a sphere unless disc32 < -G,
// G = K m_o^2 + floor. K = 2^-15 = 512 u32 (the first-order bound needs 163 u32).
constexpr double kFilterK = 3.0517578125e-05;  // 2^-15
constexpr double kFilterFloor = 1e-25;         // f32 underflow errors inside the guard
constexpr double kGuardHi = 1e12;              // max |origin| / |center| component for f32

RTW_HD float filter_neg_g(double mo) {
    return -static_cast<float>(fma(kFilterK * mo, mo * 1.000001, kFilterFloor));
}

// Per-segment ray state for the f32 walk.
struct WalkRay {
    float ox, oy, oz;   // o32
    float ex, ey, ez;   // e32 (filter direction, ~unit)
    float ix, iy, iz;   // 1 / clamped e32
    // slab offsets, padded outward: t = plane * inv + a. The near plane of axis k
    // is lo (q[2k]) for a non-negative direction, hi (q[2k+1]) for a negative one;
    // an* go with the near plane, af* with the far plane.
    float anx, any, anz, afx, afy, afz;
    float tmin;         // 0.01 |d| rounded down (distance units)
    float negG;         // -(filter margin G)
    uint32_t neg;       // bit k: e32 component k < 0 (near child = right on that axis)
    uint32_t skip;      // a leaf the walk never keeps (self_skip), 0xffff: none
};

RTW_HD float clamp_dir(float e) {
    return fabsf(e) < kDirFloor ? (e < 0.f ? -kDirFloor : kDirFloor) : e;
}

// o32/e32 as used by the pass-1 filter (e32 = fl32(d / sqrt(a))), mo = max |o_i|
// (f64), sa = sqrt(a). Returns false if the segment must be brute-forced
// (non-finite or out-of-guard ray).
RTW_HD bool walk_setup(float ox, float oy, float oz, float ex, float ey, float ez, double mo,
                       double sa, float negG, WalkRay &r) {
    if (!(mo <= static_cast<double>(kGuardBvh)) || !(sa > 0.) || !(sa < 1e30)) return false;
    if (!(fabsf(ex) <= 2.f) || !(fabsf(ey) <= 2.f) || !(fabsf(ez) <= 2.f)) return false;
    r.ox = ox, r.oy = oy, r.oz = oz, r.ex = ex, r.ey = ey, r.ez = ez;
    r.neg = (ex < 0.f ? 1u : 0u) | (ey < 0.f ? 2u : 0u) | (ez < 0.f ? 4u : 0u);
    r.skip = 0xffffu;
    r.ix = rcp32(clamp_dir(ex)), r.iy = rcp32(clamp_dir(ey)), r.iz = rcp32(clamp_dir(ez));
    const float pad = kPadK * static_cast<float>(mo) + 1e-30f;
    // lo-plane offset -(o + pad) inv, hi-plane offset -(o - pad) inv; for a
    // negative direction the hi plane is the near one (same t values as testing
    // both planes and taking min / max: the order is fixed by the sign of inv)
    const float alx = -(ox + pad) * r.ix, ahx = -(ox - pad) * r.ix;
    const float aly = -(oy + pad) * r.iy, ahy = -(oy - pad) * r.iy;
    const float alz = -(oz + pad) * r.iz, ahz = -(oz - pad) * r.iz;
    const bool nx = r.neg & 1u, ny = r.neg & 2u, nz = r.neg & 4u;
    r.anx = nx ? ahx : alx, r.afx = nx ? alx : ahx;
    r.any = ny ? ahy : aly, r.afy = ny ? aly : ahy;
    r.anz = nz ? ahz : alz, r.afz = nz ? alz : ahz;
    r.tmin = static_cast<float>(0.01 * sa * (1. - 1e-6));
    r.negG = negG;
    return true;
}

// U seeded from an exact hit at parameter t: the distance t*sa, rounded up with
// room for the final check below.
RTW_HD float seed_cut(double t, double sa) {
    return static_cast<float>(t * sa * (1. + 1. / 262144.)) * (1.f + 2.4e-7f);
}
// The cut was safe iff the final hit is no farther than U (module comment, 4).
RTW_HD bool cut_ok(float U, int best, double bt, double sa) {
    return !(U < INFINITY) || (best >= 0 && bt * sa <= static_cast<double>(U) * (1. - 1. / 1048576.));
}

RTW_HD float sqrt32(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_sqrtf(x);  // U is an estimate: the approximate root suffices
#else
    return sqrtf(x);
#endif
}

// One box slab test against the padded box of a child: its near planes (nx, ny,
// nz) and far planes (fx, fy, fz) for this ray's direction signs. Hit iff the
// entry/exit interval meets [tmin, U] (all values finite: walk_setup rejects
// non-finite rays, empty slots are masked by the caller).
RTW_HD bool slab_hit(float nx, float ny, float nz, float fx, float fy, float fz, const WalkRay &r,
                     float U) {
    const float tn = fmax3(fmaf(nx, r.ix, r.anx), fmaf(ny, r.iy, r.any), fmaf(nz, r.iz, r.anz));
    const float tf = fmin3(fmaf(fx, r.ix, r.afx), fmaf(fy, r.iy, r.afy), fmaf(fz, r.iz, r.afz));
    return fmaxf(tn, r.tmin) <= fminf(tf, U);
}

// The four children's slab tests of one node as a hit mask (bit j = child j).
// (The 24 plane FMAs as 12 v_pk_fma_f32 measured slower -- parity +2.8 %, fast mode
// +5 %: a packed pair occupies the SIMD as long as two plain f32 FMAs on gfx950, and
// the broadcast ray constants take 9 more VGPRs; profiles/r02_misc/ab_pk_slab_REJECTED.log.)
template <typename F4>
RTW_HD uint32_t slab_hit4(const F4 &nX, const F4 &nY, const F4 &nZ, const F4 &fX, const F4 &fY,
                          const F4 &fZ, const WalkRay &r, float U) {
    uint32_t hit = 0;
    hit |= slab_hit(nX.x, nY.x, nZ.x, fX.x, fY.x, fZ.x, r, U) ? 1u : 0u;
    hit |= slab_hit(nX.y, nY.y, nZ.y, fX.y, fY.y, fZ.y, r, U) ? 2u : 0u;
    hit |= slab_hit(nX.z, nY.z, nZ.z, fX.z, fY.z, fZ.z, r, U) ? 4u : 0u;
    hit |= slab_hit(nX.w, nY.w, nZ.w, fX.w, fY.w, fZ.w, r, U) ? 8u : 0u;
    return hit;
}

// The pass-1 filter on leaf k; a kept sphere joins the candidate list (an
// overflow is recorded in the scratch, the walk stops after the node) and, if it
// is a sure hit (disc beyond the filter's inflation + error, far root clearly past
// tmin), its far root bounds the closest hit: U shrinks. Both loads are issued
// together and the sure-hit bound is a select, not a branch: the wave runs this
// body once per leaf of its busiest lane, so every branch in it is paid by all.
template <typename F4, typename Scratch>
RTW_HD void leaf_test(const F4 *__restrict__ leaves, uint32_t k, const WalkRay &r, float &U,
                      Scratch &ws) {
    const F4 S = leaves[2 * k];
    const float d2 = leaves[2 * k + 1].x;
    const float ocx = r.ox - S.x, ocy = r.oy - S.y, ocz = r.oz - S.z;
    const float hb = fmaf(ocx, r.ex, fmaf(ocy, r.ey, ocz * r.ez));
    const float cc = fmaf(ocx, ocx, fmaf(ocy, ocy, fmaf(ocz, ocz, -S.w)));
    const float disc = fmaf(hb, hb, -cc);
#ifndef __HIP_DEVICE_COMPILE__  // the host check mirrors both candidate lists (tools/accel_check.cpp)
    ws.add_cand(k, !(disc < r.negG) && k != r.skip);  // kept unless the filter proves a miss
#else
    ws.add_cand(k, !(disc < r.negG));  // kept unless the filter proves a miss
#endif
    // sure hit iff disc > d2 - 2 negG (> 0, so also kept; sd is then a real root;
    // otherwise sd and slo are unused)
    const float sd = sqrt32(disc);
    const float slo = sqrt32(fmaxf(disc - d2 + 2.f * r.negG, 0.f)) - hb;
    const float sfar = sd - hb;
    const float slack = 1.953125e-3f * (fabsf(hb) + sd);  // 2^-9
    const bool sure = disc > d2 - 2.f * r.negG && slo - slack > r.tmin * 1.001f;
    U = fminf(U, sure ? sfar + slack : U);
}

// Walk scratch: the traversal stack of 16-bit node ids (LIFO) and the candidate
// list of leaf ids, sharing kScratch slots -- the stack grows up from slot 0,
// the candidates down from the last slot. put(id, h) stores id on top and keeps
// it iff h (a write that is not kept is overwritten by the next put): the walk
// puts every child slot far to near without branching, so up to 4 slots above
// the kept entries are written. Invariant: kept + 4 + candidates <= kScratch
// (else overflow: the caller brute-forces), at most kMaxCand candidates.
// add_cand never exits the walk and never branches: the leaf id is stored in the
// unclaimed next candidate slot (always inside the column) and claimed if kept; a
// kept candidate that does not fit sets `bad`.
// next() ends the node: it records a stack overflow in `bad` and pops the next
// node unless the stack is empty or the walk has failed -- the walk's one exit.
constexpr uint32_t kScratch = 16;
// ArrayScratch (host, accel_check): a plain array.
struct ArrayScratch {
    uint16_t e[kScratch] = {};
    uint32_t sp = 0, nc = 0;
    uint32_t bad = 0;  // a u32, not a bool: no lane-mask merges in the leaf loop
    RTW_HD void put(uint32_t id, uint32_t h) {
        e[sp] = static_cast<uint16_t>(id);
        sp += h;
    }
    RTW_HD bool next(uint32_t &id) {
        bad |= sp + 4u + nc > kScratch ? 1u : 0u;
        if (bad != 0u || sp == 0) return false;
        id = e[--sp];
        return true;
    }
    RTW_HD void add_cand(uint32_t k, bool keep) {
        const bool ok = nc < kMaxCand && sp + 5u + nc <= kScratch;
        e[kScratch - 1u - nc] = static_cast<uint16_t>(k);
        nc += keep && ok ? 1u : 0u;
        bad |= keep && !ok ? 1u : 0u;
    }
    RTW_HD uint32_t cand_at(uint32_t j) const { return e[kScratch - 1u - j]; }
};
#if defined(__HIPCC__)
// LdsScratch (device): a per-lane LDS column, slot k at col[k * stride] (u16);
// kept as pointers (no multiplies on the walk): top = next stack slot, cand =
// next candidate slot, lim = the highest top that keeps 4 free slots below cand.
struct LdsScratch {
    uint16_t *base, *top, *cand, *lim;
    uint32_t stride, nc = 0;
    uint32_t bad = 0;  // a u32, not a bool: no lane-mask merges in the leaf loop
    __device__ LdsScratch(uint16_t *c, uint32_t s)
        : base(c), top(c), cand(c + (kScratch - 1u) * s), lim(c + (kScratch - 4u) * s), stride(s) {}
    __device__ void put(uint32_t id, uint32_t h) {
        *top = static_cast<uint16_t>(id);
        // h in {0, 1}: one v_mad_u32_u24 on the byte address
        top = reinterpret_cast<uint16_t *>(reinterpret_cast<char *>(top) + __umul24(h, 2u * stride));
    }
    __device__ bool next(uint32_t &id) {
        bad |= top > lim ? 1u : 0u;
        if (bad != 0u || top == base) return false;
        top -= stride;
        id = *top;
        return true;
    }
    __device__ void add_cand(uint32_t k, bool keep) {
        const bool ok = nc < kMaxCand && top < lim;
        *cand = static_cast<uint16_t>(k);  // claimed only if kept: else the next one overwrites it
        const uint32_t step = keep && ok ? 2u * stride : 0u;  // bytes
        cand = reinterpret_cast<uint16_t *>(reinterpret_cast<char *>(cand) - step);
        lim = reinterpret_cast<uint16_t *>(reinterpret_cast<char *>(lim) - step);
        nc += keep && ok ? 1u : 0u;
        bad |= keep && !ok ? 1u : 0u;
    }
    __device__ uint32_t cand_at(uint32_t j) const { return base[(kScratch - 1u - j) * stride]; }
};
#endif

// Collects the leaves (leaf-order ids) the walk cannot rule out. Each iteration
// takes one 4-wide node, tests its 4 child boxes, runs the leaf filter on hit
// leaf children, continues with the nearest hit inner child and pushes the
// other hit inner children. U (distance units along e32) is
// the running cut; the caller seeds it from the "always" spheres. Returns false
// on candidate-list or stack overflow (caller brute-forces). `visits` counts
// loop iterations (node visits).
// (The lane-compacted leaf pass -- hit leaf children listed unfiltered and filtered
// wave-wide after the walk -- measured +53 % and was removed in round 6:
// profiles/r05_misc/ab_compacted_leaf_pass_REJECTED.log, git history before it.)
template <typename F4, typename Scratch>
RTW_HD bool walk(const F4 *__restrict__ nodes, const F4 *__restrict__ leaves, const WalkRay &r,
                 float &U, uint32_t &visits, Scratch &stk) {
    const uint32_t sx = r.neg & 1u, sy = (r.neg >> 1) & 1u, sz = r.neg >> 2;
    const uint32_t oct_shift = 8u * (r.neg & 3u);
    const bool oct_hi = r.neg >= 4u;
    auto visit = [&](uint32_t cur) {
        ++visits;
#if defined(RTW_STAMPS) && defined(__HIP_DEVICE_COMPILE__)
        // diagnostic: wave-level iterations, counted by the first active lane in bit 16+
        if (__builtin_ctzll(__builtin_amdgcn_read_exec()) == static_cast<int>(__lane_id())) visits += 1u << 16;
#endif
#if defined(__HIP_DEVICE_COMPILE__)
        // byte offset by a full-rate v_mul_u32_u24 (ids < 2^16; the compiler
        // otherwise picks the quarter-rate v_mul_lo_u32)
        static_assert(kNodeF4 * 16u == 144u, "node stride");
        const uint32_t off = __umul24(cur, 144u);
        const F4 *N = reinterpret_cast<const F4 *>(reinterpret_cast<const char *>(nodes) + off);
#else
        const F4 *N = nodes + kNodeF4 * cur;
#endif
        // near / far planes picked by address (per-ray direction signs): no min/max
        const F4 nX = N[sx], fX = N[sx ^ 1u], nY = N[2u + sy], fY = N[3u - sy], nZ = N[4u + sz],
                 fZ = N[5u - sz], qc = N[6], qo = N[7];
        uint32_t hit = slab_hit4(nX, nY, nZ, fX, fY, fZ, r, U);
        const uint32_t r01 = as_u32(qc.x), r23 = as_u32(qc.y), masks = as_u32(qc.z);
        hit &= masks;
        // leaf children first: they may tighten U for the inner children
        uint32_t lmask = hit & (masks >> 4);
        const uint32_t inner = hit & ~lmask & 15u;
        const uint64_t refs = (static_cast<uint64_t>(r23) << 32) | r01;
        while (lmask) {
            const uint32_t j = static_cast<uint32_t>(__builtin_ctz(lmask));
            lmask &= lmask - 1u;
            leaf_test(leaves, static_cast<uint32_t>(refs >> (16u * j)) & 0xffffu, r, U, stk);
        }
        // hit inner children onto the stack far to near (branch-free puts), then
        // continue with the top = the nearest
        const uint32_t ord = ((oct_hi ? as_u32(qo.y) : as_u32(qo.x)) >> oct_shift) & 0xffu;
        for (int t = 3; t >= 0; --t) {
            const uint32_t j = (ord >> (2 * t)) & 3u;
#if defined(__HIP_DEVICE_COMPILE__)
            stk.put(static_cast<uint32_t>(refs >> (16u * j)), __builtin_amdgcn_ubfe(inner, j, 1u));
#else
            stk.put(static_cast<uint32_t>(refs >> (16u * j)), (inner >> j) & 1u);
#endif
        }
    };
    // (Peeling the root visit off this loop -- its loads issued without waiting for a
    // pop, one loop iteration fewer per walk -- measured +0.5 %: profiles/r03_misc/
    // ab_root_peel_REJECTED.log.)
    uint32_t cur = 0;
    for (;;) {
        visit(cur);
        if (!stk.next(cur)) break;
    }
    return stk.bad == 0u;
}

// (t, i) beats (bt, best) under the scan's first-minimum rule.
RTW_HD bool better(double t, uint32_t i, double bt, int best) {
    return best < 0 || t < bt || (t == bt && static_cast<int>(i) < best);
}

// ---- Inside cut: a segment that starts inside the sphere it last hit ----------
// Rays trapped inside a sphere (refracted into glass, or scattered inward from
// the inner face of any sphere -- the reference flips the normal, hittable.rs:
// 64-81, so a Lambertian bounce from inside stays inside) make up most of the
// heaviest pixels' segments. If sphere S's near root is rejected (t < 0.01,
// interval.rs:55-57) and its far root t_f accepted, every ray point with
// t in [0.01, t_f] lies within S (up to the roots' rounding error), so a sphere
// T can beat t_f only if it comes within that error of S. The host lists, per S,
// the spheres with gap |c_S - c_T| - |r_S| - |r_T| <= delta(S, T) (overlapping or
// nearly touching); the segment's exact result is then the (t, index) minimum
// over S and its list -- the scan's first minimum, since every other sphere's
// accepted root is strictly beyond t_f.
//
// delta: the f64 root of Sphere::hit errs in distance by at most about
// sqrt(12u)(|oc| + r) = 2^-24.5 (|oc| + r) (tangent rays: the discriminant's
// error 12u|d|^2(|oc|^2 + r^2) under the square root; u = 2^-53). The device takes
// the cut only when |o - c_S|^2 - r_S^2 <= 3 r_S^2, so |oc_S| <= 2|r_S| and
// |oc_T| <= 2|r_S| + D; delta = 2^-20 (5|r_S| + 2|r_T| + D + |c_S| + |c_T|) is
// over 20x the sum of both roots' errors.
constexpr uint32_t kNbrNone = 0xffffffffu;  // ShadeRec info word: no inside cut for this sphere
constexpr uint32_t kMaxNbr = 8;             // longer lists take the normal walk
constexpr double kNbrMargin = 9.5367431640625e-07;  // 2^-20

// Sphere::hit of sphere (c, rr) when the ray starts inside it: true iff the
// discriminant is non-negative, |oc|^2 - rr <= 3 rr, the near root is rejected
// and the far root accepted; t = the far root, computed exactly as
// sphere_hit_f64 computes it (same operations, same order).
RTW_HD bool inside_far(double ox, double oy, double oz, double dx, double dy, double dz, double a,
                       double cx, double cy, double cz, double rr, double &t) {
    const double ocx = ox - cx, ocy = oy - cy, ocz = oz - cz;
    const double hb = ocx * dx + ocy * dy + ocz * dz;
    const double c = (ocx * ocx + ocy * ocy + ocz * ocz) - rr;
    // cheap exits first: origin far out, or on/outside S heading away (hb >= 0
    // with c >= 0 puts both roots at or below ~0: the cut never applies)
    if (!(c <= 3. * rr) || (hb >= 0. && c >= 0.)) return false;
    const double disc = hb * hb - a * c;
    if (!(disc >= 0.)) return false;
    const double sq = __builtin_sqrt(disc);
    if ((-sq - hb) / a >= 0.01) return false;  // entering from outside: the normal path
    t = (sq - hb) / a;
    return t >= 0.01;
}

// ---- Trapped paths -------------------------------------------------------------
// Lambertian: a bounce off the inner face of sphere S (front_face false, so the
// reference flips the normal inward, hittable.rs:64-81) scatters along
// d = n_in + u (materials.rs:22-37, u = random_unit_vec). From a surface point
// o = c + r h0 the far root along d is exactly t = r, and the ray ends at c + r u:
// a uniformly random point of S. Unless a neighbour comes nearer, the path stays
// inside S bounce after bounce until the depth cap returns black (camera.rs:
// 381-383); only its RNG draws (random_unit_vec's rejection loop, vec3.rs:218-232,
// which does not depend on the geometry) and its segment count matter.
// Dielectric: total internal reflection inside a sphere keeps its angle (the
// chords of a sphere are isosceles), draws nothing (the reflectance draw is
// short-circuited, materials.rs:96-98) and walks a great circle of S.
// The host gives every sphere S that can trap (r >= 0.02, so chords of t = r,
// 2r or 2r cos stay far above 0.01; Lambertian albedo finite and >= +0 so the
// dropped factors of the black product change no bit) a half-space
// {(x - c).w < r cap} that keeps every chord inside S at least delta away from
// each neighbour (w = 0, cap = 1: no neighbours; cap <= -2: never). The device
// checks each chord end against it and falls back to tracing on any doubt.
struct TrapRec {
    double wx, wy, wz, cap;
};
constexpr double kTrapNever = -3.;

// Host: per sphere the info word (offset << 8 | count into `ids`, or kNbrNone)
// of its inside-cut list; with `trap_ok` (per sphere: may trap) also its TrapRec.
// Scenes with a non-finite sphere get no cuts and no traps.
void build_inside(const double *centers, const double *radii, uint32_t n, std::vector<uint32_t> &info,
                  std::vector<uint16_t> &ids, const uint8_t *trap_ok = nullptr,
                  std::vector<TrapRec> *trap = nullptr);

// ---- host only (declared in both compilation passes, defined for the host) ----
// R2' of the pass-1 record of a sphere (center c, r*r = rr); +inf (always tested
// exactly) outside the guard or for non-finite input.
inline float filter_r2p(const double *c, double rr) {
    const double mc = std::fmax(std::fmax(std::fabs(c[0]), std::fabs(c[1])), std::fabs(c[2]));
    if (!(mc <= kGuardHi) || !std::isfinite(rr)) return INFINITY;
    const double x = rr + kFilterK * (mc * mc + rr / 2.) * (1. + 1e-6);
    if (!(x >= 0.) || !(x <= 1e36)) return INFINITY;
    return std::nextafter(static_cast<float>(x), INFINITY);
}

// Host builder (rtw_accel_build.cpp). Spheres as centers (3n f64) and radii;
// r2p = the pass-1 filter's R2' per sphere (the same records the brute-force
// filter uses). Returns false if the scene is not eligible (n > kMaxSpheres or
// too many "always" spheres): the kernel then scans by brute force.
struct Bvh {
    uint32_t n_node = 0, n_leaf = 0, depth = 0;
    std::vector<float> nodes;      // kNodeFloats per 4-wide node (eight float4 + pad)
    std::vector<float> leaves;     // 8 floats per leaf (two float4)
    std::vector<uint32_t> always;  // sphere indices tested exactly first, ascending
};
bool build(const double *centers, const double *radii, const float *r2p, uint32_t n, Bvh &out);

}  // namespace rtw_accel
