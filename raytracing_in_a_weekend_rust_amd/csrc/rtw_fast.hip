// rtw_fast.hip -- f32 fast mode of the sampling path (rtw_fast.h).
//
// Same model as the parity kernel (rtw_render.hip): get_ray with the stratified
// lattice and the defocus disk (camera.rs:400-456), Scene::hit's closest sphere
// from t = 0.01 (hittable.rs:131-143, sphere.rs:39-71, camera.rs:387), the three
// materials with the reference's quirks (materials.rs:22-111: Lambertian's
// near_zero without abs, vec3.rs:246-250; Metal always scatters and always draws;
// Dielectric draws only when it can refract), black at the depth cap, the sky
// gradient on a miss (camera.rs:376-398). Differences, by design:
//   * f32 arithmetic (FMA allowed) instead of f64, so paths diverge from the
//     reference after a few bounces and the gate is statistical;
//   * random numbers: xoroshiro64** (Blackman & Vigna), one stream per
//     (global pixel, lattice sample) seeded by SplitMix64's finaliser, instead of
//     one XorShift chain per pixel (random.rs:33-69). A pixel's samples are
//     independent, so one wave traces 64 of them at once;
//   * random_unit_vec and the unit-disk sample draw their distributions directly
//     (no rejection loop, whose retries diverge across a wave);
//   * the pixel mean is summed in 32.32 fixed point (LDS u64 atomics): exact and
//     order-free, so a render is deterministic and any shard reproduces the
//     unsharded pixels bit-for-bit. Per-sample colours are clamped to [0, cmax]
//     (NaN -> 0) to keep the sum in range; the reference's scenes stay in [0, 1].
//
// Execution: a persistent grid (two 512-thread workgroups per CU, scene tables +
// BVH in LDS). Each wave takes pixels from a global counter and keeps a ring of
// up to kRing pixels in flight: a lane whose path ends starts the next sample of
// the newest pixel at once, so lanes stay busy until the image runs out. A pixel
// is written when all its samples are handed out and finished.
#include "rtw_fast.h"

#include <cstdlib>

#include "rtw_accel.h"
#include "rtw_capi.h"

namespace rtw_fast {
namespace {

constexpr uint32_t kWaves = kBlock / 64;
constexpr uint32_t kRing = 4;
constexpr uint32_t kFree = 0xffffffffu;

struct Rng {
    uint32_t a, b;
};

__device__ __forceinline__ uint64_t fmix64(uint64_t z) {  // SplitMix64's finaliser
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ Rng rng_for(uint64_t mix, uint64_t pix, uint32_t k) {
    const uint64_t z = fmix64(fmix64(mix ^ (pix * 0x9e3779b97f4a7c15ull)) + k);
    Rng r{static_cast<uint32_t>(z), static_cast<uint32_t>(z >> 32)};
    if ((r.a | r.b) == 0u) r.a = 1u;
    return r;
}
// xoroshiro64**
__device__ __forceinline__ uint32_t rnext(Rng &r) {
    const uint32_t s0 = r.a;
    uint32_t s1 = r.b;
    const uint32_t res = __builtin_rotateleft32(s0 * 0x9E3779BBu, 5) * 5u;
    s1 ^= s0;
    r.a = __builtin_rotateleft32(s0, 26) ^ s1 ^ (s1 << 9);
    r.b = __builtin_rotateleft32(s1, 13);
    return res;
}
// next_bound(-1, 1) (random.rs:54-59) on a 24-bit uniform; next_01 (40-52)
__device__ __forceinline__ float rcoord(Rng &r) {
    return fmaf(static_cast<float>(rnext(r) >> 8), 1.1920928955078125e-07f, -1.f);  // 2^-23
}
__device__ __forceinline__ float r01(Rng &r) {
    return static_cast<float>(rnext(r) >> 8) * 5.9604644775390625e-08f;  // 2^-24
}
// random_unit_vec (vec3.rs:219-232) draws uniformly on the unit sphere by rejection;
// fast mode draws the same distribution directly (z uniform in [-1, 1], azimuth
// uniform: Archimedes), with no divergent retry loop. v_sin/v_cos take revolutions.
__device__ __forceinline__ void unit_vec(Rng &r, float &x, float &y, float &z) {
    z = rcoord(r);
    const float t = r01(r);
    const float s = __builtin_sqrtf(fmaxf(fmaf(-z, z, 1.f), 0.f));
    x = s * __builtin_amdgcn_cosf(t), y = s * __builtin_amdgcn_sinf(t);
}
// random_vec_in_unit_disk (vec3.rs:270-277), uniform in the open disk, directly
__device__ __forceinline__ void disk_vec(Rng &r, float &x, float &y) {
    const float rad = __builtin_sqrtf(r01(r)), t = r01(r);
    x = rad * __builtin_amdgcn_cosf(t), y = rad * __builtin_amdgcn_sinf(t);
}

// A segment: origin, unit direction, t_min = 0.01 |d| in distance units.
struct Seg {
    float ox, oy, oz, ex, ey, ez, tmin;
};

// Sphere::hit (sphere.rs:39-71) in distance units along the unit direction, with
// the discriminant from the closest-approach vector (r^2 - |oc - hb e|^2: no
// cancellation against |oc|^2 for big spheres) and the stable root pair.
__device__ __forceinline__ void sphere_test(const float4 S, int i, const Seg &g, float &best, int &hid) {
    const float ocx = g.ox - S.x, ocy = g.oy - S.y, ocz = g.oz - S.z;
    const float hb = fmaf(ocx, g.ex, fmaf(ocy, g.ey, ocz * g.ez));
    const float lx = fmaf(-hb, g.ex, ocx), ly = fmaf(-hb, g.ey, ocy), lz = fmaf(-hb, g.ez, ocz);
    const float rr = S.w * S.w;
    const float disc = rr - fmaf(lx, lx, fmaf(ly, ly, lz * lz));
    if (!(disc >= 0.f)) return;
    const float sq = __builtin_sqrtf(disc);
    const float c = fmaf(ocx, ocx, fmaf(ocy, ocy, fmaf(ocz, ocz, -rr)));
    const float q = -hb - copysignf(sq, hb);
    const float t0 = c * __builtin_amdgcn_rcpf(q), t1 = q;
    const float tn = fminf(t0, t1), tf = fmaxf(t0, t1);
    const float t = tn >= g.tmin ? tn : tf;
    if (t >= g.tmin && t < best) best = t, hid = i;
}

// Per-segment slab setup for the 4-wide BVH of rtw_accel.h (its boxes are
// padded for the parity walk; that padding only adds a few box hits here).
__device__ __forceinline__ void walk_ray(const Seg &g, rtw_accel::WalkRay &r) {
    using namespace rtw_accel;
    const float mo = fmax3(fabsf(g.ox), fabsf(g.oy), fabsf(g.oz));
    r.ox = g.ox, r.oy = g.oy, r.oz = g.oz, r.ex = g.ex, r.ey = g.ey, r.ez = g.ez;
    r.neg = (g.ex < 0.f ? 1u : 0u) | (g.ey < 0.f ? 2u : 0u) | (g.ez < 0.f ? 4u : 0u);
    r.ix = rcp32(clamp_dir(g.ex)), r.iy = rcp32(clamp_dir(g.ey)), r.iz = rcp32(clamp_dir(g.ez));
    const float pad = kPadK * mo + 1e-30f;
    const float alx = -(g.ox + pad) * r.ix, ahx = -(g.ox - pad) * r.ix;
    const float aly = -(g.oy + pad) * r.iy, ahy = -(g.oy - pad) * r.iy;
    const float alz = -(g.oz + pad) * r.iz, ahz = -(g.oz - pad) * r.iz;
    const bool nx = r.neg & 1u, ny = r.neg & 2u, nz = r.neg & 4u;
    r.anx = nx ? ahx : alx, r.afx = nx ? alx : ahx;
    r.any = ny ? ahy : aly, r.afy = ny ? aly : ahy;
    r.anz = nz ? ahz : alz, r.afz = nz ? alz : ahz;
    r.tmin = g.tmin * 0.999f;
    r.negG = 0.f;
}

// Closest hit: the "always" spheres, then the BVH walk testing leaf spheres as
// they are reached (the running best is the walk's cut), or a linear scan.
__device__ __forceinline__ void scene_hit(const FastParams &P, const float4 *__restrict__ geo,
                                          const float4 *__restrict__ nodes, const Seg &g, float &best,
                                          int &hid, uint16_t *stk, uint32_t &visits, uint32_t &wvisits) {
    best = INFINITY, hid = -1;
    if (P.n_node == 0) {
        for (uint32_t i = 0; i < P.n_sph; ++i) sphere_test(geo[i], static_cast<int>(i), g, best, hid);
        return;
    }
    for (uint32_t a = 0; a < P.n_always; ++a) {
        const uint32_t i = P.always[a];
        sphere_test(geo[i], static_cast<int>(i), g, best, hid);
    }
    if (!(rtw_accel::fmax3(fabsf(g.ox), fabsf(g.oy), fabsf(g.oz)) <= rtw_accel::kGuardBvh)) {
        for (uint32_t i = 0; i < P.n_sph; ++i) sphere_test(geo[i], static_cast<int>(i), g, best, hid);
        return;
    }
    rtw_accel::WalkRay r;
    walk_ray(g, r);
    const uint32_t sx = r.neg & 1u, sy = (r.neg >> 1) & 1u, sz = r.neg >> 2;
    const uint32_t oct_shift = 8u * (r.neg & 3u);
    const bool oct_hi = r.neg >= 4u;
    uint16_t *top = stk;
    uint32_t cur = 0;
    for (;;) {
        ++visits;
#ifdef RTW_FAST_DIAG
        // wave-level walk iterations, counted by the first active lane (diagnostic
        // builds: the count costs 2%; 9.4 per wave-iteration against 5.4 visits per lane)
        if (static_cast<int>(__lane_id()) == __builtin_ctzll(__builtin_amdgcn_read_exec())) ++wvisits;
#endif
        uint32_t off;
        asm("v_mul_u32_u24 %0, 0x90, %1" : "=v"(off) : "v"(cur));
        const float4 *N = reinterpret_cast<const float4 *>(reinterpret_cast<const char *>(nodes) + off);
        const float4 nX = N[sx], fX = N[sx ^ 1u], nY = N[2u + sy], fY = N[3u - sy], nZ = N[4u + sz],
                     fZ = N[5u - sz], qc = N[6], qo = N[7];
        uint32_t hit = 0;
        hit |= rtw_accel::slab_hit4(nX, nY, nZ, fX, fY, fZ, r, best);
        const uint32_t r01w = rtw_accel::as_u32(qc.x), r23w = rtw_accel::as_u32(qc.y);
        const uint32_t masks = rtw_accel::as_u32(qc.z);
        hit &= masks;
        uint32_t lmask = hit & (masks >> 4);
        const uint32_t inner = hit & ~lmask & 15u;
        while (lmask) {
            const uint32_t j = static_cast<uint32_t>(__builtin_ctz(lmask));
            lmask &= lmask - 1u;
            const uint32_t k = ((j & 2u ? r23w : r01w) >> (16u * (j & 1u))) & 0xffffu;
            sphere_test(geo[k], static_cast<int>(k), g, best, hid);
        }
        const uint32_t ord = ((oct_hi ? rtw_accel::as_u32(qo.y) : rtw_accel::as_u32(qo.x)) >> oct_shift) & 0xffu;
        const uint64_t refs = (static_cast<uint64_t>(r23w) << 32) | r01w;
        for (int t = 3; t >= 0; --t) {  // far to near: the nearest ends on top
            const uint32_t j = (ord >> (2 * t)) & 3u;
            *top = static_cast<uint16_t>(refs >> (16u * j));
            top += __builtin_amdgcn_ubfe(inner, j, 1u) * kBlock;
        }
        if (top == stk) break;
        top -= kBlock;
        cur = *top;
    }
}

template <bool kLds>
__global__ __launch_bounds__(kBlock, 2) void rtw_fast_render(const FastParams P) {
    extern __shared__ __attribute__((aligned(16))) float4 lds[];
    __shared__ unsigned long long acc[kWaves][kRing][3];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    // per-lane stack column: slot j at stk[j * kBlock]
    uint16_t *stk = reinterpret_cast<uint16_t *>(lds) + tid;
    const float4 *geo = P.geo, *mat = P.mat, *nodes = P.nodes;
    const uint32_t *kind = P.kind;
    if constexpr (kLds) {
        float4 *g = lds + P.n_stack * kBlock * sizeof(uint16_t) / sizeof(float4);
        float4 *m = g + P.n_sph, *nd = m + P.n_sph;
        uint32_t *kd = reinterpret_cast<uint32_t *>(nd + P.n_node * rtw_accel::kNodeF4);
        for (uint32_t i = tid; i < P.n_sph; i += kBlock) g[i] = P.geo[i], m[i] = P.mat[i], kd[i] = P.kind[i];
        for (uint32_t i = tid; i < P.n_node * rtw_accel::kNodeF4; i += kBlock) nd[i] = P.nodes[i];
        geo = g, mat = m, nodes = nd, kind = kd;
        __syncthreads();
    }
    const uint32_t npix = P.n_rows * P.W;
    const float cmax = P.cmax;
    // wave-uniform ring state
    uint32_t pixs[kRing], outst[kRing];
#pragma unroll
    for (uint32_t s = 0; s < kRing; ++s) pixs[s] = kFree, outst[s] = 0;
    uint32_t cs = kFree, cur_pix = 0, next = 0;
    bool exhausted = false;
    // lane path state
    Seg g{};
    float tr = 0.f, tg = 0.f, tb = 0.f;
    uint32_t depth = 0, slot = kFree;
    Rng rng{1u, 0u};
    uint32_t segs = 0, visits = 0, written = 0, iters = 0, wvisits = 0;
    for (;;) {
        // ---- hand out samples of the newest pixel to idle lanes
        for (;;) {
            const uint64_t need = __ballot(slot == kFree);
            if (need == 0) break;
            if (cs == kFree || next >= P.n_off) {
                if (exhausted) break;
                uint32_t f = kFree;
#pragma unroll
                for (uint32_t s = 0; s < kRing; ++s)
                    if (f == kFree && pixs[s] == kFree) f = s;
                if (f == kFree) break;
                uint32_t p = 0;
                if (lane == 0) p = atomicAdd(P.cursor, 1u);
                p = __builtin_amdgcn_readfirstlane(p);
                if (p >= npix) {
                    exhausted = true;
                    break;
                }
#pragma unroll
                for (uint32_t s = 0; s < kRing; ++s)
                    if (s == f) pixs[s] = p, outst[s] = 0;
                if (lane < 3) acc[wave][f][lane] = 0ull;
                __builtin_amdgcn_wave_barrier();
                cs = f, cur_pix = p, next = 0;
            }
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(need >> 32),
                                                            __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(need), 0u));
            const uint32_t avail = P.n_off - next;
            if (slot == kFree && rank < avail) {
                // get_ray (camera.rs:400-420) for lattice sample k of pixel cur_pix
                const uint32_t k = next + rank;
                const uint32_t lr = cur_pix / P.W, x = cur_pix - lr * P.W;
                const uint32_t y = P.row_begin + lr * P.row_step;
                rng = rng_for(P.seed_mix, static_cast<uint64_t>(y) * P.W + x, k);
                const float fx = static_cast<float>(x), fy = static_cast<float>(y);
                float sx = fmaf(P.dv[0], fy, fmaf(P.du[0], fx, P.p00[0]));
                float sy = fmaf(P.dv[1], fy, fmaf(P.du[1], fx, P.p00[1]));
                float sz = fmaf(P.dv[2], fy, fmaf(P.du[2], fx, P.p00[2]));
                if (P.s == 0) {
                    sx += P.pos0[0], sy += P.pos0[1], sz += P.pos0[2];
                } else {
                    const uint32_t ly = k / P.s, lx = k - ly * P.s;
                    const float fly = static_cast<float>(ly), flx = static_cast<float>(lx);
                    sx += fmaf(P.ldx[0], flx, fmaf(P.ldy[0], fly, P.pos0[0]));
                    sy += fmaf(P.ldx[1], flx, fmaf(P.ldy[1], fly, P.pos0[1]));
                    sz += fmaf(P.ldx[2], flx, fmaf(P.ldy[2], fly, P.pos0[2]));
                }
                g.ox = P.from[0], g.oy = P.from[1], g.oz = P.from[2];
                if (P.defocus) {  // defocus_disk_sample (camera.rs:452-456)
                    float px, py;
                    disk_vec(rng, px, py);
                    g.ox = fmaf(P.ddv[0], py, fmaf(P.ddu[0], px, g.ox));
                    g.oy = fmaf(P.ddv[1], py, fmaf(P.ddu[1], px, g.oy));
                    g.oz = fmaf(P.ddv[2], py, fmaf(P.ddu[2], px, g.oz));
                }
                const float dx = sx - g.ox, dy = sy - g.oy, dz = sz - g.oz;
                const float sa = __builtin_sqrtf(fmaf(dx, dx, fmaf(dy, dy, dz * dz)));
                const float inv = __builtin_amdgcn_rcpf(sa);
                g.ex = dx * inv, g.ey = dy * inv, g.ez = dz * inv, g.tmin = 0.01f * sa;
                tr = tg = tb = 1.f;
                depth = 0;
                slot = cs;
            }
            const uint32_t took = min(static_cast<uint32_t>(__builtin_popcountll(need)), avail);
            next += took;
#pragma unroll
            for (uint32_t s = 0; s < kRing; ++s)
                if (s == cs) outst[s] += took;
        }
        if (__ballot(slot != kFree) == 0) break;  // nothing handed out: the image is done
        ++iters;

        // ---- one segment per busy lane (camera.rs:376-398)
        bool fin = false;
        float cr = 0.f, cg = 0.f, cb = 0.f;
        if (slot != kFree) {
            if (depth >= P.max_depth) {
                fin = true;  // black at the depth cap
            } else {
                float best;
                int hid;
                ++segs;
                scene_hit(P, geo, nodes, g, best, hid, stk, visits, wvisits);
                if (hid < 0) {
                    const float a = 0.5f * (g.ey + 1.f);  // sky (camera.rs:392-396)
                    cr = tr * ((1.f - a) + a * 0.5f), cg = tg * ((1.f - a) + a * 0.7f), cb = tb;
                    fin = true;
                } else {
                    const float4 S = geo[hid], M = mat[hid];
                    const uint32_t kd = kind[hid];
                    const float px = fmaf(best, g.ex, g.ox), py = fmaf(best, g.ey, g.oy), pz = fmaf(best, g.ez, g.oz);
                    const float ir = __builtin_amdgcn_rcpf(S.w);
                    float nx = (px - S.x) * ir, ny = (py - S.y) * ir, nz = (pz - S.z) * ir;
                    const bool front = fmaf(g.ex, nx, fmaf(g.ey, ny, g.ez * nz)) < 0.f;  // hittable.rs:64-81
                    if (!front) nx = -nx, ny = -ny, nz = -nz;
                    const float en = fmaf(g.ex, nx, fmaf(g.ey, ny, g.ez * nz));
                    // reflect(unit(dir), n) (vec3.rs:252-257)
                    const float rx = fmaf(-2.f * en, nx, g.ex), ry = fmaf(-2.f * en, ny, g.ey),
                                rz = fmaf(-2.f * en, nz, g.ez);
                    float dx, dy, dz;
                    if (kd != RTW_DIELECTRIC) {
                        float ux, uy, uz;
                        unit_vec(rng, ux, uy, uz);
                        if (kd == RTW_LAMBERTIAN) {  // materials.rs:22-37, near_zero without abs
                            dx = nx + ux, dy = ny + uy, dz = nz + uz;
                            if (dx < 1e-8f && dy < 1e-8f && dz < 1e-8f) dx = nx, dy = ny, dz = nz;
                        } else {  // Metal, materials.rs:52-63
                            dx = fmaf(M.w, ux, rx), dy = fmaf(M.w, uy, ry), dz = fmaf(M.w, uz, rz);
                        }
                        tr *= M.x, tg *= M.y, tb *= M.z;
                    } else {  // Dielectric, materials.rs:83-111
                        const float ratio = front ? M.x : M.y;
                        const float cth = fminf(-en, 1.f);
                        const float sth = __builtin_sqrtf(fmaxf(1.f - cth * cth, 0.f));
                        bool refl = ratio * sth > 1.f;
                        if (!refl) {
                            const float x = 1.f - cth;
                            const float r = M.z + (1.f - M.z) * (x * ((x * x) * (x * x)));
                            refl = r > r01(rng);
                        }
                        if (refl) {
                            dx = rx, dy = ry, dz = rz;
                        } else {  // refract (vec3.rs:259-268)
                            const float qx = ratio * fmaf(cth, nx, g.ex), qy = ratio * fmaf(cth, ny, g.ey),
                                        qz = ratio * fmaf(cth, nz, g.ez);
                            const float par = -__builtin_sqrtf(fabsf(1.f - fmaf(qx, qx, fmaf(qy, qy, qz * qz))));
                            dx = fmaf(par, nx, qx), dy = fmaf(par, ny, qy), dz = fmaf(par, nz, qz);
                        }
                    }
                    const float sa = __builtin_sqrtf(fmaf(dx, dx, fmaf(dy, dy, dz * dz)));
                    const float inv = __builtin_amdgcn_rcpf(sa);
                    g.ox = px, g.oy = py, g.oz = pz;
                    g.ex = dx * inv, g.ey = dy * inv, g.ez = dz * inv, g.tmin = 0.01f * sa;
                    ++depth;
                }
            }
        }
        // ---- finished samples into their pixel's fixed-point sum
        if (fin) {
            const float sc = 4294967296.f;  // 2^32
            const unsigned long long vr = static_cast<unsigned long long>(fminf(fmaxf(cr, 0.f), cmax) * sc);
            const unsigned long long vg = static_cast<unsigned long long>(fminf(fmaxf(cg, 0.f), cmax) * sc);
            const unsigned long long vb = static_cast<unsigned long long>(fminf(fmaxf(cb, 0.f), cmax) * sc);
            unsigned long long *a = acc[wave][slot];
            atomicAdd(a + 0, vr);
            atomicAdd(a + 1, vg);
            atomicAdd(a + 2, vb);
        }
#pragma unroll
        for (uint32_t s = 0; s < kRing; ++s) outst[s] -= static_cast<uint32_t>(__builtin_popcountll(__ballot(fin && slot == s)));
        if (fin) slot = kFree;
        // ---- pixels whose samples are all handed out and finished
#pragma unroll
        for (uint32_t s = 0; s < kRing; ++s) {
            if (pixs[s] != kFree && outst[s] == 0 && (s != cs || next >= P.n_off)) {
                __builtin_amdgcn_wave_barrier();
                if (lane < 3) {
                    const double v = static_cast<double>(acc[wave][s][lane]) * (1. / 4294967296.) /
                                     static_cast<double>(P.n_off);
                    P.out[static_cast<uint64_t>(pixs[s]) * 3u + lane] = static_cast<float>(v);
                }
                pixs[s] = kFree;
                ++written;
                if (s == cs) cs = kFree;
            }
        }
    }
    // statistics: one atomic per wave
    unsigned long long sg = segs, vs = visits, wv = wvisits;
    for (int o = 32; o > 0; o >>= 1) {
        sg += __shfl_xor(sg, o);
        vs += __shfl_xor(vs, o);
        wv += __shfl_xor(wv, o);
    }
    if (lane == 0) {
        atomicAdd(P.counters + 0, sg);
        atomicAdd(P.counters + 1, vs);
        atomicAdd(P.counters + 2, static_cast<unsigned long long>(written));
        atomicAdd(P.counters + 3, static_cast<unsigned long long>(iters));
        atomicAdd(P.counters + 4, wv);
    }
}

}  // namespace

size_t lds_bytes(uint32_t n_sph, uint32_t n_node, uint32_t n_stack, bool *scene_in_lds) {
    const size_t stacks = static_cast<size_t>(n_stack) * kBlock * sizeof(uint16_t);
    const size_t scene = static_cast<size_t>(n_sph) * (2 * sizeof(float4) + sizeof(uint32_t)) +
                         static_cast<size_t>(n_node) * rtw_accel::kNodeF4 * sizeof(float4);
    *scene_in_lds = stacks + scene <= kLdsCap;
    return *scene_in_lds ? stacks + scene : (stacks ? stacks : 16);
}

hipError_t launch(const FastParams &P, int n_cu, hipStream_t st, bool scene_lds) {
    hipError_t e = hipMemsetAsync(P.cursor, 0, sizeof(uint32_t), st);
    if (e == hipSuccess) e = hipMemsetAsync(P.counters, 0, 5 * sizeof(unsigned long long), st);
    if (e != hipSuccess) return e;
    if (P.n_rows == 0 || P.W == 0) return hipSuccess;
    const uint64_t npix = static_cast<uint64_t>(P.n_rows) * P.W;
    const uint32_t blocks = static_cast<uint32_t>(std::min<uint64_t>(
        static_cast<uint64_t>(n_cu > 0 ? n_cu : 256) * 2, (npix + kWaves - 1) / kWaves));
    bool in_lds = false;
    size_t lds = lds_bytes(P.n_sph, P.n_node, P.n_stack, &in_lds);
    if (!scene_lds && in_lds) {  // A/B: RTW_FAST_LDS=0 under RTW_AB (the scene read from HBM)
        in_lds = false;
        lds = P.n_stack ? static_cast<size_t>(P.n_stack) * kBlock * sizeof(uint16_t) : 16;
    }
    if (in_lds) hipLaunchKernelGGL(rtw_fast_render<true>, dim3(blocks), dim3(kBlock), lds, st, P);
    else hipLaunchKernelGGL(rtw_fast_render<false>, dim3(blocks), dim3(kBlock), lds, st, P);
    return hipGetLastError();
}

}  // namespace rtw_fast
