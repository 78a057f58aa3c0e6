// rtw_render.hip -- CDNA4 (gfx950) path-tracing megakernel for the reference's
// per-pixel sampling hot path, plus the device half of the C ABI.
//
// Replaces Camera::threaded_render's per-pixel job loop (camera.rs:269-292),
// ray_colors_lattice (354-374), the ray_color recursion (376-398), get_ray /
// offset_lattice / defocus_disk_sample (400-456), Scene::hit (hittable.rs:131-143),
// Sphere::hit (sphere.rs:39-71) and the three Material::scatter impls
// (materials.rs:22-111).
//
// Parity mode (the only mode in this build): f64 everywhere, compiled with
// -ffp-contract=off so no a*b+c is fused; every expression is evaluated in the
// reference's order, division and sqrt are IEEE (checked on the box by
// rtw_probe_f64_ops). The RNG is the reference's u128 xorshift(23,17,26), bit-exact.
//
// Launches per render: rtw_seed_pixels (per-pixel RNG children by
// GF(2) jump-ahead), the cost probe + 6 small kernels that order the pixels by
// estimated cost, then rtw_render_persist -- the hot path. One 768-thread workgroup
// per CU stages the scene in LDS once (BVH nodes + leaves, f64 sphere records,
// shading records, pass-1 filter records) and keeps per-lane areas there (pixel
// sum, walk scratch, speculative RNG state). Cursor waves run one pixel per lane
// and refill idle lanes from a global cursor in cost order; a lane runs one
// segment per wave iteration: Scene::hit by the exact-result 4-wide BVH
// (rtw_accel.h), the scatter, and ONE rejection loop for every lane's draws.
// Pixels whose serial sample chain runs long park at a sample boundary in a
// write-through queue and are finished by whole waves (priority waves, then every
// wave once the cursor is dry). The ray_color product att0*(att1*(...*leaf)) is
// formed right-to-left from a per-path stack of sphere indices, so it associates
// exactly as the recursion. rtw_park_leftover finishes any parked pixel nobody
// claimed.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <exception>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "rtw_accel.h"
#include "rtw_capi.h"
#include "rtw_fast.h"
#include "rtw_numeric.h"
#include "host/rtw_host.h"
#include "host/rtw_internal.h"

namespace {

constexpr int kBlock = 256;  // 16 x 16 pixel tile, 4 waves
// persistent phase 1: one workgroup per CU shares one LDS copy of the scene;
// 768 threads = 3 waves per SIMD at the BVH kernel's ~150 VGPRs. (A 1024-thread
// build fits 128 VGPRs with the per-lane LDS areas and few spills, but measured
// slower: bulk throughput no better, drain groups slower.)
constexpr int kPBlock = 768;
constexpr int kChunk = 32;                // spheres per candidate mask (one bit per sphere)
constexpr int kGroup = 8;                 // spheres per scalar-load group (8 x 16 B in SGPRs)
constexpr size_t kLdsCap = 160 * 1024;    // dynamic LDS per workgroup (gfx950: 160 KiB)
constexpr int kCounters = 20;  // [11..19]: RTW_WALK_DIAG builds only
// park a pixel past this many segments x samples per pixel (10 -> 14 in round 2: the
// faster kernel leaves fewer pixels worth a whole drain wave; 12-17 all 151.4-151.5 ms
// vs 153.2 ms at 10, interleaved A/B, profiles/r02_misc/knobs_budget.log)
constexpr double kBudgetX = 14.0;
// dry-cursor parking: estimated segments left (RTW_TAIL), per lattice sample of the
// pixel: 768 at 529 spp (tuned there); 145 at 100 spp and 2940 at 2025 spp measured
// better than a fixed 768 (38.1 -> 36.1 ms; 1026 -> 864 ms per rank of 8 at 4096x2304)
constexpr double kTailSegsPerSample = 768. / 529.;
#ifndef RTW_WALK_PRIO
#define RTW_WALK_PRIO 1  // cursor waves' issue priority through Scene::hit (0: no change)
#endif
constexpr int kWalkPrio = RTW_WALK_PRIO;
constexpr uint32_t kHeavyPerBlock = 2;  // priority waves per persistent workgroup (parked pixels)
constexpr uint32_t kHeavyPerBlockFull = 6;  // ... in a shard of about one pixel per lane
constexpr uint32_t kHeavyPerBlockFullShort = 4;  // ... of fewer than 400 samples per pixel
constexpr uint32_t kSmallShardPrepark = 16; // small shards: probe segments (2 samples) that park a
                                            // pixel before its first sample
constexpr double kJoinPct = 35.;        // ... which join the cursor after this % of the pixels
constexpr uint32_t kEndgameMinSamples = 4;  // endgame parking: only pixels with this many samples left
constexpr uint32_t kPrioSplit8 = 20u * 8u;  // drains of pixels above 20 segments/sample keep the raised
                                            // priority (x 8: Parked::_pad's fixed point)
#ifndef RTW_ENDGAME_POLL
#define RTW_ENDGAME_POLL 16
#endif
constexpr uint32_t kEndgamePoll = RTW_ENDGAME_POLL;  // cursor iterations per endgame poll (a power of 2)
static_assert((kEndgamePoll & (kEndgamePoll - 1u)) == 0u, "kEndgamePoll: a power of two");

// Scene::hit strategies (one kernel instantiation each)
constexpr int kScanF64 = 0;  // the reference's scan, f64 only
constexpr int kScanF32 = 1;  // scan behind the exact-conservative f32 filter
constexpr int kBvh = 2;      // rtw_accel.h walk + exact candidates (+ scan fallback)

using rtw_accel::kFilterK;
using rtw_accel::kGuardHi;

// Wave-uniform load of a pass-1 record through the constant address space, so the
// compiler emits s_load (4 records per s_load_dwordx16) and feeds SGPR operands.
__device__ __forceinline__ float4 ld_filt(const float4 *p, uint32_t i) {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef const __attribute__((address_space(4))) float cfloat;
    const cfloat *q = (const cfloat *)(p);
    return make_float4(q[4 * i], q[4 * i + 1], q[4 * i + 2], q[4 * i + 3]);
#else
    return p[i];
#endif
}
__device__ __forceinline__ uint32_t ld_const_u32(const uint32_t *p, uint32_t i) {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef const __attribute__((address_space(4))) uint32_t cu32;
    return ((const cu32 *)(p))[i];
#else
    return p[i];
#endif
}

struct U128 {
    uint64_t lo, hi;
};

// Global words shared across workgroups (and so across XCDs, whose L2s are not
// coherent with each other) are accessed as agent-scope atomics: sc1 loads and
// write-through stores.
typedef __attribute__((address_space(1))) uint32_t gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;

// Per-sphere shading record (40 B): the sphere's material row flattened
// (materials.rs:11-111): albedo, p = fuzz (Metal) or ir (Dielectric); nbr = the
// sphere's inside-cut list (offset << 8 | count into KParams::nbr, or
// rtw_accel::kNbrNone; rtw_accel.h "Inside cut"). The radius is the sphere
// record's w (KParams::sph).
struct ShadeRec {
    double a0, a1, a2, p;
    uint32_t kind, nbr;
};

struct KParams {
    double p00[3], du[3], dv[3], from[3], ddu[3], ddv[3];
    double lat_dx[3], lat_dy[3], lat_pos0[3];  // lattice step (delta_v/s, delta_u/s) and pos0
    double defocus_angle;
    uint32_t W, s, n_off, max_depth;
    uint32_t row_begin, row_step, n_rows, n_sph;
    uint32_t jump_bits;
    uint32_t att_finite;        // every Lambertian / Metal albedo is finite: a black leaf (depth
                                // cap) makes the sample's product +-0, an exact no-op in the sum
    uint32_t n_node, n_leaf, n_always, seg_budget;
    uint32_t order, heavy_per_block;
    uint32_t rate_k, rate_x;    // park a cursor pixel after rate_k samples above rate_x seg/sample
    uint32_t tail_segs;         // once the cursor is dry: park pixels with more estimated work left
    uint32_t join_at;           // priority waves join the cursor once it has handed out this many
                                // pixels and the park queue is idle (0xffffffff: never)
    uint32_t n_cursor_waves, lane_lds_off;  // persistent kernel: byte offset of the per-lane LDS areas
    uint32_t n_nbr;             // inside-cut list entries
    uint32_t s_magic;           // ceil(2^32 / s) for k / s by a multiply-high (s <= 1625), else 0
    uint32_t endgame;           // dry cursor and at most this many pixels unfinished: park at the
                                // next sample boundary (0: off)
    uint32_t probe_sub;         // cost probe on every probe_sub-th pixel of every probe_sub-th row
    uint32_t probe_cap;         // cost probe: segments traced per probe sample at most
    uint32_t hot_segs;          // cost probe: a pixel with >= hot_segs probe segments is ordered alone
    uint32_t drain_off;         // tests (RTW_DRAIN_OFF=1): the persistent kernel drains no parked
                                // pixel; the leftover launch finishes them all
    uint32_t drain_prio;        // draining waves' issue priority after the cursor phase (RTW_DRAIN_PRIO,
                                // default 3; 0: unchanged)
    uint32_t heavy_prio;        // priority waves' issue priority while they drain (RTW_HEAVY_PRIO, default 3)
    uint32_t prio_split;        // > 0 (RTW_PRIO_SPLIT, segments per sample x 8): a drained pixel below
                                // it drains at priority 0, the others at the drain priority
    uint32_t wave_cap;          // > 0 (RTW_WAVE_CAP, A/B): a cursor wave holds at most wave_cap pixels
    uint32_t spread_q;          // > 0: hand-out ticket t < 64 q takes order position (t % 64) q + t / 64,
                                // so a wave's 64 lanes get pixels from across the cost order
                                // (RTW_SPREAD; 0: position t)
    uint32_t prepark;           // cost-ordered hand-out: a pixel whose probe traced >= prepark
                                // segments is parked before its first sample (0: off)
    uint64_t seed_lo, seed_hi;
    const double4 *sph;         // {cx, cy, cz, r} f64 (the reference's values; r*r formed at each
                                // use, as sphere.rs:49 does)
    const float4 *filt;         // {cx, cy, cz, R2'} f32, padded to kChunk (pass 1 only)
    const float4 *nodes;        // BVH inner nodes, 2 float4 each (rtw_accel.h)
    const float4 *leaves;       // BVH leaves, 2 float4 each
    const uint32_t *always;     // spheres tested exactly before the walk
    const ShadeRec *shade;      // per-sphere radius + material
    const uint16_t *nbr;        // inside-cut lists (ShadeRec::nbr indexes them)
    const double4 *trap;        // per sphere rtw_accel::TrapRec {w, cap}
    const uint4 *jump;          // [jump_bits][128] columns of T^(2^k)
    double *out;                // n_rows * W * 3
    uint16_t *spill;            // path-stack levels >= kRegSlots, region A (spill_idx)
    uint16_t *spill_b;          // region B (cooperative groups)
    uint64_t spill_stride;      // levels per column (lane-major; RTW_SPILL_LEVEL_MAJOR builds:
                                // columns per level)
    uint64_t *stamps;           // RTW_STAMPS builds only: [wave][kStampRow], persistent kernel waves
    uint64_t *stamps_drain;     // RTW_STAMPS builds only: [wave][kStampRow], rtw_park_leftover waves
    struct Parked *park;        // parked pixels (cursor lanes -> drain groups)
    uint32_t *park_count;       // parked pixels
    uint32_t *park_cursor;      // the drain groups' next queue ticket
    U128 *seeds;                // per-pixel RNG children (persistent phase 1)
    uint32_t *diag;             // RTW_DIAG=1: per pixel {segments, clock/1024 at completion}
    uint32_t diag_ev;           // RTW_DIAG=2: then per pixel {hand-out, first park, first claim} clocks
    uint32_t *order_map;        // hand-out order of the persistent kernel (pixel per ticket) or null
    uint32_t *cost;             // per 8x8 tile: probe segments, then its bucket, then its base;
                                // then per tile: its hot pixels
    uint32_t *pcost;            // per pixel: probe segments
    uint32_t *cost_hist;        // [kCostBuckets] counts, then bucket write cursors
    uint32_t *pix_cursor;       // next pixel of the persistent phase 1
    uint32_t *park_ctl_done;    // cursor-taking waves that will park no more
    uint32_t *park_flag;        // per park slot: 1 once the entry is published
    uint32_t *pixels_done;      // pixels written (completeness check of the persistent kernel)
    uint32_t *park_processed;   // park entries finished (persistent drain + leftover launch)
    uint32_t *leftover_cursor;  // slot cursor of the leftover launch (rtw_park_leftover)
    uint64_t spin_guard;        // idle waits end after this many 100 MHz ticks without progress
    const uint4 *tries;         // trapped-path replay lane table (rtw::try_table, [129][64] columns)
    unsigned long long *counters;  // [0] segments, [1] wave iterations, [2] exact tests,
                                   // [3] wave exact-pass iterations, [4] walk visits, [5] brute segments,
                                   // [6] parked pixels, [7] idle waits ended by the no-progress guard,
                                   // [8] inside cuts, [9] segments skipped by the trapped-path
                                   // fast-forward, [10] park entries left to rtw_park_leftover
};

// ------------------------------------------------------------------ XorShift --
// random.rs:33-38 on (lo, hi) halves
__device__ __forceinline__ void xs_step(U128 &s) {
    uint64_t hi = s.hi ^ ((s.hi << 23) | (s.lo >> 41));
    uint64_t lo = s.lo ^ (s.lo << 23);
    lo ^= (lo >> 17) | (hi << 47);
    hi ^= hi >> 17;
    hi ^= (hi << 26) | (lo >> 38);
    lo ^= lo << 26;
    s.lo = lo;
    s.hi = hi;
}
// random.rs:40-52: u128 % (2^32-1) by limb folding (2^32 == 1 mod 2^32-1),
// then m / 4294967295.0 correctly rounded, computed division-free
// (rtw_numeric.h; exhaustively equal to the IEEE divide for every m).
// u128 mod (2^32-1) = the four 32-bit limbs summed mod 2^32-1 (2^32 == 1): a
// 32-bit sum with its carries, the carries folded back in, 2^32-1 -> 0.
__device__ __forceinline__ uint32_t xs_next_m(U128 &s) {
    xs_step(s);
    unsigned c0, c1, c2, c3;
    uint32_t t = __builtin_addc(static_cast<uint32_t>(s.lo), static_cast<uint32_t>(s.lo >> 32), 0u, &c0);
    t = __builtin_addc(t, static_cast<uint32_t>(s.hi), 0u, &c1);
    t = __builtin_addc(t, static_cast<uint32_t>(s.hi >> 32), 0u, &c2);
    t = __builtin_addc(t, c0 + c1 + c2, 0u, &c3);  // wraps at most once, to <= 2
    t += c3;
    return t == 0xffffffffu ? 0u : t;
}
__device__ __forceinline__ double xs_next_01(U128 &s) { return rtw_num::next01_of(xs_next_m(s)); }

// Rejection sampling on -1 + 2 next_01(): the candidate is first judged in f32
// from the raw draws m. |x32 - x64| <= 2^-22.5 per coordinate (f32 conversion,
// the m / (2^32 - 1) vs m 2^-32 scale, roundings), so a squared length within
// 2^-17 of 1 is the only case that needs the exact f64 value; accepted
// candidates are then rebuilt exactly. (Same draws, same decisions as the f64
// loop: the RNG advances identically.)
constexpr float kRejBand = 7.62939453125e-06f;  // 2^-17
__device__ __forceinline__ float coord32(uint32_t m) {
    return fmaf(static_cast<float>(m), 4.656612873077393e-10f, -1.f);  // 2 m 2^-32 - 1
}
__device__ __forceinline__ double coord64(uint32_t m) { return -1. + rtw_num::next01_of(m) * 2.; }
// random.rs:61-69: the child handed out by copy_reset at parent state p
__device__ __forceinline__ U128 child_of(U128 p) {
    U128 n = p;
    xs_step(n);
    uint64_t lo = p.lo ^ n.lo, hi = p.hi ^ n.hi;
    lo ^= (lo >> 13) | (hi << 51);
    hi ^= hi >> 13;
    hi ^= (hi << 5) | (lo >> 59);
    lo ^= lo << 5;
    lo ^= (lo >> 11) | (hi << 53);
    hi ^= hi >> 11;
    return U128{lo, hi};
}
// Parent state before pixel p = T^p(seed) (the serial chain of camera.rs:269-272),
// by GF(2) jump-ahead: wave-uniform column loads, per-lane masked XOR.
__device__ __forceinline__ U128 jump_state(U128 s, uint64_t p, const uint4 *__restrict__ tab,
                                           uint32_t bits) {
    for (uint32_t k = 0; k < bits; ++k) {
        const uint4 *cols = tab + k * 128u;
        uint64_t rlo = 0, rhi = 0;
#pragma unroll 8
        for (int j = 0; j < 64; ++j) {
            const uint64_t m = 0ull - ((s.lo >> j) & 1ull);
            const uint4 c = cols[j];
            rlo ^= m & ((static_cast<uint64_t>(c.y) << 32) | c.x);
            rhi ^= m & ((static_cast<uint64_t>(c.w) << 32) | c.z);
        }
#pragma unroll 8
        for (int j = 0; j < 64; ++j) {
            const uint64_t m = 0ull - ((s.hi >> j) & 1ull);
            const uint4 c = cols[64 + j];
            rlo ^= m & ((static_cast<uint64_t>(c.y) << 32) | c.x);
            rhi ^= m & ((static_cast<uint64_t>(c.w) << 32) | c.z);
        }
        if ((p >> k) & 1ull) {
            s.lo = rlo;
            s.hi = rhi;
        }
    }
    return s;
}

// vec3.rs:207-232: rejection in [-1,1]^3 with len^2 <= 1, then / sqrt(len^2)
__device__ __forceinline__ void random_unit_vec(U128 &rng, double &ux, double &uy, double &uz) {
    double x, y, z, l2;
    for (;;) {
        const uint32_t m0 = xs_next_m(rng), m1 = xs_next_m(rng), m2 = xs_next_m(rng);
        const float x32 = coord32(m0), y32 = coord32(m1), z32 = coord32(m2);
        const float l32 = fmaf(x32, x32, fmaf(y32, y32, z32 * z32));
        if (l32 > 1.f + kRejBand) continue;  // surely rejected
        x = coord64(m0), y = coord64(m1), z = coord64(m2);
        l2 = x * x + y * y + z * z;
        if (l32 < 1.f - kRejBand || l2 <= 1.) break;  // surely / exactly accepted
    }
    const double l = __builtin_sqrt(l2);
    rtw_num::div3(x, y, z, l);  // x / l, y / l, z / l (one shared reciprocal, same bits)
    ux = x, uy = y, uz = z;
}

// Material rows of the current path's non-dielectric bounces (dielectric
// attenuation is (1,1,1): an exact no-op in the product). The first kRegSlots
// entries live in two u64 registers; deeper ones go to a coalesced HBM buffer
// (one u16 per pixel per level). No private/scratch memory is used: a scratch
// array caps the waves a CU may hold.
constexpr uint32_t kRegSlots = 8;
// Spill columns are owned by one lane (or one cooperative group) for a whole
// launch: cursor lanes use column = pixel in spill region A, cooperative groups
// column = park slot in region B. A pixel that parks on one XCD and resumes on
// another therefore never writes bytes that the first XCD's L2 may still hold
// dirty (the L2s are not coherent with each other), and plain cached accesses
// stay correct.
// Spill slot of stack level l (>= kRegSlots) in column col. Lane-major: a column's
// levels are contiguous (max_depth - kRegSlots u16 each), so a deep path dirties one
// or two cache lines instead of one line per level -- the lanes of a persistent
// wave push at different times, so the level-major layout's coalescing never
// happened there, and its ~84 MB of level rows were written back line by line.
__device__ __forceinline__ uint64_t spill_idx(uint32_t level, uint64_t col, uint64_t stride) {
    return col * stride + (level - kRegSlots);
}
struct PathStack {
    uint64_t r0 = 0, r1 = 0;
    uint32_t n = 0;
    __device__ __forceinline__ void push(uint32_t v, uint16_t *spill, uint64_t stride, uint64_t col) {
        if (n < 4) r0 |= static_cast<uint64_t>(v) << (16u * n);
        else if (n < kRegSlots) r1 |= static_cast<uint64_t>(v) << (16u * (n - 4u));
        else spill[spill_idx(n, col, stride)] = static_cast<uint16_t>(v);
        ++n;
    }
    __device__ __forceinline__ uint32_t at(uint32_t j, const uint16_t *spill, uint64_t stride,
                                           uint64_t col) const {
        if (j < 4) return static_cast<uint32_t>(r0 >> (16u * j)) & 0xffffu;
        if (j < kRegSlots) return static_cast<uint32_t>(r1 >> (16u * (j - 4u))) & 0xffffu;
        return spill[spill_idx(j, col, stride)];
    }
    __device__ __forceinline__ void clear() { r0 = r1 = 0, n = 0; }
};

// Diagnostic build only (-DRTW_STAMPS, librtw_stamps.so): per-wave s_memtime
// cycle sums per section; never compiled into the product library.
#ifdef RTW_STAMPS
constexpr int kStampSlots = 10;  // diagnostic rows: [0, kStampSlots) sections, [14] count, [15] clock
constexpr int kStampRow = 16;
__device__ __forceinline__ uint64_t stamp_now() {
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
struct Stamps {
    uint64_t last = stamp_now(), acc[kStampSlots] = {};
    uint64_t cnt[4] = {};  // draws loop (rows 10-13): [0] trips (max over lanes), [1] lanes needing
                           // a unit vector, [2] of them resumed from a speculation, [3] needing the disk
};
#define STAMP_CNT(k, v) (stp.cnt[k] += (v))
#define STAMP(k)                                   \
    do {                                           \
        const uint64_t t_ = stamp_now();           \
        stp.acc[k] += t_ - stp.last;               \
        stp.last = t_;                             \
    } while (0)
#else
struct Stamps {};
#define STAMP(k) \
    do {         \
    } while (0)
#define STAMP_CNT(k, v) ((void)0)
#endif

// ---------------------------------------------------------------- megakernel --
// A pixel's sampling state between samples (camera.rs:354-374 loop state): the
// pixel's RNG, the next lattice sample and the running sum.
struct PixelState {
    U128 rng;
    uint32_t k;
    double ar, ag, ab;
};
// Park queue entry: a pixel whose segment budget ran out at a sample boundary,
// finished by the cooperative kernel (64 B).
struct Parked {
    uint32_t x, lr, k, _pad;
    uint64_t rng_lo, rng_hi;
    double ar, ag, ab, _pad2;
};

// Scene data a kernel reads per segment: f64 sphere records, shading records,
// BVH nodes + leaves, inside-cut lists -- in LDS when they fit (kLds), else in HBM.
struct SceneView {
    const double4 *sph;
    const ShadeRec *shd;
    const float4 *nodes, *leaves;
    const uint16_t *nbr;
    float4 *end;  // first LDS float4 after the staged scene (kLds), else nullptr
};
// Shading records in LDS (read from HBM through the caches instead, the 23 KB freed
// for a fourth wave per SIMD: slower, profiles/r03_misc/ab_pblock1024_shadeglobal_REJECTED.log)
constexpr size_t kShadeLds = sizeof(ShadeRec);
// inside-cut list entries (u16) in float4 units
__host__ __device__ constexpr uint32_t nbr_f4(uint32_t n_nbr) { return (n_nbr + 7u) / 8u; }
// BVH nodes in float4 units, padded to 32 B (the double4 records after them)
__host__ __device__ constexpr uint32_t node_area_f4(uint32_t n_node) { return (rtw_accel::kNodeF4 * n_node + 1u) & ~1u; }
// LDS layout: (BVH) [node_area_f4] nodes + [2 n_leaf] leaves (float4) first -- the
// walk's node addresses are then id * 144 with no base register -- then [n] double4
// sph | [n] ShadeRec | (BVH) inside-cut lists (padded to float4)
__host__ __device__ inline size_t lds_bytes_for(uint32_t n, uint32_t n_node, uint32_t n_leaf, bool bvh,
                                                uint32_t n_nbr = 0) {
    return static_cast<size_t>(n) * sizeof(double4) + ((static_cast<size_t>(n) * kShadeLds + 15) & ~size_t(15)) +
           (bvh ? (static_cast<size_t>(node_area_f4(n_node)) + 2 * static_cast<size_t>(n_leaf) + nbr_f4(n_nbr)) *
                      sizeof(float4)
                : 0);
}
// Persistent kernel, per-lane LDS areas after the scene view: the running pixel
// sum (3 x f64 columns), the BVH walk scratch (kScratch x u16 columns) and the
// speculative draws' RNG state (one 16 B column).
__host__ __device__ constexpr size_t lane_lds_area(uint32_t threads) {
    return static_cast<size_t>(threads) * (3 * sizeof(double) + rtw_accel::kScratch * sizeof(uint16_t) + 16);
}
// + one u32 per workgroup after the lanes' areas: its cursor waves' completions,
// posted to pixels_done as each cursor wave leaves its loop (RTW_WG_DONE=0 builds: one
// device-scope atomic on pixels_done per wave iteration with a completion, as before
// round 6). Those atomics all hit one word from every CU; a wave's later
// s_waitcnt vmcnt(0) waits for its own, so at 100 spp -- five times the completions
// per segment of the headline -- they held the waves: config 3 26.62 -> 24.23 ms,
// the headline 119.19 -> 118.97 ms, the persistent kernel's writes 166 -> 140 MB
// (profiles/r06_misc/ab_wg_done.log). Launches with the endgame, whose trigger reads
// the count, keep the global atomic.
#ifndef RTW_WG_DONE
#define RTW_WG_DONE 1
#endif
constexpr bool kWgDone = RTW_WG_DONE != 0;
__host__ __device__ constexpr size_t lane_lds_bytes(uint32_t threads) {
    return lane_lds_area(threads) + 16u;
}
// One camera path in flight (the ray_color recursion flattened): the current
// ray, its depth and the material rows of its non-dielectric bounces.
struct Path {
    double ox, oy, oz, dx, dy, dz;
    uint32_t depth;
    int prev;  // sphere of the last hit (-1: camera ray): the inside-cut hint
    PathStack stk;
};

// The camera block (KParams' first 28 doubles) read at each use from the kernarg
// segment through a pointer the compiler cannot hoist (an empty asm redefines it):
// the s_loads land in SGPRs for the few instructions that use them, instead of 56
// SGPRs held -- spilled to VGPR lanes and restored by v_readlane -- through the
// whole persistent loop. Every kernel calling these helpers takes one KParams by
// value, so it sits at kernarg offset 0.
// KP(field) reads any other KParams field the same way (rarely used fields and the
// pointers of the persistent loop: a 16-SGPR kernarg tuple restored by 16
// v_readlane to use one pointer in it is what the compiler does otherwise).
#if defined(__HIP_DEVICE_COMPILE__)
typedef const __attribute__((address_space(4))) double kdouble;
typedef const __attribute__((address_space(4))) char kchar;
__device__ __forceinline__ kchar *karg_base() {
    // readfirstlane: the asm's operand must be an SGPR pair wherever the compiler
    // keeps the segment pointer ("illegal VGPR to SGPR copy" otherwise)
    const uint64_t a = reinterpret_cast<uint64_t>(__builtin_amdgcn_kernarg_segment_ptr());
    uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a));
    uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a >> 32));
    // the comment tags every expansion for the build-time guard (tools/check_karg.py,
    // `make karg-check`): the function holding it must be a lone-KParams kernel that
    // makes no call -- an outlined helper would read some other argument block
    asm volatile("; rtw-karg kparams=%2" : "+s"(lo), "+s"(hi) : "n"(sizeof(KParams)));
    return reinterpret_cast<kchar *>((static_cast<uint64_t>(hi) << 32) | lo);
}
#define KP(f) (*reinterpret_cast<const __attribute__((address_space(4))) decltype(KParams::f) *>(karg_base() + offsetof(KParams, f)))
#else
#define KP(f) (P.f)
#endif
struct CamRef {
#if defined(__HIP_DEVICE_COMPILE__)
    kdouble *c;
    __device__ __forceinline__ explicit CamRef(const KParams &) : c(reinterpret_cast<kdouble *>(karg_base())) {}
#else
    const double *c;
    __device__ __forceinline__ explicit CamRef(const KParams &P) : c(P.p00) {}
#endif
    // offsets (doubles) of the KParams camera block
    enum { kP00 = 0, kDu = 3, kDv = 6, kFrom = 9, kDdu = 12, kDdv = 15, kLatDx = 18, kLatDy = 21, kLatPos0 = 24, kDefocus = 27 };
    __device__ __forceinline__ double operator()(int i) const { return c[i]; }
};
static_assert(offsetof(KParams, p00) == 8 * CamRef::kP00 && offsetof(KParams, du) == 8 * CamRef::kDu &&
                  offsetof(KParams, dv) == 8 * CamRef::kDv && offsetof(KParams, from) == 8 * CamRef::kFrom &&
                  offsetof(KParams, ddu) == 8 * CamRef::kDdu && offsetof(KParams, ddv) == 8 * CamRef::kDdv &&
                  offsetof(KParams, lat_dx) == 8 * CamRef::kLatDx && offsetof(KParams, lat_dy) == 8 * CamRef::kLatDy &&
                  offsetof(KParams, lat_pos0) == 8 * CamRef::kLatPos0 &&
                  offsetof(KParams, defocus_angle) == 8 * CamRef::kDefocus,
              "CamRef offsets follow the KParams camera block");

// get_ray, camera.rs:403: pixel_loc = (pixel00 + i*du) + j*dv
struct PixelLoc {
    double x, y, z;
    PixelLoc() = default;
    __device__ __forceinline__ PixelLoc(const KParams &P, uint32_t px, uint32_t py) {
        const CamRef C(P);
        const double fx = static_cast<double>(px), fy = static_cast<double>(py);
        x = (C(C.kP00 + 0) + C(C.kDu + 0) * fx) + C(C.kDv + 0) * fy;
        y = (C(C.kP00 + 1) + C(C.kDu + 1) * fx) + C(C.kDv + 1) * fy;
        z = (C(C.kP00 + 2) + C(C.kDu + 2) * fx) + C(C.kDv + 2) * fy;
    }
};

// get_ray (camera.rs:400-420) with the defocus disk point (px, py) already drawn:
// the lattice offset of sample k, the origin, the direction; starts a fresh path.
// offset_lattice entry k (camera.rs:422-450; k / s exactly by a multiply-high when
// k e < 2^32, e = m s - 2^32 < s, k < s^2: s^3 <= 2^32, host: s <= 1625)
__device__ __forceinline__ void lattice_off(const KParams &P, uint32_t k, double &offx, double &offy,
                                            double &offz) {
    const CamRef C(P);
    if (KP(s) == 0) {
        offx = C(C.kLatPos0 + 0), offy = C(C.kLatPos0 + 1), offz = C(C.kLatPos0 + 2);
    } else {
        const uint32_t ly = KP(s_magic) ? __umulhi(k, KP(s_magic)) : k / KP(s), lx = k - ly * KP(s);
        const double fly = static_cast<double>(ly), flx = static_cast<double>(lx);
        offx = (C(C.kLatPos0 + 0) + C(C.kLatDy + 0) * fly) + C(C.kLatDx + 0) * flx;
        offy = (C(C.kLatPos0 + 1) + C(C.kLatDy + 1) * fly) + C(C.kLatDx + 1) * flx;
        offz = (C(C.kLatPos0 + 2) + C(C.kLatDy + 2) * fly) + C(C.kLatDx + 2) * flx;
    }
}
// the ray origin: look_from, or the defocus disk point (px, py) (camera.rs:406-410, 452-456)
__device__ __forceinline__ void ray_origin(const KParams &P, double px, double py, Path &p) {
    const CamRef C(P);
    if (C(C.kDefocus) <= 0.) {
        p.ox = C(C.kFrom + 0), p.oy = C(C.kFrom + 1), p.oz = C(C.kFrom + 2);
    } else {
        p.ox = (C(C.kFrom + 0) + C(C.kDdu + 0) * px) + C(C.kDdv + 0) * py;
        p.oy = (C(C.kFrom + 1) + C(C.kDdu + 1) * px) + C(C.kDdv + 1) * py;
        p.oz = (C(C.kFrom + 2) + C(C.kDdu + 2) * px) + C(C.kDdv + 2) * py;
    }
}

__device__ __forceinline__ void ray_from_disk(const KParams &P, const PixelLoc &pl, uint32_t k, double px,
                                              double py, Path &p) {
    double offx, offy, offz;
    lattice_off(P, k, offx, offy, offz);
    const double sx = pl.x + offx, sy = pl.y + offy, sz = pl.z + offz;
    ray_origin(P, px, py, p);
    p.dx = sx - p.ox, p.dy = sy - p.oy, p.dz = sz - p.oz;
    p.depth = 0;
    p.prev = -1;
    p.stk.clear();
}

// camera.rs:400-420 + offset_lattice (422-450) + defocus_disk_sample (452-456):
// the ray of lattice sample k; starts a fresh path.
__device__ __forceinline__ void gen_ray(const KParams &P, const PixelLoc &pl, uint32_t k, U128 &rng,
                                        Path &p, Stamps &stp) {
    double offx, offy, offz;
    lattice_off(P, k, offx, offy, offz);
    const double sx = pl.x + offx, sy = pl.y + offy, sz = pl.z + offz;
    STAMP(8);  // 8: lattice sample position
    if (CamRef(P)(CamRef::kDefocus) <= 0.) {
        ray_origin(P, 0., 0., p);
    } else {
        double px, py;
        for (;;) {  // vec3.rs:270-277: strict len^2 < 1 (f32 pre-judged, as random_unit_vec)
            const uint32_t m0 = xs_next_m(rng), m1 = xs_next_m(rng);
            const float x32 = coord32(m0), y32 = coord32(m1);
            const float l32 = fmaf(x32, x32, y32 * y32);
            if (l32 > 1.f + kRejBand) continue;
            px = -1. + 2. * rtw_num::next01_of(m0);
            py = -1. + 2. * rtw_num::next01_of(m1);
            if (l32 < 1.f - kRejBand || (px * px + py * py + 0. * 0.) < 1.) break;
        }
        ray_origin(P, px, py, p);
    }
    STAMP(9);  // 9: defocus disk sample
    p.dx = sx - p.ox, p.dy = sy - p.oy, p.dz = sz - p.oz;
    p.depth = 0;
    p.prev = -1;
    p.stk.clear();
}

// What a scatter tells the trapped-path fast-forward (rtw_accel.h "Trapped
// paths"): a Lambertian bounce off S's inner face (lam) or a total internal
// reflection inside S (tir), S's outward normal h0 at the hit, and for Lambertian
// the unit vector u, whether near_zero replaced the direction, and |d|^2.
struct TrapHint {
    bool lam = false, tir = false, quirk = false;
    double h0x = 0., h0y = 0., h0z = 0., ux = 0., uy = 0., uz = 0., a1 = 0.;
};

// After Scene::hit: HitRecord + Material::scatter (materials.rs:22-111) on a hit,
// the sky colour (camera.rs:395-397) on a miss. Returns true when the sample's
// path ended (sky, or depth cap -> black); then (lr, lg, lb) is the leaf colour.
// unit(dir) (vec3.rs:183-185) is formed once for whichever of the sky, Metal
// (materials.rs:55) and Dielectric (materials.rs:91) the wave's lanes need, and
// the reflection (vec3.rs:252-257) once for Metal and reflecting Dielectric lanes.
// With kTrap the scatter also fills *th (trapped-path hints).
template <bool kTrap = false>
__device__ __forceinline__ bool shade(const KParams &P, const double4 *__restrict__ sph,
                                      const ShadeRec *__restrict__ shd, int best, double bt, double a,
                                      Path &p, U128 &rng, uint16_t *spill, uint64_t col, uint64_t stride,
                                      double &lr, double &lg, double &lb, Stamps &stp, TrapHint *th = nullptr) {
    lr = lg = lb = 0.;
    const uint32_t kind = best >= 0 ? shd[best].kind : 3u;  // 3: the sky
    double vx = 0., vy = 0., vz = 0.;
    if (kind != RTW_LAMBERTIAN) {
        vx = p.dx, vy = p.dy, vz = p.dz;
        rtw_num::div3(vx, vy, vz, __builtin_sqrt(a));  // unit(dir): / l, one shared reciprocal
    }
    if (best < 0) {
        const double t = 0.5 * (vy + 1.0);
        const double om = 1.0 - t;
        lr = om + 0.5 * t;
        lg = om + 0.7 * t;
        lb = om + t;
        return true;
    }
    // HitRecord: point = dir*t + orig, outward = (p - c)/r, face_normal
    const double4 S = sph[best];
    const ShadeRec M = shd[best];
    const double r = S.w;
    const double px = p.dx * bt + p.ox, py = p.dy * bt + p.oy, pz = p.dz * bt + p.oz;
    double nx = px - S.x, ny = py - S.y, nz = pz - S.z;
    rtw_num::div3(nx, ny, nz, r);  // (p - c) / r
    const bool front = (p.dx * nx + p.dy * ny + p.dz * nz) < 0.;
    if constexpr (kTrap) th->h0x = nx, th->h0y = ny, th->h0z = nz;
    if (!front) nx = -nx, ny = -ny, nz = -nz;
    STAMP(6);  // 6: hit record (point, normal, face)
    double ux = 0., uy = 0., uz = 0.;
    if (kind != RTW_DIELECTRIC) {
        // Lambertian and Metal each draw exactly one random_unit_vec and nothing
        // else from the RNG: one rejection loop serves both (less divergence)
        random_unit_vec(rng, ux, uy, uz);
    }
    bool refl = kind == RTW_METAL;
    double ratio = 0., cos_t = 0.;
    if (kind == RTW_DIELECTRIC) {  // materials.rs:83-111 (attenuation 1: exact no-op)
        // M.a0 = 1/ir and M.a1 = r0*r0 of reflectance (75-80), formed by the host
        // with the reference's own IEEE operations: the same bits
        ratio = front ? M.a0 : M.p;
        cos_t = fmin((-vx) * nx + (-vy) * ny + (-vz) * nz, 1.);
        // ratio * sqrt(1 - cos^2) > 1, its square root taken only near the boundary
        const double sin2 = 1.0 - cos_t * cos_t;
        refl = rtw_num::tir_exceeds(ratio, sin2, 1.);
        if constexpr (kTrap) {  // TIR with margin, chords 2 r cos well above 0.01
            th->tir = !front && refl && rtw_num::tir_exceeds(ratio, sin2, 1. + 1e-9) && r * cos_t > 0.0055;
        }
        if (!refl) {
            const double r0 = M.a1;
            const double q = 1. - cos_t;
            const double schlick = r0 + (1. - r0) * (q * ((q * q) * (q * q)));
            refl = schlick > xs_next_01(rng);
        }
    }
    double ndx = 0., ndy = 0., ndz = 0.;
    if (refl) {  // vec3.rs:252-257
        const double dt = vx * nx + vy * ny + vz * nz;
        ndx = vx - (nx * dt) * 2., ndy = vy - (ny * dt) * 2., ndz = vz - (nz * dt) * 2.;
    }
    if (kind == RTW_LAMBERTIAN) {  // materials.rs:22-37; near_zero has no abs (vec3.rs:246-250)
        ndx = nx + ux, ndy = ny + uy, ndz = nz + uz;
        const bool quirk = ndx < 1e-8 && ndy < 1e-8 && ndz < 1e-8;
        if (quirk) ndx = nx, ndy = ny, ndz = nz;
        if constexpr (kTrap) {
            th->lam = !front, th->quirk = quirk;
            th->ux = ux, th->uy = uy, th->uz = uz;
            th->a1 = ndx * ndx + ndy * ndy + ndz * ndz;
        }
    } else if (kind == RTW_METAL) {  // materials.rs:52-63: reflected + fuzz * u
        ndx = ndx + ux * M.p, ndy = ndy + uy * M.p, ndz = ndz + uz * M.p;
    } else if (!refl) {  // vec3.rs:259-268 (its cos is cos_t: the same expression)
        const double qx = (vx + nx * cos_t) * ratio, qy = (vy + ny * cos_t) * ratio,
                     qz = (vz + nz * cos_t) * ratio;
        const double w = -__builtin_sqrt(__builtin_fabs(1. - (qx * qx + qy * qy + qz * qz)));
        ndx = qx + nx * w, ndy = qy + ny * w, ndz = qz + nz * w;
    }
    if (kind != RTW_DIELECTRIC) p.stk.push(static_cast<uint32_t>(best), spill, stride, col);  // attenuation row
    p.ox = px, p.oy = py, p.oz = pz;
    p.dx = ndx, p.dy = ndy, p.dz = ndz;
    p.prev = best;
    ++p.depth;
    return p.depth >= P.max_depth;  // ray_color(depth >= max) -> black
}

// One 64-lane round of random_unit_vec tries (vec3.rs:219-232) after the wave-uniform
// RNG state s: lane j takes try j -- the three draws after 3 j draws -- from its state
// T^(3 j) s, the XOR of the try table's columns over s's set bits (rtw::try_table; s is
// wave-uniform, so the bit loop is scalar and each step one coalesced 1-KB load). The
// accept decision is random_unit_vec's, so the accepted tries of the round are, in lane
// order, the unit vectors the serial loop would return, and a lane's state after its
// draws is the serial loop's state after that try. Returns the ballot of accepted tries;
// (ux, uy, uz) = the lane's unit vector, st = its state after its three draws.
#ifndef RTW_TRY_GATHER
#define RTW_TRY_GATHER 4
#endif
constexpr int kGather = RTW_TRY_GATHER;  // table columns loaded per trip of the gather loop
__device__ __forceinline__ uint64_t unit_vec_round(const uint4 *__restrict__ tries, U128 s, U128 &st, double &ux,
                                                   double &uy, double &uz) {
    const uint32_t lane = __lane_id();
#ifdef RTW_STAMPS  // diagnostic build: the whole-wave, wave-uniform-state assumption
    if (__ballot(1) != ~0ull ||
        static_cast<uint32_t>(s.lo) != static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(s.lo))) ||
        static_cast<uint32_t>(s.hi >> 32) !=
            static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(s.hi >> 32))))
        __builtin_trap();
#endif
    const uint4 *col = tries + lane;
    uint64_t lo = 0, hi = 0;
    for (uint32_t h = 0; h < 2; ++h) {
        uint64_t m = h ? s.hi : s.lo;
        // (readfirstlane returns int: the low word goes through uint32_t, not sign-extended)
        m = (static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(m >> 32))))
             << 32) |
            static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(m)));
        const uint32_t off = h ? 64u : 0u;
        while (m) {  // kGather columns per trip, their loads in flight together (row 128 is zero)
            uint32_t b[kGather];
#pragma unroll
            for (int q = 0; q < kGather; ++q) {
                b[q] = m ? static_cast<uint32_t>(__builtin_ctzll(m)) + off : 128u;
                m &= m - 1ull;
            }
            uint4 c[kGather];
#pragma unroll
            for (int q = 0; q < kGather; ++q) c[q] = col[b[q] * 64u];
#pragma unroll
            for (int q = 0; q < kGather; ++q) {
                lo ^= (static_cast<uint64_t>(c[q].y) << 32) | c[q].x;
                hi ^= (static_cast<uint64_t>(c[q].w) << 32) | c[q].z;
            }
        }
    }
    st = U128{lo, hi};
    const uint32_t m0 = xs_next_m(st), m1 = xs_next_m(st), m2 = xs_next_m(st);
    const float x32 = coord32(m0), y32 = coord32(m1), z32 = coord32(m2);
    const float l32 = fmaf(x32, x32, fmaf(y32, y32, z32 * z32));
    const double x = coord64(m0), y = coord64(m1), z = coord64(m2);
    const double l2 = x * x + y * y + z * z;
    // random_unit_vec's decision: surely rejected in f32, else surely or exactly accepted
    const bool ok = !(l32 > 1.f + kRejBand) && (l32 < 1.f - kRejBand || l2 <= 1.);
    ux = x, uy = y, uz = z;
    rtw_num::div3(ux, uy, uz, __builtin_sqrt(l2));  // x / l, y / l, z / l (random_unit_vec's)
    return __ballot(ok);
}
__device__ __forceinline__ double readlane_f64(double v, uint32_t l) {
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                            __builtin_amdgcn_readlane(__double2loint(v), l));
}
__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, uint32_t l) {
    return (static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(v >> 32), l)))
            << 32) |
           static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(v), l));
}

// Trapped-path fast-forward (rtw_accel.h "Trapped paths"). The path has just
// scattered inside sphere S (record T) with `rem` segments left before the depth
// cap. Returns rem if every one of them provably stays inside S -- the sample
// then ends black, and for a Lambertian trap the RNG has advanced by the rem
// random_unit_vec draws those bounces make -- or 0 with nothing changed.
// kWave (64-lane drain groups: every lane of the wave holds this path): the draws are
// replayed 64 tries at a time, one per lane (unit_vec_round), and the wave walks the
// accepted ones in order -- the serial rejection loop (89 % of a Lambertian-trapped
// chain's time in round 4) becomes a table gather per 64 tries.
template <bool kWave = false>
__device__ __forceinline__ uint32_t trap_forward(const double4 T, uint32_t rem, const TrapHint &th,
                                                 double dx, double dy, double dz, U128 &rng,
                                                 const uint4 *__restrict__ tries = nullptr) {
    const double cap = T.w;
    if (!(th.h0x * T.x + th.h0y * T.y + th.h0z * T.z < cap)) return 0u;  // the next chord's start
    if (th.tir) {
        // the path walks the great circle of S in the plane of h0 and d: all of it
        // below the cap (|w projected on the plane| < cap) keeps every chord clear
        double mx = th.h0y * dz - th.h0z * dy, my = th.h0z * dx - th.h0x * dz, mz = th.h0x * dy - th.h0y * dx;
        const double ml = __builtin_sqrt(mx * mx + my * my + mz * mz);
        if (!(ml > 1e-3)) return 0u;
        mx /= ml, my /= ml, mz /= ml;
        const double wm = T.x * mx + T.y * my + T.z * mz;
        const double px = T.x - wm * mx, py = T.y - wm * my, pz = T.z - wm * mz;
        return px * px + py * py + pz * pz < cap * cap && cap > 0. ? rem : 0u;
    }
    if (!th.quirk && !(th.a1 >= 1e-9)) return 0u;
    // end of the next chord: c + r u, or the antipode when near_zero set d = n_in
    double hx = th.quirk ? -th.h0x : th.ux, hy = th.quirk ? -th.h0y : th.uy, hz = th.quirk ? -th.h0z : th.uz;
    if constexpr (kWave) {
        U128 base = rng;
        uint32_t i = 1;  // the bounce whose chord end is checked next
        for (;;) {
            U128 st;
            double ux, uy, uz;
            uint64_t acc = unit_vec_round(tries, base, st, ux, uy, uz);
            while (acc) {
                const uint32_t a = static_cast<uint32_t>(__builtin_ctzll(acc));
                acc &= acc - 1ull;
                if (!(hx * T.x + hy * T.y + hz * T.z < cap)) return 0u;  // end of chord i
                if (i >= rem) {  // the scatter at the end of segment rem: its draws are the last
                    rng = U128{readlane_u64(st.lo, a), readlane_u64(st.hi, a)};
                    return rem;
                }
                const double vx = readlane_f64(ux, a), vy = readlane_f64(uy, a), vz = readlane_f64(uz, a);
                const double ex = vx - hx, ey = vy - hy, ez = vz - hz;
                const bool q_yes = ex < -1e-6 && ey < -1e-6 && ez < -1e-6;
                const bool q_no = ex > 1e-6 || ey > 1e-6 || ez > 1e-6;
                if (q_yes == q_no) return 0u;
                if (q_yes) {
                    hx = -hx, hy = -hy, hz = -hz;
                } else {
                    if (!(ex * ex + ey * ey + ez * ez >= 1e-8)) return 0u;
                    hx = vx, hy = vy, hz = vz;
                }
                ++i;
            }
            base = U128{readlane_u64(st.lo, 63u), readlane_u64(st.hi, 63u)};  // after the round's 64 tries
        }
    }
    U128 r2 = rng;
    for (uint32_t i = 1;; ++i) {
        if (!(hx * T.x + hy * T.y + hz * T.z < cap)) return 0u;  // end of chord i
        double vx, vy, vz;
        random_unit_vec(r2, vx, vy, vz);  // the scatter at the end of segment i
        if (i >= rem) break;
        // its direction ~ n_in + u = u - h: near_zero decided with margin, |d|^2 >= 1e-9
        const double ex = vx - hx, ey = vy - hy, ez = vz - hz;
        const bool q_yes = ex < -1e-6 && ey < -1e-6 && ez < -1e-6;
        const bool q_no = ex > 1e-6 || ey > 1e-6 || ez > 1e-6;
        if (q_yes == q_no) return 0u;
        if (q_yes) {
            hx = -hx, hy = -hy, hz = -hz;
        } else {
            if (!(ex * ex + ey * ey + ez * ez >= 1e-8)) return 0u;
            hx = vx, hy = vy, hz = vz;
        }
    }
    rng = r2;
    return rem;
}

// att0 * (att1 * (... * leaf)) -- right-to-left, as the recursion associates
// (camera.rs:389); then the sample's colour is added to the pixel sum.
// The spilled levels (deepest, rare) first; then the register levels, whose row
// index is picked branch-free (a select of r0 / r1 and a shift), so the wave runs
// one short loop body per level instead of a three-way branch.
__device__ __forceinline__ void fold(const ShadeRec *__restrict__ shd, Path &p, const uint16_t *spill,
                                     uint64_t col, uint64_t stride, double &lr, double &lg, double &lb) {
    const uint32_t n = p.stk.n;
    for (uint32_t j = n; j-- > kRegSlots;) {
        const ShadeRec &A = shd[spill[spill_idx(j, col, stride)]];
        lr = A.a0 * lr;
        lg = A.a1 * lg;
        lb = A.a2 * lb;
    }
    for (uint32_t j = n < kRegSlots ? n : kRegSlots; j-- > 0;) {
        const uint64_t w = j < 4u ? p.stk.r0 : p.stk.r1;
        const ShadeRec &A = shd[static_cast<uint32_t>(w >> (16u * (j & 3u))) & 0xffffu];
        lr = A.a0 * lr;
        lg = A.a1 * lg;
        lb = A.a2 * lb;
    }
    p.stk.clear();
}
__device__ __forceinline__ void fold(const ShadeRec *__restrict__ shd, Path &p, const uint16_t *spill,
                                     uint64_t col, uint64_t stride, double lr, double lg, double lb,
                                     PixelState &ps) {
    fold(shd, p, spill, col, stride, lr, lg, lb);
    ps.ar = ps.ar + lr, ps.ag = ps.ag + lg, ps.ab = ps.ab + lb;
}

// The reference's per-pixel loop: samples k.. of pixel (x, y) (ray_colors_lattice,
// camera.rs:354-374) with the ray_color recursion (376-398) flattened into a
// segment loop. `hit(ox, oy, oz, dx, dy, dz, a, bt) -> best` is the Scene::hit
// strategy. Returns true if the pixel parked: `budget` segments were exceeded at
// a sample boundary (ps then holds the state to resume from).
// With kTrap (drain groups: one path per group, so the branch is uniform) a
// path trapped inside a sphere is fast-forwarded to its depth cap (trap_forward);
// `trapped` counts the segments skipped that way.
// tir_run (64-lane drain groups): called after a total internal reflection inside S
// whose great-circle forward already failed; it may trace the run's next bounces in
// place (returning how many), leaving the path exactly as the generic loop would.
struct NoTirRun {
    __device__ uint32_t operator()(Path &, int) const { return 0u; }
};
template <bool kTrap = false, bool kWave = false, class HitFn, class TirRun = NoTirRun>
__device__ __forceinline__ bool trace_samples(const KParams &P, const SceneView &sv,
                                              uint32_t x, uint32_t y, uint16_t *spill, uint64_t col,
                                              PixelState &ps, uint32_t budget, uint32_t &seg, Stamps &stp,
                                              HitFn &&hit, uint32_t *trapped = nullptr, TirRun &&tir_run = TirRun{}) {
    const uint32_t n_off = P.n_off;
    if (P.max_depth == 0) {  // every sample is black (no Scene::hit call)
        ps.k = n_off;
        return false;
    }
    if (ps.k >= n_off) return false;
    const PixelLoc pl(P, x, y);
    const uint64_t stride = P.spill_stride;
    Path p;
    int tir_no = -1;  // kTrap: S whose great-circle test failed on the last TIR bounce
    gen_ray(P, pl, ps.k, ps.rng, p, stp);
    STAMP(0);  // 0: seed jump + pixel setup
    for (;;) {
        // ---- Scene::hit (hittable.rs:131-143): first minimum over all spheres ----
        ++seg;
        const double a = p.dx * p.dx + p.dy * p.dy + p.dz * p.dz;
        double bt = 0.;
        const int best = hit(p.ox, p.oy, p.oz, p.dx, p.dy, p.dz, a, p.prev, bt);
        STAMP(1);
        double lr, lg, lb;
        TrapHint th;
        bool done = shade<kTrap>(P, sv.sph, sv.shd, best, bt, a, p, ps.rng, spill, col, stride, lr, lg, lb, stp, &th);
        STAMP(7);  // 7: scatter (after the hit record)
        if constexpr (kTrap) {
            // a total internal reflection keeps the path in the great circle it walks
            // (the chord, the normal and the reflection share S's centre), and the
            // circle test of trap_forward does not depend on the position on it: after
            // one failed test every further TIR bounce inside the same S fails too, so
            // it is skipped (tir_no) until the path leaves the circle -- tracing on is
            // always exact, the forward only saves work
            const bool skip = th.tir && best == tir_no;
            if (!skip) tir_no = -1;  // kept through a run of TIR bounces in the same S
            if (!done && (th.lam || th.tir) && !skip) {
                const uint32_t k = trap_forward<kWave>(KP(trap)[best], P.max_depth - p.depth, th, p.dx, p.dy, p.dz,
                                                       ps.rng, KP(tries));
                if (!k && th.tir) tir_no = best;
                if (k) seg += k, *trapped += k, done = true;  // (lr, lg, lb) = 0: the black leaf
            }
            // the run goes on: its next bounces by the lean loop (they draw nothing and
            // their forward tests would fail again)
            if (!done && th.tir && best == tir_no) seg += tir_run(p, best);
        }
        STAMP(3);  // 3: trapped-path check (kTrap)
        if (done) {
            // a depth-capped (or fast-forwarded) path's product is att x ... x 0 = +-0 with
            // finite attenuations, and adding +-0 to the sum changes no bit: no fold
            if (best >= 0 && KP(att_finite)) p.stk.clear();
            else fold(sv.shd, p, spill, col, stride, lr, lg, lb, ps);
            if (++ps.k >= n_off) break;
            if (seg >= budget) return true;  // sample boundary: hand the rest to the coop kernel
            gen_ray(P, pl, ps.k, ps.rng, p, stp);
        }
        STAMP(4);  // 4: fold + next sample
    }
    return false;
}

// RTW_KARG_SELFTEST (`make karg-selftest` only, never a library): write_pixel outlined,
// so the karg guard must reject the build
#ifdef RTW_KARG_SELFTEST
#define RTW_KARG_HELPER __attribute__((noinline))
#else
#define RTW_KARG_HELPER __forceinline__
#endif
__device__ RTW_KARG_HELPER void write_pixel(const KParams &P, uint32_t x, uint32_t lr,
                                            const PixelState &ps, bool count = true) {
    if (count && KP(pixels_done)) atomicAdd(KP(pixels_done), 1u);
    const double nf = static_cast<double>(KP(n_off));
    double *o = KP(out) + (static_cast<uint64_t>(lr) * KP(W) + x) * 3u;
    o[0] = ps.ar / nf;
    o[1] = ps.ag / nf;
    o[2] = ps.ab / nf;
}

// Exact f64 Sphere::hit (sphere.rs:39-71) of sphere i against the current best,
// keeping the lexicographic (t, index) minimum = the scan's first-minimum rule.
__device__ __forceinline__ void exact_test(const double4 *__restrict__ sph, uint32_t i, double ox,
                                           double oy, double oz, double dx, double dy, double dz,
                                           double a, int &best, double &bt) {
    const double4 S = sph[i];
    double t;
    if (rtw_accel::sphere_hit_f64(ox, oy, oz, dx, dy, dz, a, S.x, S.y, S.z, S.w * S.w, t) &&
        rtw_accel::better(t, i, bt, best)) {
        bt = t;
        best = static_cast<int>(i);
    }
}

// f32 pass-1 state of one segment (shared by the filtered scan and the walk).
// Exact-conservative filter: with ê = d/|d| the discriminant's sign is that of
// D' = (OC.ê)^2 - (|OC|^2 - R2) = D / a. Computed in f32 with oc = o32 - c32,
// e = fl32(ê), and R2' >= R2 + K (m_c^2 + R2/2) in place of R2 (host, rounded
// up), a first-order bound of the f32 error is  u32 (81 M^2 + 4 R2') with
// M_i = |o_i| + |c_i|, M^2 <= 2 (m_o^2 + m_c^2); K = 512 u32 then leaves
//   disc32 >= D' - K m_o^2 - (floor)
// so every sphere whose f64 discriminant is >= 0 (or NaN) passes the test
// disc32 >= -G, G = K m_o^2 + floor. NaN/inf anywhere -> kept.
struct Seg32 {
    float ox, oy, oz, ex, ey, ez, negG;
    double mo, sa;
    bool fast;
    __device__ __forceinline__ Seg32(double x, double y, double z, double dx, double dy, double dz,
                                     double a, bool filter) {
        mo = fmax(fmax(__builtin_fabs(x), __builtin_fabs(y)), __builtin_fabs(z));
        fast = filter && mo <= kGuardHi;  // false for NaN too
        sa = __builtin_sqrt(a);
        const double inv = 1.0 / sa;
        ex = static_cast<float>(dx * inv), ey = static_cast<float>(dy * inv), ez = static_cast<float>(dz * inv);
        ox = static_cast<float>(x), oy = static_cast<float>(y), oz = static_cast<float>(z);
        negG = rtw_accel::filter_neg_g(mo);
    }
    __device__ __forceinline__ bool pass(const float4 S) const {
        const float ocx = ox - S.x, ocy = oy - S.y, ocz = oz - S.z;
        const float hb = fmaf(ocx, ex, fmaf(ocy, ey, ocz * ez));
        const float cc = fmaf(ocx, ocx, fmaf(ocy, ocy, fmaf(ocz, ocz, -S.w)));
        const float disc = fmaf(hb, hb, -cc);
        return !(disc < negG);
    }
};

// Counters kept per lane, atomically added at the end of a kernel.
struct Tally {
    uint32_t seg = 0, ntest = 0, nwave2 = 0, visits = 0, nbrute = 0, parked = 0, witer = 0, inside = 0,
             trap = 0;
};

// The scan: every sphere in index order (first = lane's sub-range start, step =
// sphere stride for cooperative groups); pass 1 = f32 filter on wave-uniform
// records, pass 2 = f64 on the lane's candidates in index order.
__device__ __forceinline__ int scan_hit(const KParams &P, const double4 *__restrict__ sph,
                                        const Seg32 &g, double ox, double oy, double oz, double dx,
                                        double dy, double dz, double a, double &bt, Tally &tl) {
    const uint32_t n = KP(n_sph);
    const float4 *filt = KP(filt);
    const uint32_t lane = threadIdx.x & 63u;
    int best = -1;
    for (uint32_t base = 0; base < n; base += kChunk) {
        const uint32_t cnt = n - base < static_cast<uint32_t>(kChunk) ? n - base : kChunk;
        // sphere base+j is bit (31 - j): highest set bit = lowest index
        uint32_t mask;
        if (g.fast) {
            mask = 0;
            for (uint32_t q = 0; q < static_cast<uint32_t>(kChunk); q += kGroup) {
#pragma unroll
                for (int j = 0; j < kGroup; ++j)
                    mask = mask + mask + static_cast<uint32_t>(g.pass(ld_filt(filt, base + q + j)));
            }
            if (cnt < static_cast<uint32_t>(kChunk)) mask &= ~((1u << (kChunk - cnt)) - 1u);
        } else {
            mask = cnt == static_cast<uint32_t>(kChunk) ? ~0u : ~((1u << (kChunk - cnt)) - 1u);
        }
        while (mask) {
            {  // the wave's first active lane counts the wave-level iteration
                const uint64_t exm = __builtin_amdgcn_read_exec();
                tl.nwave2 += static_cast<uint32_t>(__builtin_ctzll(exm) == static_cast<int>(lane));
            }
            const uint32_t top = 31u - static_cast<uint32_t>(__builtin_clz(mask));
            mask ^= 1u << top;
            ++tl.ntest;
            exact_test(sph, base + (31u - top), ox, oy, oz, dx, dy, dz, a, best, bt);
        }
    }
    return best;
}

// Scene::hit by the BVH (rtw_accel.h): always-spheres exactly, the f32 walk,
// exact candidates, the cut check; anything unproven falls back to the scan.
// kStride: the LDS scratch column stride (the workgroup size; a constant, so the
// walk's pointer steps are immediates and hold no register)
template <bool kLdsStack = false, uint32_t kStride = 0>
__device__ __forceinline__ int bvh_hit(const KParams &P, const SceneView &sv, double ox, double oy,
                                       double oz, double dx, double dy, double dz, double a, int prev,
                                       double &bt, Tally &tl, Stamps &stp, uint16_t *scol = nullptr,
                                       double *sa_out = nullptr) {
    const double4 *__restrict__ sph = sv.sph;
    const float4 *__restrict__ nodes = sv.nodes;
    const float4 *__restrict__ leaves = sv.leaves;
    int best = -1;
    const Seg32 g(ox, oy, oz, dx, dy, dz, a, true);
    if (sa_out) *sa_out = g.sa;  // sqrt(a): the scatter's unit(dir) divides by the same value
    bool brute = !g.fast;
    if (g.fast) {
        const uint32_t n_always = KP(n_always);
        for (uint32_t j = 0; j < n_always; ++j) {  // ground planes etc.
            const uint32_t i = ld_const_u32(KP(always), j);
            if (g.pass(ld_filt(KP(filt), i))) {
                ++tl.ntest;
                exact_test(sph, i, ox, oy, oz, dx, dy, dz, a, best, bt);
            }
        }
        STAMP(5);  // 5: segment setup + always-spheres
        rtw_accel::WalkRay wr;
        if (KP(n_node) == 0) {  // every sphere is an "always" sphere
        } else if (!rtw_accel::walk_setup(g.ox, g.oy, g.oz, g.ex, g.ey, g.ez, g.mo, g.sa, g.negG, wr)) {
            brute = true;
        } else {
            float U = best >= 0 ? rtw_accel::seed_cut(bt, g.sa) : INFINITY;
            auto run = [&](auto &ws) {
                // the node walk at raised issue priority (cursor waves, kLdsStack): it is
                // a chain of dependent LDS round trips, so its wave should issue the
                // moment a load returns while the other waves' f64 code fills the gaps
                // (127.3 -> 124.9 ms; all of Scene::hit raised 125.9, the scatter raised
                // instead +1.9 %: profiles/r03_misc/ab_walk_prio.log). Back to priority 0
                // after it: every wave that walks with kLdsStack is a cursor wave at that
                // point (a priority wave that joins the cursor runs as one).
                if constexpr (kLdsStack && kWalkPrio > 0) __builtin_amdgcn_s_setprio(kWalkPrio);
                const bool walked = rtw_accel::walk(nodes, leaves, wr, U, tl.visits, ws);
                if constexpr (kLdsStack && kWalkPrio > 0) __builtin_amdgcn_s_setprio(0);
                STAMP(2);  // 2: BVH walk
                if (!walked) return false;
                for (uint32_t j = 0; j < ws.nc; ++j) {
                    ++tl.ntest;
                    exact_test(sph, ws.cand_at(j), ox, oy, oz, dx, dy, dz,
                               a, best, bt);
                }
                return true;
            };
            bool walked;
            if constexpr (kLdsStack) {
                static_assert(!kLdsStack || kStride > 0, "LDS scratch needs its stride");
                rtw_accel::LdsScratch ws(scol, kStride);
                walked = run(ws);
            } else {
                rtw_accel::ArrayScratch ws;
                walked = run(ws);
            }
            if (!walked) {
                brute = true;
            } else {
                brute = !rtw_accel::cut_ok(U, best, bt, g.sa);
            }
        }
    }
    if (brute) {
        ++tl.nbrute;
        best = scan_hit(P, sph, g, ox, oy, oz, dx, dy, dz, a, bt, tl);
    }
    return best;
}

__device__ __forceinline__ void flush_tally(const KParams &P, const Tally &tl, bool wave_iters) {
    if (!P.counters) return;
    const uint32_t lane = threadIdx.x & 63u;
    if (tl.seg) atomicAdd(&P.counters[0], static_cast<unsigned long long>(tl.seg));
    if (wave_iters) {  // one-lane-per-pixel kernel: the wave's trip count = max over lanes
        uint32_t m = tl.seg;
        for (int off = 32; off > 0; off >>= 1) m = max(m, static_cast<uint32_t>(__shfl_xor(static_cast<int>(m), off)));
        if (lane == 0 && m) atomicAdd(&P.counters[1], static_cast<unsigned long long>(m));
    }
    if (tl.ntest) atomicAdd(&P.counters[2], static_cast<unsigned long long>(tl.ntest));
    if (tl.nwave2) atomicAdd(&P.counters[3], static_cast<unsigned long long>(tl.nwave2));
    if (tl.witer) atomicAdd(&P.counters[1], static_cast<unsigned long long>(tl.witer));
#ifdef RTW_STAMPS  // visits carries wave-level walk iterations in bits 16+ (diagnostic build)
    if (tl.visits & 0xffffu) atomicAdd(&P.counters[4], static_cast<unsigned long long>(tl.visits & 0xffffu));
    if (tl.visits >> 16) atomicAdd(&P.counters[5], static_cast<unsigned long long>(tl.visits >> 16));
#else
    if (tl.visits) atomicAdd(&P.counters[4], static_cast<unsigned long long>(tl.visits));
#endif
    if (tl.nbrute) atomicAdd(&P.counters[5], static_cast<unsigned long long>(tl.nbrute));
    if (tl.parked) atomicAdd(&P.counters[6], static_cast<unsigned long long>(tl.parked));
    if (tl.inside) atomicAdd(&P.counters[8], static_cast<unsigned long long>(tl.inside));
    if (tl.trap) atomicAdd(&P.counters[9], static_cast<unsigned long long>(tl.trap));
}

template <bool kLds, int kMode>
__device__ __forceinline__ SceneView stage_scene(const KParams &P, double4 *lds) {
    SceneView v{P.sph, P.shade, P.nodes, P.leaves, P.nbr, nullptr};
    if (kLds) {
        const uint32_t n = P.n_sph;
        double4 *ld = lds;
        if (kMode == kBvh) {  // nodes at LDS offset 0, then the leaves
            float4 *lf = reinterpret_cast<float4 *>(lds);
            const uint32_t nn = rtw_accel::kNodeF4 * P.n_node, na = node_area_f4(P.n_node), nl = 2u * P.n_leaf;
            for (uint32_t i = threadIdx.x; i < nn; i += blockDim.x) lf[i] = P.nodes[i];
            for (uint32_t i = threadIdx.x; i < nl; i += blockDim.x) lf[na + i] = P.leaves[i];
            v.nodes = lf;
            v.leaves = lf + na;
            ld = reinterpret_cast<double4 *>(lf + na + nl);
        }
        for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) ld[i] = P.sph[i];
        char *end = reinterpret_cast<char *>(ld + n);
        if constexpr (kShadeLds != 0) {
            ShadeRec *ls = reinterpret_cast<ShadeRec *>(end);
            for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) ls[i] = P.shade[i];
            v.shd = ls;
            end += (static_cast<size_t>(n) * sizeof(ShadeRec) + 15) & ~size_t(15);
        }
        if (kMode == kBvh) {
            uint16_t *lnb = reinterpret_cast<uint16_t *>(end);
            for (uint32_t i = threadIdx.x; i < P.n_nbr; i += blockDim.x) lnb[i] = P.nbr[i];
            v.nbr = lnb;
            end += static_cast<size_t>(nbr_f4(P.n_nbr)) * sizeof(float4);
        }
        __syncthreads();
        v.sph = ld;
        v.end = reinterpret_cast<float4 *>(end);
    }
    return v;
}

// Per-pixel RNG children (copy_reset, camera.rs:269-272) of the shard's pixels, in
// shard order, by device jump-ahead: the persistent kernel refills lanes from it.
// One thread per run of kSeedRun pixels of a row: one jump-ahead to the run's
// first pixel, then the serial chain's own step per pixel (T^(p+1) = T(T^p)).
constexpr uint32_t kSeedRun = 8;
__global__ __launch_bounds__(kBlock) void rtw_seed_pixels(const KParams P) {
    const uint32_t runs = (P.W + kSeedRun - 1) / kSeedRun;
    const uint64_t t = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (t >= static_cast<uint64_t>(P.n_rows) * runs) return;
    const uint32_t lr = static_cast<uint32_t>(t / runs);
    const uint32_t x0 = static_cast<uint32_t>(t - static_cast<uint64_t>(lr) * runs) * kSeedRun;
    const uint32_t y = P.row_begin + lr * P.row_step;
    U128 s = jump_state(U128{P.seed_lo, P.seed_hi}, static_cast<uint64_t>(y) * P.W + x0, P.jump, P.jump_bits);
    U128 *out = P.seeds + static_cast<uint64_t>(lr) * P.W + x0;
    const uint32_t n = min(kSeedRun, P.W - x0);
    for (uint32_t k = 0; k < n; ++k) {
        out[k] = child_of(s);
        xs_step(s);
    }
}

// Shared words of the park queue (agent scope): relaxed atomics; payload stored
// write-through (sc1) by 8-byte atomic stores, then a drain, then the flag
// (cdna_hip_programming.md Guideline 16, recipe R1); consumers poll the flag
// relaxed and load the entry by sc1 loads (no stale copy of a reused slot).
// RTW_DIAG=2: the first time event k (0 hand-out, 1 park, 2 drain claim) happened to pixel pix
__device__ __forceinline__ void diag_event(const KParams &P, uint64_t npix, uint64_t pix, uint32_t k) {
    uint32_t *d = KP(diag);
    if (d && KP(diag_ev))
        atomicCAS(d + 2 * npix + 4 + 3 * pix + k, 0u, static_cast<uint32_t>(__builtin_amdgcn_s_memrealtime()) | 1u);
}
// s_setprio takes an immediate: a run-time level (0-3) by a wave-uniform switch
__device__ __forceinline__ void set_prio(uint32_t level) {
    switch (level) {
        case 0: __builtin_amdgcn_s_setprio(0); break;
        case 1: __builtin_amdgcn_s_setprio(1); break;
        case 2: __builtin_amdgcn_s_setprio(2); break;
        default: __builtin_amdgcn_s_setprio(3); break;
    }
}
__device__ __forceinline__ uint32_t ld_rlx(uint32_t *p) {
    return __hip_atomic_load((gu32 *)(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Idle-wait guard of the persistent kernel. A waiting lane gives up only when
// NOTHING has progressed anywhere for P.spin_guard ticks of the 100 MHz clock:
// no pixel handed out, finished or parked, no cursor wave retired (a sum of
// monotonic counters changes iff one of them moved). So a long render never
// trips it (pixels finish every few ms); a wave that does leave holds no entry
// it alone could finish -- a ticket it claimed stays published-but-unclaimed
// (flag 1) and the leftover launch (rtw_park_leftover) finishes it. Progress
// therefore never depends on every workgroup being resident at once.
__device__ __forceinline__ uint32_t progress_sig(const KParams &P) {
    return ld_rlx(P.park_count) + ld_rlx(P.pixels_done) + ld_rlx(P.pix_cursor) + ld_rlx(P.park_ctl_done);
}
struct SpinGuard {
    uint64_t t0;
    uint32_t sig;
    __device__ explicit SpinGuard(const KParams &P) : t0(__builtin_amdgcn_s_memrealtime()), sig(progress_sig(P)) {}
    __device__ bool expired(const KParams &P) {
        const uint32_t s = progress_sig(P);
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (s != sig) {
            sig = s, t0 = now;
            return false;
        }
        return now - t0 > P.spin_guard;
    }
};
// Park slot flags: 0 free, 1 published, 2 claimed by a group that finishes it.
constexpr uint32_t kSlotPublished = 1u, kSlotClaimed = 2u;
__device__ __forceinline__ void claim_slot(const KParams &P, uint32_t t) {
    __hip_atomic_store((gu32 *)(P.park_flag + t), kSlotClaimed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void publish_parked(const KParams &P, const Parked &q) {
    const uint32_t slot = atomicAdd(KP(park_count), 1u);
    const unsigned long long *w = reinterpret_cast<const unsigned long long *>(&q);
    gu64 *dst = (gu64 *)(KP(park) + slot);
#pragma unroll
    for (int j = 0; j < 8; ++j) __hip_atomic_store(dst + j, w[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store((gu32 *)(KP(park_flag) + slot), 1u, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// (t, index) minimum across a group of `kG` lanes (16 or 64): DPP butterflies
// inside each row of 16 (xor 1, xor 2, half-row mirror, row mirror), then
// cross-row exchanges. Every lane of the group ends with the same result.
template <int kCtrl>
__device__ __forceinline__ void dpp_min_step(double &bt, int &best) {
    const int ob = __builtin_amdgcn_update_dpp(-1, best, kCtrl, 0xf, 0xf, false);
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(bt), kCtrl, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(bt), kCtrl, 0xf, 0xf, false);
    const double ot = __hiloint2double(hi, lo);
    // selects, not a branch: every lane of the wave runs the step (a branch cost the
    // exec-mask bookkeeping of a divergent if on the drain's serial chain)
    const bool take = (ob >= 0) & ((best < 0) | (ot < bt) | ((ot == bt) & (ob < best)));  // rtw_accel::better
    bt = take ? ot : bt;
    best = take ? ob : best;
}
__device__ __forceinline__ void shfl_min_step(double &bt, int &best, int off) {
    const int ob = __shfl_xor(best, off);
    const double ot = __shfl_xor(bt, off);
    const bool take = (ob >= 0) & ((best < 0) | (ot < bt) | ((ot == bt) & (ob < best)));  // rtw_accel::better
    bt = take ? ot : bt;
    best = take ? ob : best;
}
template <uint32_t kG>
__device__ __forceinline__ void group_min(double &bt, int &best) {
    if constexpr (kG == 64) {
        // most segments leave at most one lane of the group with a hit (the scan spreads
        // a segment's 1-2 candidates over the lanes, and a miss leaves none): that lane's
        // record is the minimum -- broadcast it (wave-uniform branch) instead of six
        // reduction steps on the drain's serial chain
        const uint64_t hm = __ballot(best >= 0);
        if ((hm & (hm - 1ull)) == 0ull) {
            if (hm) {
                const int src = __builtin_ctzll(hm);
                best = __builtin_amdgcn_readlane(best, src);
                bt = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(bt), src),
                                      __builtin_amdgcn_readlane(__double2loint(bt), src));
            }
            return;
        }
    }
    dpp_min_step<0xB1>(bt, best);   // quad_perm [1,0,3,2]
    dpp_min_step<0x4E>(bt, best);   // quad_perm [2,3,0,1]
    dpp_min_step<0x141>(bt, best);  // row_half_mirror
    dpp_min_step<0x140>(bt, best);  // row_mirror
    if (kG >= 32) shfl_min_step(bt, best, 16);
    if (kG >= 64) shfl_min_step(bt, best, 32);
}

// Inside cut (rtw_accel.h): the segment starts inside `prev`, the sphere it last
// hit, and leaves it through the far root -- then only prev's list can come
// nearer: the scan's (best, bt) is the (t, index) minimum over prev and its list.
// Used by cooperative groups: every lane of the group holds the same path, so S's
// far root is formed on every lane, and lane j of the group
// tests entry j of S's list (at most rtw_accel::kMaxNbr <= kG entries) -- the list's
// exact tests run side by side instead of one after another on the pixel's serial
// chain -- then the group's (t, index) minimum. Same result as inside_hit.
template <uint32_t kG>
__device__ __forceinline__ bool inside_hit_group(const double4 *__restrict__ sph, const ShadeRec *__restrict__ shd,
                                                 const uint16_t *__restrict__ nbr, int prev, double ox,
                                                 double oy, double oz, double dx, double dy, double dz, double a,
                                                 int &best, double &bt, Tally &tl, uint32_t sub) {
    static_assert(rtw_accel::kMaxNbr <= kG, "one list entry per lane");
    if (prev < 0) return false;
    const uint32_t info = shd[prev].nbr;
    if (info == rtw_accel::kNbrNone) return false;
    const uint32_t n = info & 0xffu;  // group-uniform, <= kMaxNbr < 16
    // One pass for S and its list, side by side on the group's first n + 1 lanes (the
    // serial chain pays one sphere test instead of two in a row): lane j < n tests list
    // entry j as Sphere::hit does, lane n tests S as inside_far does -- the same
    // operations in the same order as those two functions, both roots formed -- then
    // S's verdict is read from lane n and the (t, index) minimum of lanes 0..15 (one
    // DPP row) is the group's. The candidates and the minimum are those of the serial
    // form, so the result is too.
    static_assert(rtw_accel::kMaxNbr < 16u, "the list and S fit one DPP row");
    {
        uint32_t i = static_cast<uint32_t>(prev);
        if (sub < n) {
            uint32_t e = (info >> 8) + sub;
            asm volatile("" : "+v"(e));  // formed here (see below)
            i = nbr[e];
        }
        const double4 T = sph[i];
        const double ocx = ox - T.x, ocy = oy - T.y, ocz = oz - T.z;
        const double rr = T.w * T.w;
        const double hb = ocx * dx + ocy * dy + ocz * dz;
        const double c = (ocx * ocx + ocy * ocy + ocz * ocz) - rr;
        const double disc = hb * hb - a * c;
        const double sq = __builtin_sqrt(disc);
        const double tn = (-sq - hb) / a, tf = (sq - hb) / a;
        // lane n (S): inside_far's tests; lanes < n: sphere_hit_f64's
        const bool s_ok = (c <= 3. * rr) && !(hb >= 0. && c >= 0.) && disc >= 0. && !(tn >= 0.01) && tf >= 0.01;
        int okn;
        if constexpr (kG == 64) {
            okn = __builtin_amdgcn_readlane(static_cast<int>(s_ok), __builtin_amdgcn_readfirstlane(static_cast<int>(n)));
        } else {
            okn = __shfl(static_cast<int>(s_ok), static_cast<int>(n + (threadIdx.x & 63u & ~(kG - 1u))));
        }
        if (!okn) return false;
        if (sub == 0) tl.inside += 1u, tl.ntest += 1u + n;
        const double t = tn >= 0.01 ? tn : tf;
        const bool cand = sub < n ? (disc >= 0. && t >= 0.01) : sub == n;
        bt = sub == n ? tf : t;
        best = cand ? static_cast<int>(i) : -1;
        if constexpr (kG == 64) {  // S alone (no list entry hit): its far root, broadcast
            if (__ballot(cand) == (1ull << n)) {
                best = prev;
                bt = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(bt), __builtin_amdgcn_readfirstlane(static_cast<int>(n))),
                                      __builtin_amdgcn_readlane(__double2loint(bt), __builtin_amdgcn_readfirstlane(static_cast<int>(n))));
                return true;
            }
        }
        dpp_min_step<0xB1>(bt, best);   // quad_perm [1,0,3,2]
        dpp_min_step<0x4E>(bt, best);   // quad_perm [2,3,0,1]
        dpp_min_step<0x141>(bt, best);  // row_half_mirror
        dpp_min_step<0x140>(bt, best);  // row_mirror
        if (kG > 16) {  // every lane of the group takes row 0's result
            const int src = static_cast<int>(threadIdx.x & 63u & ~(kG - 1u));
            best = __builtin_amdgcn_readlane(best, src);
            bt = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(bt), src),
                                  __builtin_amdgcn_readlane(__double2loint(bt), src));
        }
        return true;
    }
    const double4 S = sph[prev];
    double t;
    if (!rtw_accel::inside_far(ox, oy, oz, dx, dy, dz, a, S.x, S.y, S.z, S.w * S.w, t)) return false;
    if (sub == 0) tl.inside += 1u, tl.ntest += 1u + n;
    best = prev, bt = t;
    if (n == 0) return true;
    if (sub < n) {
        // the entry's address formed here: hoisted out of the pixel's loop, the
        // compiler kept it through the whole chain and spilled it to scratch
        uint32_t e = (info >> 8) + sub;
        asm volatile("" : "+v"(e));
        const uint32_t i = nbr[e];
        const double4 T = sph[i];
        if (rtw_accel::sphere_hit_f64(ox, oy, oz, dx, dy, dz, a, T.x, T.y, T.z, T.w * T.w, t) &&
            rtw_accel::better(t, i, bt, best))
            bt = t, best = static_cast<int>(i);
    }
    group_min<kG>(bt, best);
    return true;
}

// A run of total internal reflections inside sphere S, traced by a whole drain wave
// (the long serial chains of the strong split: 66 % of row 308's segments are such
// bounces inside the big glass sphere, 4.2 per run, profiles/r05_misc/
// trace_pixel_567_308.log). The path has just reflected totally inside S and S's
// great-circle forward failed, so the generic loop would take, bounce after bounce,
// the inside cut (S's far root beside its list, inside_hit_group), the dielectric
// scatter's reflection (shade) and skip the forward test. Here S's record, its
// shading row and each lane's list entry stay in registers for the run, and a
// bounce is exactly those operations, in the same order on the same values:
// a = |d|^2, inside_hit_group's roots and (t, index) minimum, the hit point,
// (p - c) / r, front, unit(d), cos_t, tir_exceeds, the reflection. The run hands the
// path back, untouched for the bounce in question, as soon as anything else could
// happen: the inside cut does not apply, a list sphere is hit first (the run's usual
// end: the ray leaves through the small glass sphere that overlaps S), the hit is a
// front face, the reflection is partial (a Schlick draw), or the next bounce would
// reach the depth cap. Returns the bounces traced (segments).
__device__ __forceinline__ uint32_t tir_run_64(const SceneView &sv, int S_idx, Path &p, uint32_t max_depth,
                                               Tally &tl) {
    const uint32_t lane = __lane_id();
    const uint32_t info = sv.shd[S_idx].nbr;
    if (info == rtw_accel::kNbrNone) return 0u;
    const uint32_t n = info & 0xffu;  // list entries, < 16
    const uint32_t nl = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(n)));
    const double4 S = sv.sph[S_idx];
    const double ratio = sv.shd[S_idx].p;  // back face: ratio = ir (materials.rs:86)
    // lane j < n: list entry j (inside_hit_group's lane roles); lane n and above: S
    uint32_t i = static_cast<uint32_t>(S_idx);
    if (lane < n) {
        uint32_t e = (info >> 8) + lane;
        asm volatile("" : "+v"(e));
        i = sv.nbr[e];
    }
    const double4 T = sv.sph[i];
    const double rrT = T.w * T.w;
    const uint64_t only_s = 1ull << nl;
    uint32_t k = 0;
    while (p.depth + 1u < max_depth) {
        const double a = p.dx * p.dx + p.dy * p.dy + p.dz * p.dz;
        // inside_hit_group (kG = 64), the same operations per lane
        const double ocx = p.ox - T.x, ocy = p.oy - T.y, ocz = p.oz - T.z;
        const double hb = ocx * p.dx + ocy * p.dy + ocz * p.dz;
        const double c = (ocx * ocx + ocy * ocy + ocz * ocz) - rrT;
        const double disc = hb * hb - a * c;
        const double sq = __builtin_sqrt(disc);
        const double tn = (-sq - hb) / a, tf = (sq - hb) / a;
        const bool s_ok = (c <= 3. * rrT) && !(hb >= 0. && c >= 0.) && disc >= 0. && !(tn >= 0.01) && tf >= 0.01;
        const double t = tn >= 0.01 ? tn : tf;
        const bool cand = lane < n ? (disc >= 0. && t >= 0.01) : lane == n;
        if (!__builtin_amdgcn_readlane(static_cast<int>(s_ok), nl)) break;  // no inside cut: the scan
        double bt;
        if (__ballot(cand) == only_s) {
            bt = readlane_f64(tf, nl);
        } else {  // a list sphere has an accepted root too (inside an overlap): the minimum
            int b = cand ? static_cast<int>(i) : -1;
            bt = lane == n ? tf : t;
            dpp_min_step<0xB1>(bt, b);   // quad_perm [1,0,3,2]
            dpp_min_step<0x4E>(bt, b);   // quad_perm [2,3,0,1]
            dpp_min_step<0x141>(bt, b);  // row_half_mirror
            dpp_min_step<0x140>(bt, b);  // row_mirror
            if (__builtin_amdgcn_readlane(b, 0) != S_idx) break;  // another sphere is hit: the generic loop
            bt = readlane_f64(bt, 0u);
        }
        // shade (dielectric): unit(dir), the hit record, the reflection
        double vx = p.dx, vy = p.dy, vz = p.dz;
        rtw_num::div3(vx, vy, vz, __builtin_sqrt(a));
        const double px = p.dx * bt + p.ox, py = p.dy * bt + p.oy, pz = p.dz * bt + p.oz;
        double nx = px - S.x, ny = py - S.y, nz = pz - S.z;
        rtw_num::div3(nx, ny, nz, S.w);
        if ((p.dx * nx + p.dy * ny + p.dz * nz) < 0.) break;  // a front face: the generic loop
        nx = -nx, ny = -ny, nz = -nz;
        const double cos_t = fmin((-vx) * nx + (-vy) * ny + (-vz) * nz, 1.);
        if (!rtw_num::tir_exceeds(ratio, 1.0 - cos_t * cos_t, 1.)) break;  // Schlick's draw: the generic loop
        const double dt = vx * nx + vy * ny + vz * nz;
        p.dx = vx - (nx * dt) * 2., p.dy = vy - (ny * dt) * 2., p.dz = vz - (nz * dt) * 2.;
        p.ox = px, p.oy = py, p.oz = pz;
        ++p.depth;  // p.prev stays S
        ++k;
        if (lane == 0) tl.inside += 1u, tl.ntest += 1u + n;
    }
    return k;
}

// Phase 2: the parked pixels, kG lanes per pixel. Persistent groups take pixels
// in park order (the heaviest parked first) from an atomic cursor. Scene::hit is
// split across the group: lane j filters spheres j, j + kG, ... against the
// LDS-staged pass-1 records, runs the exact f64 test on its candidates, then
// the group takes the (t, index) minimum. Every lane of a group then runs the
// identical scatter on the identical RNG state.
// One parked pixel finished by a group of kG lanes (all lanes of the group run
// the identical path; lane j of the group filters spheres j, j + kG, ...).
// Returns the pixel's segments on the group's first lane (0 on the others).
template <uint32_t kG>
__device__ __forceinline__ uint32_t coop_pixel(const KParams &P, const SceneView &sv,
                                               const float4 *__restrict__ filt, uint32_t fsh, const Parked &q,
                                               uint64_t col, Tally &tl, Stamps &stp) {
    if constexpr (kG == 64) {
        // one group per wave: the spill column is wave-uniform -- in SGPRs, its offset
        // col * stride is scalar arithmetic (held in a VGPR, the compiler spilled it to
        // scratch and reloaded it at every drained segment behind a vmcnt(0) wait)
        col = (static_cast<uint64_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(col >> 32))) << 32) |
              static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(col)));
    }
    const uint32_t sub = threadIdx.x & (kG - 1u);
    const uint32_t n = P.n_sph;
    const double4 *sph = sv.sph;
    const uint32_t y = P.row_begin + q.lr * P.row_step;
    PixelState ps;
    ps.rng = U128{q.rng_lo, q.rng_hi};
    ps.k = q.k;
    ps.ar = q.ar, ps.ag = q.ag, ps.ab = q.ab;
    // (the pixel index is formed where the diagnostics use it: held from here to the
    // end of the pixel, it was spilled to scratch)
    if (sub == 0) diag_event(P, static_cast<uint64_t>(P.n_rows) * P.W, static_cast<uint64_t>(q.lr) * P.W + q.x, 2);
    // scenes of up to kCoopRegRec * kG spheres: the lane's pass-1 records live in
    // registers for the whole pixel (no LDS round trip on the serial chain)
    constexpr uint32_t kCoopRegRec = 8;
    const bool rec_in_regs = n <= kCoopRegRec * kG;
    float4 rr[kCoopRegRec];
    if (rec_in_regs) {
        // the record addresses are formed per pixel from a laundered lane id: hoisted
        // out of the drain loop, the compiler kept all eight through it and spilled them
        uint32_t sl = sub;
        asm volatile("" : "+v"(sl));
#pragma unroll
        for (uint32_t j = 0; j < kCoopRegRec; ++j) rr[j] = filt[min(sl + j * kG, n - 1u) << fsh];
    }
    auto hit = [&](double ox, double oy, double oz, double dx, double dy, double dz, double a, int prev,
                   double &bt) -> int {
        int best = -1;
        bt = 0.;
        // inside cut: every lane of the group holds the same path, so the branch
        // is group-uniform and the lanes run the (short) list redundantly
        if (inside_hit_group<kG>(sph, sv.shd, sv.nbr, prev, ox, oy, oz, dx, dy, dz, a, best, bt, tl, sub))
            return best;
        const Seg32 g(ox, oy, oz, dx, dy, dz, a, true);
        STAMP(0);  // coop: loop back + segment setup (Seg32)
        if (rec_in_regs) {
            uint32_t mask = 0;
#pragma unroll
            for (uint32_t j = 0; j < kCoopRegRec; ++j) {
                const uint32_t i = sub + j * kG;
                mask |= static_cast<uint32_t>((i < n) & (!g.fast | g.pass(rr[j]))) << j;
            }
            STAMP(5);
            while (mask) {
                const uint32_t j = static_cast<uint32_t>(__builtin_ctz(mask));
                mask &= mask - 1u;
                ++tl.ntest;
                exact_test(sph, sub + j * kG, ox, oy, oz, dx, dy, dz, a, best, bt);
            }
            STAMP(2);
            group_min<kG>(bt, best);
            return best;
        }
        for (uint32_t base = 0; base < n; base += 32u * kG) {
            uint32_t mask = 0;  // bit j: sphere base + sub + j*kG is a candidate
            const uint32_t jn = min(32u, (n - base + kG - 1u) / kG);  // group-uniform
            // branch-free: every load is issued before the first test needs it
#pragma unroll 8
            for (uint32_t j = 0; j < jn; ++j) {
                const uint32_t i = base + sub + j * kG;
                const float4 rec = filt[min(i, n - 1u) << fsh];
                mask |= static_cast<uint32_t>((i < n) & (!g.fast | g.pass(rec))) << j;
            }
            STAMP(5);  // coop: segment setup + filter
            while (mask) {
                const uint32_t j = static_cast<uint32_t>(__builtin_ctz(mask));
                mask &= mask - 1u;
                ++tl.ntest;
                exact_test(sph, base + sub + j * kG, ox, oy, oz, dx, dy, dz, a, best, bt);
            }
            STAMP(2);  // coop: exact tests
        }
        group_min<kG>(bt, best);
        return best;
    };
    uint32_t s = 0, trapped = 0;
    // the lane-parallel replay (trap_forward<true>, unit_vec_round) needs the whole wave
    // on one path with one RNG state: only 64-lane groups take it
    constexpr bool kWaveReplay = kG == 64;
    static_assert(!kWaveReplay || kG == 64, "the trapped-path replay runs on whole waves only");
    if constexpr (kWaveReplay) {
        auto run = [&](Path &p, int S_idx) { return tir_run_64(sv, S_idx, p, P.max_depth, tl); };
        trace_samples<true, true>(P, sv, q.x, y, KP(spill_b), col, ps, 0xffffffffu, s, stp, hit, &trapped, run);
    } else {
        trace_samples<true, false>(P, sv, q.x, y, KP(spill_b), col, ps, 0xffffffffu, s, stp, hit, &trapped);
    }
    if (sub == 0) tl.trap += trapped;
    if (sub == 0) {
        write_pixel(P, q.x, q.lr, ps);
        uint32_t *diag = KP(diag);
        if (diag) {
            const uint64_t pix = static_cast<uint64_t>(q.lr) * P.W + q.x;
            atomicAdd(diag + 2 * pix, s);
            __hip_atomic_store((gu32 *)(diag + 2 * pix + 1),
                               static_cast<uint32_t>(__builtin_amdgcn_s_memrealtime()), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        return s;
    }
    return 0;
}

// pass-1 records staged in LDS after the scene view (cooperative groups scan them)
template <bool kLds>
__device__ __forceinline__ const float4 *stage_filt(const KParams &P, float4 *lf) {
    if (!kLds) return P.filt;
    for (uint32_t i = threadIdx.x; i < P.n_sph; i += blockDim.x) lf[i] = P.filt[i];
    __syncthreads();
    return lf;
}

// Hand-out order by estimated cost. rtw_cost_probe traces kProbeSamples of every
// pixel's lattice (spread over the lattice) on a COPY of the pixel's RNG -- the
// render itself is untouched -- and records the pixel's segment count. "Hot"
// pixels (>= kHotSegs probe segments: long serial chains) are ordered one by one
// by their own cost; the others by the cost of their 8x8 tile. Units are
// bucketed by cost per sample (descending) and laid out in the order the
// persistent kernel hands pixels out: hot pixels and expensive tiles start first
// (a chain started late ends late), the cheapest tiles fill the drain, and lanes
// refilled together get neighbouring pixels (coherent rays).
constexpr uint32_t kProbeSamples = 2;
constexpr uint32_t kHotSegs = kProbeSamples * 10;  // probe segments: >= 10 per sample
constexpr uint32_t kProbeCap = 8;  // probe segments per sample at most
constexpr uint32_t kCostBuckets = 256;
constexpr uint32_t kOrderTile = 8;
struct TileGrid {
    uint32_t tx, ty;
    __host__ __device__ TileGrid(const KParams &P)
        : tx((P.W + kOrderTile - 1) / kOrderTile), ty((P.n_rows + kOrderTile - 1) / kOrderTile) {}
    __host__ __device__ uint32_t count() const { return tx * ty; }
    __device__ uint32_t of(uint32_t x, uint32_t lr) const { return (lr / kOrderTile) * tx + x / kOrderTile; }
    __device__ uint32_t pixels(const KParams &P, uint32_t t) const {
        const uint32_t bx = (t % tx) * kOrderTile, by = (t / tx) * kOrderTile;
        return min(kOrderTile, P.W - bx) * min(kOrderTile, P.n_rows - by);
    }
};
__device__ __forceinline__ uint32_t cost_bucket(uint32_t segs, uint32_t pixels) {
    const uint32_t per = static_cast<uint32_t>((8ull * segs) / (static_cast<uint64_t>(pixels) * kProbeSamples));
    return kCostBuckets - 1u - min(per, kCostBuckets - 1u);  // 1/8 segment per sample
}
// Persistent: one 768-thread workgroup per CU stages the scene once and strides
// over the pixels (a 256-thread block per 256 pixels staged ~100 KB of scene for
// each and ran at one workgroup per CU); the walk stack lives in per-lane LDS
// columns at P.lane_lds_off (kLds) instead of scratch memory.
constexpr uint32_t kProbeBlock = 768;
// SplitMix64's finaliser (Steele, Lea & Flood), for the probe's per-pixel xorshift state
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ U128 probe_state(uint64_t seed_lo, uint64_t seed_hi, uint64_t gpix) {
    const uint64_t a = seed_lo + (gpix + 1ull) * 0x9e3779b97f4a7c15ull;
    const U128 r{mix64(a), mix64(a ^ seed_hi ^ 0x6a09e667f3bcc909ull)};
    return (r.lo | r.hi) ? r : U128{1ull, 0ull};  // xorshift's state must not be zero
}
template <bool kLds>
__global__ __launch_bounds__(kProbeBlock) void rtw_cost_probe(const KParams P) {
    extern __shared__ __attribute__((aligned(16))) double4 lds_sph[];
    const SceneView sv = stage_scene<kLds, kBvh>(P, lds_sph);
    uint16_t *scol = reinterpret_cast<uint16_t *>(reinterpret_cast<char *>(lds_sph) + P.lane_lds_off) + threadIdx.x;
    // probe_sub > 1: one probed pixel per probe_sub x probe_sub block stands for the
    // block in its tile's cost (the others keep pcost 0: ordered with their tile).
    // Hand-out order only, never the image. The estimate is biased when probe_sub
    // does not divide the 8x8 order tile (a straddling block puts its whole weight on
    // the probed pixel's tile) and a hot probed pixel counts 1, not its block's
    // weight; the default (1) is exact, and RTW_PROBE_SUB > 1 stays an A/B knob
    // (2: neutral, 3: +18 %, profiles/r02_misc/knob_probe_sub.log).
    const uint32_t sub = P.probe_sub > 1u ? P.probe_sub : 1u;
    const uint32_t wq = (P.W + sub - 1u) / sub, hq = (P.n_rows + sub - 1u) / sub;
    const uint64_t nq = static_cast<uint64_t>(wq) * hq;
    Tally tl;
    Stamps stp;
    for (uint64_t j = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; j < nq;
         j += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
        const uint32_t qr = static_cast<uint32_t>(j / wq), qx = static_cast<uint32_t>(j - static_cast<uint64_t>(qr) * wq);
        const uint32_t lr = qr * sub, x = qx * sub;
        const uint64_t i = static_cast<uint64_t>(lr) * P.W + x;
        const uint32_t wgt = min(sub, P.W - x) * min(sub, P.n_rows - lr);
        // the probe's own stream (a hash of the render seed and the global pixel index),
        // not the pixel's RNG child: the estimate is as good, and the probe no longer
        // waits for rtw_seed_pixels, which runs beside it on the session's second stream
        auto probe_pixel = [&](uint32_t px_, uint32_t lr_) {
            const PixelLoc pl(P, px_, P.row_begin + lr_ * P.row_step);
            U128 rng = probe_state(P.seed_lo, P.seed_hi, static_cast<uint64_t>(P.row_begin + lr_ * P.row_step) * P.W + px_);
            uint32_t segs = 0;
            for (uint32_t q = 0; q < kProbeSamples && P.max_depth > 0; ++q) {
                Path p;
                gen_ray(P, pl, (q * P.n_off) / kProbeSamples, rng, p, stp);
                for (;;) {  // one path, at most probe_cap segments (only counted: no attenuation rows kept)
                    ++segs;
                    const double a = p.dx * p.dx + p.dy * p.dy + p.dz * p.dz;
                    double bt = 0.;
                    const int best = bvh_hit<kLds, kProbeBlock>(P, sv, p.ox, p.oy, p.oz, p.dx, p.dy, p.dz, a, p.prev, bt, tl, stp, scol);
                    if (best < 0 || p.depth + 1 >= P.max_depth || p.depth + 1 >= P.probe_cap) break;
                    double cr, cg, cb;
                    shade(P, sv.sph, sv.shd, best, bt, a, p, rng, nullptr, 0, 0, cr, cg, cb, stp);
                    p.stk.clear();  // the register slots never fill, whatever the cap
                }
            }
            return segs;
        };
        const uint32_t segs = probe_pixel(x, lr);
        P.pcost[i] = segs;
        const TileGrid tg(P);
        const bool hot = segs >= P.hot_segs;
        const uint32_t key = (hot ? tg.count() : 0u) + tg.of(x, lr);
        const uint32_t val = hot ? 1u : segs * wgt;
        const uint32_t lane = __lane_id();
        for (uint64_t todo = __ballot(1); todo;) {  // the active lanes, one tile word per trip
            const uint32_t leader = static_cast<uint32_t>(__builtin_ctzll(todo));
            const uint32_t k = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(key), leader));
            const uint64_t grp = __ballot(key == k) & todo;
            uint32_t v = 0;  // the group's values by lane reads (only active lanes are read)
            for (uint64_t g = grp; g; g &= g - 1ull)
                v += static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(val), __builtin_ctzll(g)));
            if (lane == leader) atomicAdd(P.cost + k, v);
            todo &= ~grp;
        }
    }
}
// Per-wave aggregation of histogram atomics: neighbouring tiles fall in few buckets,
// so one atomic per distinct bucket of the wave instead of one per tile (the 256
// counters were contended: 46-48 us per kernel and frame). Returns the base the
// bucket's atomic returned plus the counts of the lanes below in the same bucket.
__device__ __forceinline__ uint32_t hist_add_wave(uint32_t *hist, uint32_t key, uint32_t val, bool on) {
    const uint32_t lane = __lane_id();
    uint32_t mine = 0;
    for (uint64_t todo = __ballot(on); todo;) {  // wave-uniform trips, one bucket each
        const uint32_t leader = static_cast<uint32_t>(__builtin_ctzll(todo));
        const uint32_t k = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(key), leader));
        const uint64_t grp = __ballot(on && key == k) & todo;
        uint32_t tot = 0, below = 0;
        for (uint64_t g = grp; g; g &= g - 1ull) {
            const uint32_t l = static_cast<uint32_t>(__builtin_ctzll(g));
            const uint32_t v = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(val), l));
            below += l < lane ? v : 0u;
            tot += v;
        }
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(hist + k, tot);
        base = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(base), leader));
        if ((grp >> lane) & 1ull) mine = base + below;
        todo &= ~grp;
    }
    return mine;
}
// per tile: cost bucket of its non-hot pixels and their count into the histogram
__global__ __launch_bounds__(kBlock) void rtw_cost_bucket(const KParams P) {
    const TileGrid tg(P);
    const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
    const bool in = t < tg.count();
    const uint32_t np = in ? tg.pixels(P, t) - P.cost[tg.count() + t] : 0u;
    const uint32_t b = np ? cost_bucket(P.cost[t], np) : 0u;
    if (in) P.cost[t] = b;
    hist_add_wave(P.cost_hist, b, np, np != 0u);
}
// per hot pixel: its own bucket into the histogram
__global__ __launch_bounds__(kBlock) void rtw_cost_hot_bucket(const KParams P) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (i >= static_cast<uint64_t>(P.n_rows) * P.W || P.pcost[i] < P.hot_segs) return;
    atomicAdd(P.cost_hist + cost_bucket(P.pcost[i], 1u), 1u);
}
// exclusive prefix sums of pixel counts over the buckets -> bucket write cursors
__global__ void rtw_cost_scan(const KParams P) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        uint32_t acc = 0;
        for (uint32_t b = 0; b < kCostBuckets; ++b) {
            const uint32_t c = P.cost_hist[b];
            P.cost_hist[b] = acc;
            acc += c;
        }
    }
}
// per tile: the base of its non-hot pixels in the order (tiles of one bucket in any order)
__global__ __launch_bounds__(kBlock) void rtw_cost_place(const KParams P) {
    const TileGrid tg(P);
    const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
    const bool in = t < tg.count();
    const uint32_t np = in ? tg.pixels(P, t) - P.cost[tg.count() + t] : 0u;
    const uint32_t base = hist_add_wave(P.cost_hist, in ? P.cost[t] : 0u, np, np != 0u);
    if (np) P.cost[t] = base;
}
// per hot pixel: its slot in the order
__global__ __launch_bounds__(kBlock) void rtw_cost_hot_place(const KParams P) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (i >= static_cast<uint64_t>(P.n_rows) * P.W || P.pcost[i] < P.hot_segs) return;
    P.order_map[atomicAdd(P.cost_hist + cost_bucket(P.pcost[i], 1u), 1u)] = static_cast<uint32_t>(i);
}
// one wave per tile (lane = row-major rank in the tile): order[tile base + rank
// among the tile's non-hot pixels] = pixel
__global__ __launch_bounds__(kBlock) void rtw_cost_scatter(const KParams P) {
    const TileGrid tg(P);
    const uint32_t t = (blockIdx.x * kBlock + threadIdx.x) / 64u, r = threadIdx.x & 63u;
    if (t >= tg.count()) return;  // wave-uniform
    const uint32_t bx = (t % tg.tx) * kOrderTile, by = (t / tg.tx) * kOrderTile;
    const uint32_t wx = min(kOrderTile, P.W - bx), wy = min(kOrderTile, P.n_rows - by);
    const uint32_t x = bx + r % wx, lr = by + r / wx;
    const uint64_t i = static_cast<uint64_t>(lr) * P.W + x;
    const bool mine = r < wx * wy && P.pcost[i] < P.hot_segs;
    const uint64_t m = __ballot(mine);
    if (mine) P.order_map[P.cost[t] + static_cast<uint32_t>(__popcll(m & ((1ull << r) - 1ull)))] = static_cast<uint32_t>(i);
}

// Phase 1, persistent form, with the heavy tail folded in. Every lane of a
// cursor wave runs one pixel at a time and, when the pixel completes, takes the
// next pixel of the shard from a global cursor (one atomic per wave per refill).
// A pixel whose cost runs away -- more than P.rate_x segments per sample after
// P.rate_k samples, or P.seg_budget segments in all -- parks at a sample
// boundary in the park queue (published write-through, Guideline 16 R1). Parked
// pixels are finished by 16-lane cooperative groups (coop_pixel): from the start
// by the first P.heavy_per_block waves of every workgroup, which run at raised
// issue priority and do nothing else, and at the end by every cursor wave whose
// cursor ran dry. Groups claim queue tickets in order and wait for a claimed
// ticket to be published; they stop once every cursor wave has signalled that it
// parks no more and their ticket lies past the final queue length.
template <bool kLds, int kMode, uint32_t kThreads, uint32_t kCoopG = 16>
__global__ __launch_bounds__(kThreads) void rtw_render_persist(const KParams P) {
    extern __shared__ __attribute__((aligned(16))) double4 lds_sph[];
    if (kWgDone && threadIdx.x == 0)
        *reinterpret_cast<uint32_t *>(reinterpret_cast<char *>(lds_sph) + P.lane_lds_off + lane_lds_area(kThreads)) = 0u;
    const SceneView sv = stage_scene<kLds, kMode>(P, lds_sph);
    if (kWgDone && !kLds) __syncthreads();  // (kLds: stage_scene's barrier orders the zero)
    // pass-1 records after the scene view: after the inside-cut lists (BVH) or the
    // shading records
    // BVH scenes in LDS: the leaves (indexed by sphere, every sphere's record, rtw_accel.h)
    // are the pass-1 records, at a stride of 2 float4; else staged after the scene
    constexpr bool kLeafFilt = kLds && kMode == kBvh;
    constexpr uint32_t fsh = kLeafFilt ? 1u : 0u;
    const float4 *filt = kLeafFilt ? sv.leaves : stage_filt<kLds>(P, sv.end);
    // per-lane LDS areas (lane_lds_bytes): the pixel's running sum (3 f64 columns,
    // read and written once per sample) and the BVH walk scratch (kScratch u16
    // columns) -- state that would otherwise hold ~12 VGPRs through the walk
    double *acc = reinterpret_cast<double *>(lds_sph) + P.lane_lds_off / 8u + threadIdx.x;
    uint16_t *lane_stk = reinterpret_cast<uint16_t *>(acc - threadIdx.x + 3u * kThreads);
    uint4 *spec_lds = reinterpret_cast<uint4 *>(lane_stk + rtw_accel::kScratch * kThreads) + threadIdx.x;
    const double4 *sph = sv.sph;
    Tally tl;
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t npix = static_cast<uint64_t>(P.n_rows) * P.W;
    const uint64_t stride = P.spill_stride;
    // spill column of this lane for the whole launch: consecutive lanes of a wave
    // share L2 lines, and the live columns stay dense
    // re-formed at each use from the workgroup id and the lane's thread id (laundered
    // through an empty asm so it is not one 64-bit value held across the whole
    // persistent loop: the compiler spilled it to scratch, round 5's private segment)
    auto gid = [&]() -> uint64_t {
        uint32_t t = threadIdx.x;
        asm volatile("" : "+v"(t));
        return static_cast<uint64_t>(blockIdx.x) * kThreads + t;
    };
    const bool heavy_wave = (threadIdx.x >> 6) < P.heavy_per_block;

    Stamps stp_unused, stp;  // stp: cursor-loop sections (RTW_STAMPS builds only)
    double seg_sa = 0.;  // sqrt(a) of the current segment (BVH hit), reused by the scatter
    auto hit = [&](double ox, double oy, double oz, double dx, double dy, double dz, double a, int prev,
                   double &bt) -> int {
        if constexpr (kMode == kBvh) {
            return bvh_hit<true, kThreads>(P, sv, ox, oy, oz, dx, dy, dz, a, prev, bt, tl, stp,
                                           lane_stk + threadIdx.x, &seg_sa);
        } else {
            const Seg32 g(ox, oy, oz, dx, dy, dz, a, kMode == kScanF32);
            return scan_hit(P, sph, g, ox, oy, oz, dx, dy, dz, a, bt, tl);
        }
    };
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    if (P.diag && blockIdx.x == 0 && threadIdx.x == 0)  // diagnostic: launch start after the pixels
        P.diag[2 * npix] = static_cast<uint32_t>(t_start);
    // priority waves: drain parked pixels from the start; with P.join_at they leave
    // for the cursor once it has handed out join_at pixels and no published entry is
    // unclaimed (claims by compare-and-swap, so a leaving wave holds no ticket that
    // may never be published), and then count as cursor waves
    bool cursor_wave = !heavy_wave;
    if (heavy_wave) {
        set_prio(KP(heavy_prio));
        const uint32_t sub = threadIdx.x & (kCoopG - 1u);
        const int gl = static_cast<int>(lane & ~(kCoopG - 1u));
        uint32_t cseg = 0;
        while (P.join_at != 0xffffffffu) {
            uint32_t t = 0, state = 0;  // 1: ticket t, 2: join the cursor
            if (sub == 0) {
                SpinGuard guard(P);
                for (uint32_t spins = 0;; ++spins) {
                    const uint32_t c = ld_rlx(P.park_cursor), n = ld_rlx(P.park_count);
                    if (c < n) {
                        if (atomicCAS(P.park_cursor, c, c + 1u) == c) {
                            t = c;
                            while (ld_rlx(P.park_flag + t) != kSlotPublished) __builtin_amdgcn_s_sleep(2);
                            claim_slot(P, t);
                            state = 1;
                            break;
                        }
                        continue;
                    }
                    if (ld_rlx(P.pix_cursor) >= P.join_at) {
                        state = 2;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(16);
                    if ((spins & 255u) == 255u && guard.expired(P)) {
                        atomicAdd(&P.counters[7], 1ull);  // nothing moves: join the cursor
                        state = 2;
                        break;
                    }
                }
            }
            t = __shfl(t, gl);
            state = __shfl(state, gl);
            if (state == 2) {
                cursor_wave = true;
                __builtin_amdgcn_s_setprio(0);
                break;
            }
            Parked q;
            unsigned long long *w = reinterpret_cast<unsigned long long *>(&q);
            gu64 *src = (gu64 *)(P.park + t);
#pragma unroll
            for (int j = 0; j < 8; ++j) w[j] = __hip_atomic_load(src + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // per-pixel issue priority (RTW_PRIO_SPLIT): the long chains at the waves'
            // priority, the others at the cursor waves' (0)
            if (P.prio_split) set_prio(q._pad >= P.prio_split ? KP(heavy_prio) : 0u);
            cseg += coop_pixel<kCoopG>(P, sv, filt, fsh, q, gid() & ~static_cast<uint64_t>(kCoopG - 1u), tl, stp_unused);
            if (sub == 0) atomicAdd(P.park_processed, 1u);
        }
        tl.seg += cseg;
    }
    if (cursor_wave) {
        bool need = true;  // lane holds no pixel
        bool dry = false;  // wave-uniform: the cursor ran dry
        bool endgame = false;  // wave-uniform: latched endgame (P.endgame)
        uint32_t wave_it = 0;  // wave-uniform: iterations of this wave's cursor loop
        uint32_t x = 0, lr = 0, pseg = 0;
        bool spec = false;  // spec_lds holds the state the lane's next unit vector draws from
        uint64_t pix = 0;
        PixelState ps;
        Path p;
        for (;;) {
            {  // the wave's first active lane counts the wave-level iteration
                const uint64_t exm = __builtin_amdgcn_read_exec();
                tl.witer += static_cast<uint32_t>(__builtin_ctzll(exm) == static_cast<int>(lane));
            }
            bool dry_now = false;
            if (need && !dry) {  // refill: one atomic for the wave's idle lanes
                const uint64_t m = __ballot(1);
                const uint32_t rank = static_cast<uint32_t>(__popcll(m & ((1ull << lane) - 1ull)));
                uint32_t base = 0, take = static_cast<uint32_t>(__popcll(m));
                if (const uint32_t cap = KP(wave_cap)) {  // RTW_WAVE_CAP (A/B): at most cap pixels per wave
                    const uint32_t live = 64u - take;
                    take = cap > live ? min(take, cap - live) : 0u;
                }
                if (rank == 0 && take) base = atomicAdd(KP(pix_cursor), take);
#ifdef RTW_WALK_DIAG  // diagnostic build: device-scope atomics of the cursor loop
                if (rank == 0) atomicAdd(&P.counters[16], 1ull);
#endif
                base = __shfl(base, __ffsll(static_cast<unsigned long long>(m)) - 1);
                const uint64_t ticket = static_cast<uint64_t>(base) + rank;
                if (rank >= take) {
                    // over the wave's cap (RTW_WAVE_CAP): stays idle
                } else if (ticket < npix) {
                    // hand-out order: by descending estimated cost (P.order_map,
                    // rtw_cost_probe), so the cheapest pixels fill the drain; else
                    // rows bottom-up when P.order == 1, or row-major
                    const uint32_t *order_map = KP(order_map);
                    if (order_map) {
                        const uint64_t q = KP(spread_q);
                        const uint64_t pos = ticket < 64u * q ? (ticket & 63u) * q + (ticket >> 6) : ticket;
                        pix = order_map[pos];
                        lr = static_cast<uint32_t>(pix / P.W);
                        x = static_cast<uint32_t>(pix - static_cast<uint64_t>(lr) * P.W);
                    } else {
                        const uint32_t tr = static_cast<uint32_t>(ticket / P.W);
                        x = static_cast<uint32_t>(ticket - static_cast<uint64_t>(tr) * P.W);
                        lr = P.order ? P.n_rows - 1u - tr : tr;
                        pix = static_cast<uint64_t>(lr) * P.W + x;
                    }
                    ps.rng = KP(seeds)[pix];
                    ps.k = 0;
                    diag_event(P, npix, pix, 0);
                    acc[0] = acc[kThreads] = acc[2 * kThreads] = 0.;
                    pseg = 0;
                    spec = false;
                    if (KP(max_depth) == 0) {  // every sample black, no Scene::hit call
                        ps.k = KP(n_off);
                        write_pixel(P, x, lr, ps);
                    } else if (P.prepark && order_map && KP(pcost)[pix] >= P.prepark) {
                        // a long serial chain by the probe's estimate: to a drain wave
                        // from its first sample
                        diag_event(P, npix, pix, 1);
                        Parked q;
                        q.x = x, q.lr = lr, q.k = 0, q._pad = KP(pcost)[pix] * 4u;  // 8 x segments per sample (2 probe samples)
                        q.rng_lo = ps.rng.lo, q.rng_hi = ps.rng.hi;
                        q.ar = q.ag = q.ab = 0., q._pad2 = 0.;
                        publish_parked(P, q);
                        ++tl.parked;
                    } else {
                        gen_ray(P, PixelLoc(P, x, KP(row_begin) + lr * KP(row_step)), 0, ps.rng, p, stp);
                        need = false;
                    }
                } else {
                    dry_now = true;
                }
            }
            dry = dry || __any(dry_now);  // wave-uniform
            ++wave_it;
            // endgame: once the cursor is dry and at most P.endgame pixels of the shard
            // are unfinished (about one per drain group), every lane parks its pixel
            // at its next sample boundary -- the last chains then run on a whole wave
            // each (a segment every ~2 us) instead of one lane of a wave (~16 us).
            // The count is polled every kEndgamePoll-th iteration: the device-scope load
            // is waited on at once, and in a small shard (dry from the first fill) every
            // cursor wave paid that round trip in every iteration
            if (dry && !endgame && P.endgame && (wave_it & (kEndgamePoll - 1u)) == 0u)
                endgame = static_cast<uint64_t>(__builtin_amdgcn_readfirstlane(ld_rlx(KP(pixels_done)))) + P.endgame >= npix;

            if (__all(need)) {
                if (dry) {
                    if (kWgDone && lane == static_cast<uint32_t>(__ffsll(static_cast<unsigned long long>(__ballot(1))) - 1)) {
                        uint32_t *wg = reinterpret_cast<uint32_t *>(reinterpret_cast<char *>(lds_sph) + KP(lane_lds_off) +
                                                                    lane_lds_area(kThreads));
                        const uint32_t c = atomicExch(wg, 0u);
                        if (c) atomicAdd(KP(pixels_done), c);
                    }
                    break;
                }
                continue;
            }
            if (need) continue;  // this lane waits while the others work
            ++tl.seg, ++pseg;
            const double a = p.dx * p.dx + p.dy * p.dy + p.dz * p.dz;
            double bt = 0.;
            STAMP(0);  // 0: loop top, refill
#ifdef RTW_WALK_DIAG  // diagnostic build: the wave's walk length with and without its camera rays
            const uint32_t v_before = tl.visits;
#endif
            const int best = hit(p.ox, p.oy, p.oz, p.dx, p.dy, p.dz, a, p.prev, bt);
#ifdef RTW_WALK_DIAG
            {
                const uint32_t v = tl.visits - v_before;
                const bool prim = p.depth == 0;
                uint32_t m_all = v, m_sec = prim ? 0u : v, m_prim = prim ? v : 0u;
                for (int off = 32; off > 0; off >>= 1) {
                    m_all = max(m_all, static_cast<uint32_t>(__shfl_xor(static_cast<int>(m_all), off)));
                    m_sec = max(m_sec, static_cast<uint32_t>(__shfl_xor(static_cast<int>(m_sec), off)));
                    m_prim = max(m_prim, static_cast<uint32_t>(__shfl_xor(static_cast<int>(m_prim), off)));
                }
                const uint64_t pm = __ballot(prim);
                if (lane == static_cast<uint32_t>(__ffsll(static_cast<unsigned long long>(__ballot(1))) - 1)) {
                    atomicAdd(&P.counters[11], static_cast<unsigned long long>(m_all));
                    atomicAdd(&P.counters[12], static_cast<unsigned long long>(m_sec));
                    atomicAdd(&P.counters[13], static_cast<unsigned long long>(m_prim));
                    atomicAdd(&P.counters[14], static_cast<unsigned long long>(__popcll(pm)));
                }
                if (prim) atomicAdd(&P.counters[15], static_cast<unsigned long long>(v));
            }
#endif
            STAMP(1);  // 1: hit tail (exact candidates, cut check)
            // ---- segment end: HitRecord + scatter (materials.rs:22-111) or the sky, the
            // sample boundary, and ONE rejection loop for every lane's draws --
            // random_unit_vec (Lambertian / Metal, vec3.rs:218-232) and, for a lane whose
            // sample ended, the next sample's defocus disk (vec3.rs:270-277), in that
            // lane's own order (the scatter's draws first). The wave pays the max over
            // lanes of their combined tries instead of two separate maxima. Decisions
            // that need no draw (fold, done, park) come before the loop, every action
            // that depends on the RNG state (park entry, new ray) after it.
            const uint32_t kind = best >= 0 ? sv.shd[best].kind : 3u;  // 3: the sky
            double vx = 0., vy = 0., vz = 0.;
            if (kind != RTW_LAMBERTIAN) {  // unit(dir), vec3.rs:183-185
                const double l = kMode == kBvh ? seg_sa : __builtin_sqrt(a);
                vx = p.dx, vy = p.dy, vz = p.dz;
                rtw_num::div3(vx, vy, vz, l);  // / l, one shared reciprocal (rtw_numeric.h)
            }
            double cr = 0., cg = 0., cb = 0.;  // leaf colour of a sample that ends here
            bool ended = true;
            double fz = 1.;  // Lambertian / Metal: new direction = p.d + u fz (p.d = n or the reflection)
            if (best < 0) {  // camera.rs:395-397
                const double t = 0.5 * (vy + 1.0);
                const double om = 1.0 - t;
                cr = om + 0.5 * t, cg = om + 0.7 * t, cb = om + t;
            } else {
                // HitRecord: point = dir*t + orig, outward = (p - c)/r, face_normal
                const double4 S = sph[best];
                const ShadeRec M = sv.shd[best];
                const double r = S.w;
                const double hx = p.dx * bt + p.ox, hy = p.dy * bt + p.oy, hz = p.dz * bt + p.oz;
                double nx = hx - S.x, ny = hy - S.y, nz = hz - S.z;
                rtw_num::div3(nx, ny, nz, r);  // (p - c) / r
                const bool front = (p.dx * nx + p.dy * ny + p.dz * nz) < 0.;
                if (!front) nx = -nx, ny = -ny, nz = -nz;
                ended = p.depth + 1u >= KP(max_depth);  // ray_color(depth >= max) -> black
                double ndx = nx, ndy = ny, ndz = nz;
                if (kind == RTW_METAL) {  // materials.rs:52-63: reflect(unit(dir), n) + fuzz u
                    const double dt = vx * nx + vy * ny + vz * nz;
                    ndx = vx - (nx * dt) * 2., ndy = vy - (ny * dt) * 2., ndz = vz - (nz * dt) * 2.;
                    fz = M.p;
                } else if (kind == RTW_DIELECTRIC) {  // materials.rs:83-111 (attenuation 1)
                    const double ratio = front ? M.a0 : M.p;  // host: a0 = 1/ir, a1 = r0*r0
                    const double cos_t = fmin((-vx) * nx + (-vy) * ny + (-vz) * nz, 1.);
                    // ratio * sqrt(1 - cos^2) > 1, the square root only near the boundary
                    bool refl = rtw_num::tir_exceeds(ratio, 1.0 - cos_t * cos_t, 1.);
                    if (!refl) {
                        const double r0 = M.a1;
                        const double q = 1. - cos_t;
                        const double schlick = r0 + (1. - r0) * (q * ((q * q) * (q * q)));
                        refl = schlick > xs_next_01(ps.rng);
                    }
                    if (refl) {  // vec3.rs:252-257
                        const double dt = vx * nx + vy * ny + vz * nz;
                        ndx = vx - (nx * dt) * 2., ndy = vy - (ny * dt) * 2., ndz = vz - (nz * dt) * 2.;
                    } else {  // vec3.rs:259-268 (its cos is cos_t: the same expression)
                        const double qx = (vx + nx * cos_t) * ratio, qy = (vy + ny * cos_t) * ratio,
                                     qz = (vz + nz * cos_t) * ratio;
                        const double w = -__builtin_sqrt(__builtin_fabs(1. - (qx * qx + qy * qy + qz * qz)));
                        ndx = qx + nx * w, ndy = qy + ny * w, ndz = qz + nz * w;
                    }
                }
                if (kind != RTW_DIELECTRIC) {  // the bounce's attenuation row
                    if (ended) cr = M.a0 * 0., cg = M.a1 * 0., cb = M.a2 * 0.;  // att x black
                    else p.stk.push(static_cast<uint32_t>(best), KP(spill), stride, gid());
#ifdef RTW_WALK_DIAG
                    if (!ended && p.stk.n > kRegSlots) atomicAdd(&P.counters[18], 1ull);  // spill-level pushes
#endif
                }
                p.ox = hx, p.oy = hy, p.oz = hz;
                p.dx = ndx, p.dy = ndy, p.dz = ndz;
                p.prev = best;
                ++p.depth;
            }
            STAMP(6);  // 6: hit record + scatter without draws
            bool done = false, park = false;
            if (ended) {
                if (best >= 0 && KP(att_finite)) {  // black leaf: +-0, no fold (see trace_samples)
                    p.stk.clear();
                } else {
                    fold(sv.shd, p, KP(spill), gid(), stride, cr, cg, cb);
                    acc[0] = acc[0] + cr, acc[kThreads] = acc[kThreads] + cg, acc[2 * kThreads] = acc[2 * kThreads] + cb;
                }
                done = ++ps.k >= KP(n_off);
                // park: the budget is spent, the rate runs away, or -- once the
                // cursor is dry, so drain groups are about to be plentiful -- the
                // estimated remaining work exceeds KP(tail_segs)
                park = !done && (pseg >= KP(seg_budget) || (ps.k >= KP(rate_k) && pseg > KP(rate_x) * ps.k) ||
                                 (endgame && KP(n_off) - ps.k >= kEndgameMinSamples) ||
                                 (dry && static_cast<uint64_t>(KP(n_off) - ps.k) * pseg > static_cast<uint64_t>(KP(tail_segs)) * ps.k));
                uint32_t *diag = KP(diag);
                if ((done || park) && diag) {  // a pixel's records may come from two XCDs
                    atomicAdd(diag + 2 * pix, pseg);
                    __hip_atomic_store((gu32 *)(diag + 2 * pix + 1),
                                       static_cast<uint32_t>(__builtin_amdgcn_s_memrealtime()),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                {  // one completion-count atomic per wave (write_pixel leaves it to us)
                    const uint64_t dm = __ballot(done);
                    if (dm && lane == static_cast<uint32_t>(__ffsll(static_cast<unsigned long long>(dm)) - 1)) {
                        // RTW_WG_DONE: an LDS add without the endgame (whose trigger reads the
                        // global count); the workgroup's sum is posted as its cursor waves leave
                        if (kWgDone && !KP(endgame))
                            atomicAdd(reinterpret_cast<uint32_t *>(reinterpret_cast<char *>(lds_sph) + KP(lane_lds_off) +
                                                                   lane_lds_area(kThreads)),
                                      static_cast<uint32_t>(__popcll(dm)));
                        else
                            atomicAdd(KP(pixels_done), static_cast<uint32_t>(__popcll(dm)));
                    }
#ifdef RTW_WALK_DIAG
                    if (dm && lane == static_cast<uint32_t>(__ffsll(static_cast<unsigned long long>(dm)) - 1))
                        atomicAdd(&P.counters[17], 1ull);
#endif
                }
            }
            STAMP(7);  // 7: fold + pixel sum + decisions
            // the draws: phase 1 = random_unit_vec (3 per try, accept len^2 <= 1),
            // phase 2 = the defocus disk (2 per try, accept len^2 < 1); each candidate is
            // judged in f32 first and rebuilt exactly only near the boundary
            const bool want_u = kind <= RTW_METAL;  // Lambertian or Metal
            const bool want_disk = ended && !done && !park && !(KP(defocus_angle) <= 0.);
            // Speculation: a lane whose draws are done while others still loop goes on,
            // on a copy of its RNG state, with the unit vector its NEXT segment will
            // probably need (random_unit_vec's candidates do not depend on the
            // geometry), and keeps the state its last try started from (the accepting
            // try, or the next one). A Lambertian / Metal hit resumes from that state:
            // the rejected tries are skipped, the same draws accepted. Anything else
            // (the Schlick draw, the sky, the disk) goes on from the lane's own state.
            STAMP_CNT(1, want_u ? 1u : 0u);
            STAMP_CNT(2, spec && want_u ? 1u : 0u);
            STAMP_CNT(3, want_disk ? 1u : 0u);
            if (spec && want_u) {
                const uint4 r = *spec_lds;
                ps.rng.lo = static_cast<uint64_t>(r.x) | static_cast<uint64_t>(r.y) << 32;
                ps.rng.hi = static_cast<uint64_t>(r.z) | static_cast<uint64_t>(r.w) << 32;
            }
            const bool may_spec = !done && !park;  // the lane traces on from this state
            // A lane's draws in order: phase 1 (its unit vector), 2 (the disk), 3 (the
            // speculative unit vector of its next segment), 4 = finished. The wave loops
            // while a lane is in phase 1 or 2; phase 3 never extends the loop.
            // The loop keeps only the accepted raw draws; their f64 coordinates are formed
            // once after it (inside it, only the rare candidates within 2^-17 of the
            // boundary need them, for the exact test).
            const uint32_t after2 = may_spec ? 3u : 4u;
            const uint32_t after1 = want_disk ? 2u : after2;
            uint32_t phase = want_u ? 1u : after1;
            uint32_t um0 = 0, um1 = 0, um2 = 0, dm0 = 0, dm1 = 0;  // accepted draws (sphere, disk)
            U128 own = ps.rng;  // the lane's own state (phase 3 runs on a copy)
            bool did3 = phase == 3u;
            bool any_real = __any(phase <= 2u);  // a lane leaves once finished; all, once no
            while (any_real && phase <= 3u) {    // lane has a draw it needs
                STAMP_CNT(0, 1u);
                U128 st = ps.rng;
                const bool pu = phase != 2u;  // a unit-sphere try (1 or 3)
                const uint32_t m0 = xs_next_m(st), m1 = xs_next_m(st);
                uint32_t m2 = 0;
                if (pu) m2 = xs_next_m(st);
                const float x32 = coord32(m0), y32 = coord32(m1), z32 = pu ? coord32(m2) : 0.f;
                const float l32 = fmaf(x32, x32, fmaf(y32, y32, z32 * z32));
                bool ok = l32 < 1.f - kRejBand;  // surely accepted
                if (!ok && !(l32 > 1.f + kRejBand)) {  // near the boundary: the exact test
                    const double x = coord64(m0), y = coord64(m1);
                    if (pu) {
                        const double z = coord64(m2);
                        ok = x * x + y * y + z * z <= 1.;          // vec3.rs:219-226
                    } else {
                        ok = (x * x + y * y + 0. * 0.) < 1.;      // vec3.rs:270-277
                    }
                }
                // the bookkeeping as selects: no branch for the wave to pay
                const bool a1 = ok && phase == 1u, a2 = ok && phase == 2u, a3 = ok && phase == 3u;
                um0 = a1 ? m0 : um0, um1 = a1 ? m1 : um1, um2 = a1 ? m2 : um2;
                dm0 = a2 ? m0 : dm0, dm1 = a2 ? m1 : dm1;
                // every try advances the state except phase 3's accepting one: that
                // state (the try's start) is the resume point
                ps.rng.lo = a3 ? ps.rng.lo : st.lo, ps.rng.hi = a3 ? ps.rng.hi : st.hi;
                const uint32_t next = a1 ? after1 : a2 ? after2 : a3 ? 4u : phase;
                const bool enter3 = next == 3u && phase != 3u;
                own.lo = enter3 ? ps.rng.lo : own.lo, own.hi = enter3 ? ps.rng.hi : own.hi;
                did3 = did3 || enter3;
                phase = next;
                any_real = __any(phase <= 2u);
            }
            spec = did3;
            if (did3) {  // keep the resume point (the accepting try's start, or the next try's),
                         // back to the lane's own state
                *spec_lds = make_uint4(static_cast<uint32_t>(ps.rng.lo), static_cast<uint32_t>(ps.rng.lo >> 32),
                                       static_cast<uint32_t>(ps.rng.hi), static_cast<uint32_t>(ps.rng.hi >> 32));
                ps.rng = own;
            }
            STAMP(9);  // 9: the draws
            double ux, uy, uz;
            if (want_u && !ended) {  // materials.rs:22-37 / 52-63 with u = unit(the point)
                ux = coord64(um0), uy = coord64(um1), uz = coord64(um2);
                const double l = __builtin_sqrt(ux * ux + uy * uy + uz * uz);
                rtw_num::div3(ux, uy, uz, l);  // u / l
                double ndx = p.dx + ux * fz, ndy = p.dy + uy * fz, ndz = p.dz + uz * fz;
                // near_zero without abs (vec3.rs:246-250): Lambertian falls back to n
                if (kind == RTW_LAMBERTIAN && ndx < 1e-8 && ndy < 1e-8 && ndz < 1e-8) ndx = p.dx, ndy = p.dy, ndz = p.dz;
                p.dx = ndx, p.dy = ndy, p.dz = ndz;
            }
            if (ended) {
                if (done) {
                    ps.ar = acc[0], ps.ag = acc[kThreads], ps.ab = acc[2 * kThreads];
                    write_pixel(P, x, lr, ps, false);
                    need = true;
                } else if (park) {  // park at the sample boundary
                    diag_event(P, npix, pix, 1);
                    ps.ar = acc[0], ps.ag = acc[kThreads], ps.ab = acc[2 * kThreads];
                    Parked q;
                    q.x = x, q.lr = lr, q.k = ps.k, q._pad = (pseg * 8u) / max(ps.k, 1u);  // 8 x segments per sample so far
                    q.rng_lo = ps.rng.lo, q.rng_hi = ps.rng.hi;
                    q.ar = ps.ar, q.ag = ps.ag, q.ab = ps.ab, q._pad2 = 0.;
                    publish_parked(P, q);
                    ++tl.parked;
                    need = true;
                } else {  // the next sample's defocus disk point (camera.rs:452-456)
                    const double dpx = -1. + 2. * rtw_num::next01_of(dm0), dpy = -1. + 2. * rtw_num::next01_of(dm1);
                    ray_from_disk(P, PixelLoc(P, x, KP(row_begin) + lr * KP(row_step)), ps.k, dpx, dpy, p);
                }
            }
            STAMP(4);  // 4: fold + next sample / pixel end
        }
#ifdef RTW_STAMPS
        {  // diagnostic: per cursor wave, the max over lanes of each section sum
            uint64_t *row = P.stamps + (static_cast<uint64_t>(blockIdx.x) * (kThreads / 64u) + threadIdx.x / 64u) * kStampRow;
            for (int k = 0; k < kStampSlots; ++k) {
                uint64_t v = stp.acc[k];
                for (int off = 32; off > 0; off >>= 1) {
                    const uint64_t o = __shfl_xor(v, off);
                    v = v > o ? v : o;
                }
                if (lane == 0) row[k] = v;
            }
            uint32_t wi = tl.witer;  // wave iterations (counted on one lane each)
            for (int off = 32; off > 0; off >>= 1) wi += static_cast<uint32_t>(__shfl_xor(static_cast<int>(wi), off));
            if (lane == 0) row[14] = wi, row[15] = stamp_now();
            for (int k = 0; k < 4; ++k) {  // draws-loop counters: trips = max over lanes, the rest sums
                uint64_t v = stp.cnt[k];
                for (int off = 32; off > 0; off >>= 1) {
                    const uint64_t o = __shfl_xor(v, off);
                    v = k == 0 ? (v > o ? v : o) : v + o;
                }
                if (lane == 0) row[10 + k] = v;
            }
        }
#endif
        // this wave parks no more (its parks are published: drained stores + flags)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == static_cast<uint32_t>(__ffsll(static_cast<unsigned long long>(__ballot(1))) - 1))
            atomicAdd(P.park_ctl_done, 1u);
    }
    // cooperative drain of the park queue, kCoopG lanes per parked pixel
    const uint32_t sub = threadIdx.x & (kCoopG - 1u);
    const int gl = static_cast<int>(lane & ~(kCoopG - 1u));
    uint32_t cseg = 0;
    // RTW_DRAIN_OFF=1 (tests): no drain here, so every parked pixel is left to the
    // follow-up launch (rtw_park_leftover) -- that path then runs on every entry
    // a wave that drains runs one pixel's serial chain for the whole wave: raised
    // issue priority (as the priority waves), so the chains that set the launch's end
    // are not held back by the cursor waves still sharing the SIMD (RTW_DRAIN_PRIO=0: off)
    if (KP(drain_prio)) set_prio(KP(drain_prio));
    for (bool drain = !KP(drain_off); drain;) {
        uint32_t t = 0, state = 0;  // state 1: ticket t is published, 2: stop
        if (sub == 0) {
            t = atomicAdd(P.park_cursor, 1u);
            SpinGuard guard(P);
            for (uint32_t spins = 0;; ++spins) {
                if (t < ld_rlx(P.park_count)) {
                    while (ld_rlx(P.park_flag + t) != kSlotPublished) __builtin_amdgcn_s_sleep(2);
                    claim_slot(P, t);
                    state = 1;
                    break;
                }
                const uint32_t dn = ld_rlx(P.park_ctl_done);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (dn >= P.n_cursor_waves && t >= ld_rlx(P.park_count)) {
                    state = 2;  // every cursor wave is done and t lies past the queue
                    break;
                }
                __builtin_amdgcn_s_sleep(16);
                // nothing moves anywhere (e.g. workgroups of this launch that are not
                // resident yet): leave; a ticket t published later stays unclaimed
                // and the leftover launch finishes it
                if ((spins & 255u) == 255u && guard.expired(P)) {
                    atomicAdd(&P.counters[7], 1ull);
                    state = 2;
                    break;
                }
            }
        }
        t = __shfl(t, gl);
        state = __shfl(state, gl);
        if (state == 2) break;
        // every load of the handed-off entry is an sc1 load (Guideline 16)
        Parked q;
        unsigned long long *w = reinterpret_cast<unsigned long long *>(&q);
        gu64 *src = (gu64 *)(P.park + t);
#pragma unroll
        for (int j = 0; j < 8; ++j) w[j] = __hip_atomic_load(src + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (P.prio_split) set_prio(q._pad >= P.prio_split ? KP(drain_prio) : 0u);
        cseg += coop_pixel<kCoopG>(P, sv, filt, fsh, q, gid() & ~static_cast<uint64_t>(kCoopG - 1u), tl, stp_unused);
        if (sub == 0) atomicAdd(P.park_processed, 1u);
    }
    tl.seg += cseg;
    flush_tally(P, tl, false);
}

// Leftover launch after the persistent kernel: park entries that were published
// but never claimed -- only possible when waiting waves left on the no-progress
// guard (SpinGuard). Exits at once in the normal case (every entry finished).
// Kernel boundary: every entry and flag is visible with plain loads.
template <bool kLds, uint32_t kG>
__global__ __launch_bounds__(kBlock) void rtw_park_leftover(const KParams P) {
    if (*P.park_processed >= *P.park_count) return;  // block-uniform
    extern __shared__ __attribute__((aligned(16))) double4 lds_sph[];
    const SceneView sv = stage_scene<kLds, kScanF32>(P, lds_sph);
    const float4 *filt = stage_filt<kLds>(P, sv.end);
    const uint32_t sub = threadIdx.x & (kG - 1u);
    const int gl = static_cast<int>(threadIdx.x & 63u & ~(kG - 1u));
    Tally tl;
    Stamps stp;
    uint32_t seg = 0;
    const uint32_t n = *P.park_count;
    for (;;) {
        uint32_t item = 0, flag = 0;
        if (sub == 0) {
            item = atomicAdd(P.leftover_cursor, 1u);
            if (item < n) flag = P.park_flag[item];
        }
        item = __shfl(item, gl);
        flag = __shfl(flag, gl);
        if (item >= n) break;
        if (flag != kSlotPublished) continue;  // finished by the persistent kernel
        const Parked q = P.park[item];
        // spill columns: region B, column = slot (the persistent kernel's groups
        // used group-base columns; a kernel boundary separates the two uses)
        seg += coop_pixel<kG>(P, sv, filt, 0u, q, item, tl, stp);
        if (sub == 0) {
            atomicAdd(&P.counters[10], 1ull);
            atomicAdd(P.park_processed, 1u);
        }
    }
#ifdef RTW_STAMPS
    if ((threadIdx.x & 63u) == 0) {  // diagnostic: per drain wave, its section sums (tools/stamps_drain.py)
        uint64_t *row = P.stamps_drain + (static_cast<uint64_t>(blockIdx.x) * (kBlock / 64u) + threadIdx.x / 64u) * kStampRow;
        for (int k = 0; k < kStampSlots; ++k) row[k] = stp.acc[k];
        row[14] = seg, row[15] = stamp_now();
    }
#endif
    tl.seg = seg;
    flush_tally(P, tl, false);
}

// Completeness latch, enqueued after every render: an image with fewer pixel
// writes than pixels bumps the session's error word, which stays set until
// rtw_session_stats reads it -- so a failed render is reported even when the
// caller enqueued the next render before asking for stats.
template <typename T>
__global__ void rtw_latch_check(const T *written, T expect, uint32_t *err) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && *written != expect) atomicAdd(err, 1u);
}

// ------------------------------------------------------------------- probes --
__global__ void probe_seeds(U128 seed, uint64_t first, uint64_t count, const uint4 *tab,
                            uint32_t bits, U128 *out) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < count) out[i] = child_of(jump_state(seed, first + i, tab, bits));
}
__global__ void probe_f64(const double *a, const double *b, uint64_t n, double *osq, double *odiv) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < n) {
        osq[i] = __builtin_sqrt(a[i]);
        odiv[i] = a[i] / b[i];
    }
}

// ------------------------------------------------------------------- host ---
#define HIPCHECK(expr)                                                                   \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess)                                                            \
            throw rtw::Error(RTW_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

uint32_t bit_length(uint64_t v) {
    uint32_t b = 0;
    while (v) ++b, v >>= 1;
    return b;
}

}  // namespace

struct rtw_session {
    int device = 0;
    hipStream_t own = nullptr;
    double4 *d_sph = nullptr;
    float4 *d_filt = nullptr;
    ShadeRec *d_shade = nullptr;
    uint16_t *d_nbr = nullptr;  // inside-cut lists
    uint32_t n_nbr = 0;
    double4 *d_trap = nullptr;  // per-sphere trapped-path records
    uint4 *d_jump = nullptr;
    uint4 *d_tries = nullptr;  // rtw::try_table (trapped-path replay, 129 x 64 columns)
    unsigned long long *d_counters = nullptr;
    uint16_t *d_spill = nullptr;
    size_t spill_bytes = 0;
    Parked *d_park = nullptr;  // park queue, one slot per pixel of the largest shard so far
    size_t park_cap = 0;
    uint32_t *d_park_ctl = nullptr;  // [0] parked count, [1] phase-2 cursor, [2] pixel cursor
    U128 *d_seeds = nullptr;         // per-pixel RNG children of the current shard
    uint32_t *d_park_flag = nullptr; // per park slot publish flags
    uint32_t *d_order = nullptr, *d_cost = nullptr, *d_cost_hist = nullptr;  // cost-ordered hand-out
    uint32_t *d_pcost = nullptr;
    uint32_t *d_diag = nullptr;      // RTW_DIAG=1 per-pixel records
    size_t diag_bytes = 0, diag_n = 0;
    int n_cu = 0;
    uint32_t n_sph = 0, n_mats = 0;
    bool scene_set = false;
    // BVH (rtw_accel.h); has_bvh = false -> the filtered scan
    float4 *d_nodes = nullptr, *d_leaves = nullptr;
    uint32_t *d_always = nullptr;
    uint32_t n_node = 0, n_leaf = 0, n_always = 0;
    bool has_bvh = false;
    bool att_finite = true;  // every Lambertian / Metal albedo component finite (KParams::att_finite)
    // the scene's device tables live in one grow-only arena, uploaded with one copy
    // (d_sph, d_filt, d_shade, d_nbr, d_trap, d_nodes, d_leaves, d_always, d_fgeo,
    // d_fmat and d_fkind point into it)
    char *d_arena = nullptr;
    size_t arena_cap = 0;
    void *d_out = nullptr;  // the one-shot API's framebuffer (grow-only)
    size_t out_cap = 0;
    uint32_t bvh_depth = 0;
    // f32 fast mode (rtw_fast.h): per-sphere geometry / material rows / kinds
    float4 *d_fgeo = nullptr, *d_fmat = nullptr;
    uint32_t *d_fkind = nullptr, *d_fcursor = nullptr;
    unsigned long long *d_fcount = nullptr;
    bool last_fast = false;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    hipEvent_t ev_k0 = nullptr, ev_k1 = nullptr;  // around the main kernel (rtw_stats.main_kernel_ms)
    // the seed kernel runs on `aux` beside the cost probe (fork / join events on the
    // render's stream)
    hipStream_t aux = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    bool main_ev = false;                         // the last render recorded them
    uint32_t *d_err = nullptr;  // latched count of incomplete renders (rtw_latch_check)
    hipStream_t last_stream = nullptr;
    bool pending = false;
    rtw_stats last{};
};

namespace {

void dev_free(void *p) {
    if (p) (void)hipFree(p);
}

void upload_jump(rtw_session *s) {
    const auto &t = rtw::jump_table();
    std::vector<uint4> cols(t.size());
    for (size_t i = 0; i < t.size(); ++i) {
        const uint64_t lo = static_cast<uint64_t>(t[i]), hi = static_cast<uint64_t>(t[i] >> 64);
        cols[i] = make_uint4(static_cast<uint32_t>(lo), static_cast<uint32_t>(lo >> 32),
                             static_cast<uint32_t>(hi), static_cast<uint32_t>(hi >> 32));
    }
    HIPCHECK(hipMalloc(&s->d_jump, cols.size() * sizeof(uint4)));
    HIPCHECK(hipMemcpy(s->d_jump, cols.data(), cols.size() * sizeof(uint4), hipMemcpyHostToDevice));
    const auto &tt = rtw::try_table();
    std::vector<uint4> tc(tt.size());
    for (size_t i = 0; i < tt.size(); ++i) {
        const uint64_t lo = static_cast<uint64_t>(tt[i]), hi = static_cast<uint64_t>(tt[i] >> 64);
        tc[i] = make_uint4(static_cast<uint32_t>(lo), static_cast<uint32_t>(lo >> 32), static_cast<uint32_t>(hi),
                           static_cast<uint32_t>(hi >> 32));
    }
    HIPCHECK(hipMalloc(&s->d_tries, tc.size() * sizeof(uint4)));
    HIPCHECK(hipMemcpy(s->d_tries, tc.data(), tc.size() * sizeof(uint4), hipMemcpyHostToDevice));
}

void validate_scene(const rtw_sphere *sp, uint32_t n, const rtw_material *m, uint32_t nm) {
    if ((n && !sp) || (nm && !m)) throw rtw::Error(RTW_E_ARG, "null scene buffer");
    if (nm > 65536) throw rtw::Error(RTW_E_UNSUPPORTED, "more than 65536 materials");
    if (n > 65535) throw rtw::Error(RTW_E_UNSUPPORTED, "more than 65535 spheres (u16 path stack)");
    for (uint32_t i = 0; i < nm; ++i) {
        if (m[i].kind > RTW_DIELECTRIC) throw rtw::Error(RTW_E_ARG, "unknown material kind");
        if (m[i].kind == RTW_METAL && !(m[i].fuzz <= 1.))
            throw rtw::Error(RTW_E_FUZZ, "Fuzz cannot be more than 1");  // materials.rs:47
    }
    for (uint32_t i = 0; i < n; ++i)
        if (sp[i].mat >= nm) throw rtw::Error(RTW_E_MAT_INDEX, "sphere material index out of range");
}

// Host staging of the scene tables: each table at a 256-B aligned offset of one
// buffer, copied to the session's arena in one transfer (a dozen hipMalloc /
// hipFree / hipMemcpy round trips per scene before).
struct SceneStage {
    std::vector<char> host;
    std::vector<std::pair<void **, size_t>> slots;
    template <class T>
    void add(T **slot, const T *src, size_t count) {
        const size_t off = (host.size() + 255) & ~static_cast<size_t>(255);
        host.resize(off + std::max<size_t>(count * sizeof(T), 16));
        if (count) std::memcpy(host.data() + off, src, count * sizeof(T));
        slots.emplace_back(reinterpret_cast<void **>(slot), off);
    }
    void upload(rtw_session *s) {
        if (host.size() > s->arena_cap) {
            dev_free(s->d_arena);
            s->d_arena = nullptr, s->arena_cap = 0;
            HIPCHECK(hipMalloc(&s->d_arena, host.size()));
            s->arena_cap = host.size();
        }
        HIPCHECK(hipMemcpy(s->d_arena, host.data(), host.size(), hipMemcpyHostToDevice));
        for (auto &sl : slots) *sl.first = s->d_arena + sl.second;
    }
};

void set_scene(rtw_session *s, const rtw_sphere *sp, uint32_t n, const rtw_material *m, uint32_t nm) {
    validate_scene(sp, n, m, nm);
    HIPCHECK(hipSetDevice(s->device));
    if (s->pending) HIPCHECK(hipEventSynchronize(s->ev1));  // a render may still read the arena
    SceneStage stage;
    s->d_fgeo = s->d_fmat = nullptr, s->d_fkind = nullptr;
    s->d_sph = nullptr, s->d_filt = nullptr;
    s->d_shade = nullptr, s->d_nbr = nullptr, s->n_nbr = 0, s->d_trap = nullptr;
    s->d_nodes = nullptr, s->d_leaves = nullptr, s->d_always = nullptr;
    s->has_bvh = false, s->scene_set = false;
    s->n_node = s->n_leaf = s->n_always = s->bvh_depth = 0;
    const uint32_t npad = (n + kChunk - 1) / kChunk * kChunk;
    std::vector<double4> a(n ? n : 1);
    // padding records can never be candidates (R2' = -inf -> disc = -inf)
    std::vector<float4> f(npad ? npad : kChunk, make_float4(0.f, 0.f, 0.f, -INFINITY));
    std::vector<ShadeRec> sh(n ? n : 1);
    for (uint32_t i = 0; i < n; ++i) {
        const double rad = sp[i].radius;
        const double rr = rad * rad;  // sphere.rs:49 `self.radius * self.radius`
        const double *c = sp[i].center;
        a[i] = make_double4(c[0], c[1], c[2], rad);  // r*r formed at each use (sphere.rs:49)
        // R2' >= r*r + K (m_c^2 + r*r/2), m_c = max |c_i|, rounded up to f32; +inf
        // (always tested exactly) outside the guard or for non-finite input.
        const float r2p = rtw_accel::filter_r2p(c, rr);
        f[i] = make_float4(static_cast<float>(c[0]), static_cast<float>(c[1]),
                           static_cast<float>(c[2]), r2p);
        // the sphere's material row, flattened next to its radius
        const rtw_material &M = m[sp[i].mat];
        ShadeRec &R = sh[i];
        R.a0 = M.albedo[0], R.a1 = M.albedo[1], R.a2 = M.albedo[2];
        R.p = M.kind == RTW_METAL ? M.fuzz : M.kind == RTW_DIELECTRIC ? M.ir : 0.;
        R.kind = M.kind, R.nbr = rtw_accel::kNbrNone;
        if (M.kind == RTW_DIELECTRIC) {
            // the refraction ratio 1/ir and reflectance's r0*r0 (materials.rs:75-89),
            // with the reference's IEEE operations (attenuation is 1: no albedo row)
            const double ir = M.ir;
            double r0 = (1. - ir) / (1. + ir);
            r0 = r0 * r0;
            R.a0 = 1. / ir, R.a1 = r0, R.a2 = 0.;
        }
    }
    // inside-cut lists (rtw_accel.h): per sphere the spheres that can come nearer
    // than its far root for a ray starting inside it
    std::vector<uint16_t> nbr_ids;
    {
        std::vector<double> cen(3 * static_cast<size_t>(n)), rad(n);
        for (uint32_t i = 0; i < n; ++i) {
            for (int k = 0; k < 3; ++k) cen[3 * i + k] = sp[i].center[k];
            rad[i] = sp[i].radius;
        }
        // spheres that can trap a path (rtw_accel.h "Trapped paths"): Lambertian
        // with a finite albedo >= +0 (the black product then keeps its bits), or
        // Dielectric with a finite ir (total internal reflection)
        std::vector<uint8_t> trap_ok(n, 0);
        for (uint32_t i = 0; i < n; ++i) {
            const rtw_material &M = m[sp[i].mat];
            bool ok = false;
            if (M.kind == RTW_LAMBERTIAN) {
                ok = true;
                for (int k = 0; k < 3; ++k)
                    ok = ok && std::isfinite(M.albedo[k]) && !std::signbit(M.albedo[k]);
            } else if (M.kind == RTW_DIELECTRIC) {
                ok = std::isfinite(M.ir) && M.ir > 0.;
            }
            trap_ok[i] = ok ? 1 : 0;
        }
        std::vector<uint32_t> info;
        std::vector<rtw_accel::TrapRec> traps;
        rtw_accel::build_inside(cen.data(), rad.data(), n, info, nbr_ids, trap_ok.data(), &traps);
        for (uint32_t i = 0; i < n; ++i) sh[i].nbr = info[i];
        static_assert(sizeof(rtw_accel::TrapRec) == sizeof(double4), "TrapRec layout");
        stage.add(reinterpret_cast<rtw_accel::TrapRec **>(&s->d_trap), traps.data(), n);
    }
    nbr_ids.resize(nbr_ids.size() + 8, 0);  // padded (staged like the old allocation)
    stage.add(&s->d_nbr, nbr_ids.data(), nbr_ids.size());
    s->n_nbr = static_cast<uint32_t>(nbr_ids.size() - 8);
    stage.add(&s->d_sph, a.data(), a.size());
    stage.add(&s->d_filt, f.data(), f.size());
    stage.add(&s->d_shade, sh.data(), sh.size());
    // BVH over the same records (rtw_accel_build.cpp); ineligible scenes scan
    {
        std::vector<double> cen(3 * static_cast<size_t>(n)), rad(n);
        std::vector<float> r2p(n);
        for (uint32_t i = 0; i < n; ++i) {
            for (int k = 0; k < 3; ++k) cen[3 * i + k] = sp[i].center[k];
            rad[i] = sp[i].radius;
            r2p[i] = f[i].w;
        }
        rtw_accel::Bvh bvh;
        if (n && rtw_accel::build(cen.data(), rad.data(), r2p.data(), n, bvh)) {
            static_assert(sizeof(float4) == 4 * sizeof(float), "node layout");
            stage.add(&s->d_nodes, reinterpret_cast<const float4 *>(bvh.nodes.data()), bvh.nodes.size() / 4);
            stage.add(&s->d_leaves, reinterpret_cast<const float4 *>(bvh.leaves.data()), bvh.leaves.size() / 4);
            bvh.always.push_back(0u);  // one spare entry, as the old allocation had
            stage.add(&s->d_always, bvh.always.data(), bvh.always.size());
            bvh.always.pop_back();
            s->n_node = bvh.n_node, s->n_leaf = bvh.n_leaf;
            s->n_always = static_cast<uint32_t>(bvh.always.size());
            s->bvh_depth = bvh.depth;
            s->has_bvh = true;
        }
    }
    // fast-mode rows: f32 geometry, material row, kind
    {
        std::vector<float4> fg(n ? n : 1), fm(n ? n : 1);
        std::vector<uint32_t> fk(n ? n : 1, 0);
        for (uint32_t i = 0; i < n; ++i) {
            const rtw_material &M = m[sp[i].mat];
            fg[i] = make_float4(static_cast<float>(sp[i].center[0]), static_cast<float>(sp[i].center[1]),
                                static_cast<float>(sp[i].center[2]), static_cast<float>(sp[i].radius));
            if (M.kind == RTW_DIELECTRIC) {
                const double r0 = (1. - M.ir) / (1. + M.ir);
                fm[i] = make_float4(static_cast<float>(1. / M.ir), static_cast<float>(M.ir),
                                    static_cast<float>(r0 * r0), 0.f);
            } else {
                fm[i] = make_float4(static_cast<float>(M.albedo[0]), static_cast<float>(M.albedo[1]),
                                    static_cast<float>(M.albedo[2]),
                                    M.kind == RTW_METAL ? static_cast<float>(M.fuzz) : 0.f);
            }
            fk[i] = M.kind;
        }
        stage.add(&s->d_fgeo, fg.data(), fg.size());
        stage.add(&s->d_fmat, fm.data(), fm.size());
        stage.add(&s->d_fkind, fk.data(), fk.size());
    }
    stage.upload(s);
    s->att_finite = true;
    for (uint32_t i = 0; i < n; ++i) {
        const rtw_material &M = m[sp[i].mat];
        if (M.kind != RTW_DIELECTRIC)
            for (int k = 0; k < 3; ++k) s->att_finite = s->att_finite && std::isfinite(M.albedo[k]);
    }
    s->n_sph = n;
    s->n_mats = nm;
    s->scene_set = true;
}

rtw_shard resolve_shard(const rtw_camera *cam, const rtw_shard *shard) {
    rtw_shard sh{0, 1, cam->img_height, 0};
    if (shard) {
        sh = *shard;
        if (sh.row_step == 0) throw rtw::Error(RTW_E_ARG, "shard row_step must be > 0");
        if (sh.n_rows && static_cast<uint64_t>(sh.row_begin) +
                                 static_cast<uint64_t>(sh.n_rows - 1) * sh.row_step >=
                             cam->img_height)
            throw rtw::Error(RTW_E_ARG, "shard rows outside the image");
    }
    return sh;
}

#ifdef RTW_STAMPS
uint64_t *&stamp_buf() { static uint64_t *p = nullptr; return p; }
size_t &stamp_n() { static size_t n = 0; return n; }
#endif

// Every render of a session shares its buffers (counters, park queue, seeds,
// spill): a render enqueued on another stream than the previous one first waits
// for it, so at most one render per session runs at a time.
void order_after_last(rtw_session *s, hipStream_t st) {
    if (s->pending && s->last_stream != st) HIPCHECK(hipStreamWaitEvent(st, s->ev1, 0));
}

void render(rtw_session *s, const rtw_camera *cam, uint32_t samples_sqrt, rtw_u128 seed,
            const rtw_shard *shard_in, double *out, hipStream_t stream) {
    if (!cam || !out) throw rtw::Error(RTW_E_ARG, "null argument");
    const rtw::Knobs kn;  // tuning only under RTW_AB (rtw_internal.h)
    if (!s->scene_set) throw rtw::Error(RTW_E_ARG, "session has no scene");
    if (cam->img_height == 0 || cam->img_width == 0)
        throw rtw::Error(RTW_E_EMPTY_IMAGE, "image height and width must be > 0");  // camera.rs:267
    if (samples_sqrt > 65535) throw rtw::Error(RTW_E_UNSUPPORTED, "samples_sqrt > 65535");
    const uint64_t npix = static_cast<uint64_t>(cam->img_height) * cam->img_width;
    const uint32_t bits = bit_length(npix - 1);
    if (bits > static_cast<uint32_t>(rtw::kJumpBits)) throw rtw::Error(RTW_E_UNSUPPORTED, "image > 2^40 pixels");
    const rtw_shard sh = resolve_shard(cam, shard_in);

    KParams P{};
    auto cp = [](double *d, const rtw_vec3 &v) { d[0] = v.x, d[1] = v.y, d[2] = v.z; };
    cp(P.p00, cam->pixel00);
    cp(P.du, cam->pixel_delta_u);
    cp(P.dv, cam->pixel_delta_v);
    cp(P.from, cam->look_from);
    cp(P.ddu, cam->defocus_disk_u);
    cp(P.ddv, cam->defocus_disk_v);
    // offset_lattice(&pixel_delta_v, &pixel_delta_u, s) (camera.rs:243-244): dx := delta_v
    const rtw::Vec3 dxv = rtw::Vec3::of(cam->pixel_delta_v), dyv = rtw::Vec3::of(cam->pixel_delta_u);
    if (samples_sqrt == 0) {
        cp(P.lat_pos0, (dxv / 2. + dyv / 2.).c());
    } else {
        const double n = static_cast<double>(samples_sqrt);
        const rtw::Vec3 dx = dxv / n, dy = dyv / n;
        cp(P.lat_dx, dx.c());
        cp(P.lat_dy, dy.c());
        cp(P.lat_pos0, (dx / 2. + dy / 2.).c());
    }
    P.defocus_angle = cam->defocus_angle;
    P.W = cam->img_width;
    P.s = samples_sqrt;
    P.s_magic = samples_sqrt >= 2 && samples_sqrt <= 1625
                    ? static_cast<uint32_t>(((1ull << 32) + samples_sqrt - 1) / samples_sqrt)
                    : 0u;
    P.n_off = samples_sqrt ? samples_sqrt * samples_sqrt : 1;
    P.max_depth = cam->max_depth;
    P.row_begin = sh.row_begin;
    P.row_step = sh.row_step;
    P.n_rows = sh.n_rows;
    P.n_sph = s->n_sph;
    P.n_node = s->n_node;
    P.n_leaf = s->n_leaf;
    P.n_always = s->n_always;
    P.nodes = s->d_nodes;
    P.leaves = s->d_leaves;
    P.always = s->d_always;
    P.jump_bits = bits;
    P.att_finite = (s->att_finite && !kn.get("RTW_FOLD_BLACK")) ? 1u : 0u;
    P.seed_lo = seed.lo;
    P.seed_hi = seed.hi;
    P.sph = s->d_sph;
    P.filt = s->d_filt;
    P.shade = s->d_shade;
    P.nbr = s->d_nbr;
    P.n_nbr = s->n_nbr;
    P.trap = s->d_trap;
    P.jump = s->d_jump;
    P.tries = s->d_tries;
    P.out = out;
    // path-stack spill levels: (max_depth - kRegSlots) x pixels x u16, grown on demand
    // path-stack spill: 2 regions x (max_depth - kRegSlots) levels x columns (u16);
    // columns = pixels (tile kernel), persistent lanes / drain groups (persistent)
    const uint64_t spill_cols = std::max<uint64_t>(static_cast<uint64_t>(sh.n_rows) * cam->img_width,
                                                   static_cast<uint64_t>(s->n_cu > 0 ? s->n_cu : 256) * 4 * 1024);
    const size_t spill_need = cam->max_depth > kRegSlots
                                  ? static_cast<size_t>(cam->max_depth - kRegSlots) * spill_cols * sizeof(uint16_t) * 2
                                  : 0;
    if (spill_need > s->spill_bytes) {
        HIPCHECK(hipSetDevice(s->device));
        HIPCHECK(hipStreamSynchronize(stream ? stream : nullptr));
        if (s->pending) HIPCHECK(hipEventSynchronize(s->ev1));
        dev_free(s->d_spill);
        s->d_spill = nullptr, s->spill_bytes = 0;
        HIPCHECK(hipMalloc(&s->d_spill, spill_need));
        s->spill_bytes = spill_need;
    }
    P.spill = s->d_spill;
    P.spill_b = s->d_spill ? s->d_spill + spill_need / (2 * sizeof(uint16_t)) : nullptr;
    P.spill_stride = cam->max_depth > kRegSlots ? cam->max_depth - kRegSlots : 0;
    // park queue (one slot per pixel) and the per-pixel segment budget of phase 1
    const size_t npix_sh = static_cast<size_t>(sh.n_rows) * cam->img_width;
    if (npix_sh > s->park_cap) {
        HIPCHECK(hipSetDevice(s->device));
        HIPCHECK(hipStreamSynchronize(stream ? stream : nullptr));
        if (s->pending) HIPCHECK(hipEventSynchronize(s->ev1));
        dev_free(s->d_park);
        s->d_park = nullptr, s->park_cap = 0;
        dev_free(s->d_seeds), dev_free(s->d_park_flag), dev_free(s->d_order), dev_free(s->d_cost);
        dev_free(s->d_pcost);
        s->d_seeds = nullptr, s->d_park_flag = nullptr, s->d_order = nullptr, s->d_cost = nullptr;
        s->d_pcost = nullptr;
        HIPCHECK(hipMalloc(&s->d_park, npix_sh * sizeof(Parked)));
        HIPCHECK(hipMalloc(&s->d_seeds, npix_sh * sizeof(U128)));
        HIPCHECK(hipMalloc(&s->d_park_flag, npix_sh * sizeof(uint32_t)));
        HIPCHECK(hipMalloc(&s->d_order, npix_sh * sizeof(uint32_t)));
        HIPCHECK(hipMalloc(&s->d_cost, 2 * npix_sh * sizeof(uint32_t)));  // 2 words per 8x8 tile
        HIPCHECK(hipMalloc(&s->d_pcost, npix_sh * sizeof(uint32_t)));
        s->park_cap = npix_sh;
    }
    P.park = s->d_park;
    P.park_count = s->d_park_ctl;
    P.park_cursor = s->d_park_ctl + 1;
    P.pix_cursor = s->d_park_ctl + 2;
    P.park_ctl_done = s->d_park_ctl + 3;
    P.pixels_done = s->d_park_ctl + 4;
    P.park_processed = s->d_park_ctl + 5;
    P.leftover_cursor = s->d_park_ctl + 6;
    {
        // idle-wait guard (SpinGuard): RTW_SPIN_GUARD_MS of no progress anywhere
        double ms = 100.;
        if (const char *e = kn.get("RTW_SPIN_GUARD_MS")) ms = std::atof(e);
        P.spin_guard = static_cast<uint64_t>(std::max(0., ms) * 1e5);  // 100 MHz ticks
    }
    P.park_flag = s->d_park_flag;
    P.seeds = s->d_seeds;
    {
        // budget = X x samples per pixel (X: RTW_BUDGET_X, default kBudgetX; 0 = off)
        double bx = kBudgetX;
        if (const char *e = kn.get("RTW_BUDGET_X")) bx = std::atof(e);
        const double b = bx * static_cast<double>(P.n_off);
        P.seg_budget = (bx > 0. && b < 4e9) ? static_cast<uint32_t>(std::ceil(b)) : 0xffffffffu;
    }
#ifdef RTW_STAMPS
    {
        // one row per wave of the persistent launch (one workgroup per CU), then one
        // per wave of the leftover launch (one kBlock workgroup per CU)
        const size_t ncu = static_cast<size_t>(s->n_cu > 0 ? s->n_cu : 256);
        const size_t np = ncu * (kPBlock / 64), nw = np + ncu * (kBlock / 64);
        static uint64_t *d_st = nullptr;
        static size_t cap = 0;
        if (nw * kStampRow * 8 > cap) {
            if (d_st) (void)hipFree(d_st);
            HIPCHECK(hipMalloc(&d_st, nw * kStampRow * 8));
            cap = nw * kStampRow * 8;
        }
        HIPCHECK(hipMemset(d_st, 0, nw * kStampRow * 8));
        P.stamps = d_st;
        P.stamps_drain = d_st + np * kStampRow;
        stamp_buf() = d_st;
        stamp_n() = nw;
    }
#endif
    P.counters = s->d_counters;
    P.diag = nullptr;
    P.diag_ev = 0;
    if (const char *e = kn.get("RTW_DIAG")) {
        if (std::atoi(e) != 0) {
            // RTW_DIAG=2: also per pixel {hand-out, first park, first drain claim} clocks
            // after the {segments, completion} records
            const size_t per = std::atoi(e) >= 2 ? 5u : 2u;
            const size_t need = (static_cast<size_t>(sh.n_rows) * cam->img_width * per + 4) * sizeof(uint32_t);
            if (need > s->diag_bytes) {
                HIPCHECK(hipSetDevice(s->device));
                HIPCHECK(hipDeviceSynchronize());
                dev_free(s->d_diag);
                s->d_diag = nullptr, s->diag_bytes = 0;
                HIPCHECK(hipMalloc(&s->d_diag, need));
                s->diag_bytes = need;
            }
            HIPCHECK(hipMemsetAsync(s->d_diag, 0, need, stream));
            P.diag = s->d_diag;
            P.diag_ev = per == 5u ? 1u : 0u;
            s->diag_n = need / sizeof(uint32_t);
        }
    }

    HIPCHECK(hipSetDevice(s->device));
    hipStream_t st = stream;  // NULL = HIP's null stream (torch's default stream handle is 0)
    order_after_last(s, st);
    // Scene::hit strategy: RTW_ACCEL=0 f64 scan, 1 filtered scan, 2 BVH (default
    // when the scene is eligible); A/B and tests only (RTW_AB) -- results are identical.
    int mode = s->has_bvh ? kBvh : kScanF32;
    if (const char *e = kn.get("RTW_ACCEL")) mode = std::atoi(e);
    if (mode == kBvh && !s->has_bvh) mode = kScanF32;
    if (mode < kScanF64 || mode > kBvh) mode = kScanF32;
    size_t lds = lds_bytes_for(P.n_sph, P.n_node, P.n_leaf, mode == kBvh, P.n_nbr);
    // pass-1 records for the coop groups (BVH scenes read them from the leaves)
    if (mode != kBvh) lds += static_cast<size_t>(P.n_sph) * sizeof(float4);
    const bool use_lds = lds <= kLdsCap;
    if (!use_lds) lds = 0;
    HIPCHECK(hipMemsetAsync(s->d_counters, 0, kCounters * sizeof(unsigned long long), st));
    HIPCHECK(hipMemsetAsync(s->d_park_ctl, 0, 8 * sizeof(uint32_t), st));
    HIPCHECK(hipEventRecord(s->ev0, st));
    P.order = 2;
    if (const char *e = kn.get("RTW_ORDER")) P.order = static_cast<uint32_t>(std::atoi(e));
    uint32_t grid_p = 0;
    if (P.n_rows) {
        const uint64_t npix = static_cast<uint64_t>(P.n_rows) * P.W;
        // per-pixel seeds (a separate launch: measured 0.7 ms faster than deriving
        // them inside the LDS-heavy cost probe)
        const uint64_t seed_threads = static_cast<uint64_t>(P.n_rows) * ((P.W + kSeedRun - 1) / kSeedRun);
        const dim3 g_seed(static_cast<uint32_t>((seed_threads + kBlock - 1) / kBlock));
        // hand-out order: RTW_ORDER=2 (default with a BVH) by estimated cost, 1 rows
        // bottom-up, 0 row-major
        P.order_map = nullptr;
        const bool probe = P.order == 2 && mode == kBvh && P.max_depth > 0;
        // With the probe, the seeds are computed on the session's second stream beside
        // it (the probe draws from its own per-pixel stream) and joined before the
        // persistent kernel: the seed kernel's 0.14 ms leaves the frame's serial part.
        if (probe) {
            HIPCHECK(hipEventRecord(s->ev_fork, st));
            HIPCHECK(hipStreamWaitEvent(s->aux, s->ev_fork, 0));
            hipLaunchKernelGGL(rtw_seed_pixels, g_seed, dim3(kBlock), 0, s->aux, P);
            HIPCHECK(hipGetLastError());
            HIPCHECK(hipEventRecord(s->ev_join, s->aux));
        } else {
            hipLaunchKernelGGL(rtw_seed_pixels, g_seed, dim3(kBlock), 0, st, P);
            HIPCHECK(hipGetLastError());
        }
        if (probe) {
            P.cost = s->d_cost, P.cost_hist = s->d_cost_hist, P.order_map = s->d_order, P.pcost = s->d_pcost;
            const dim3 g1(static_cast<uint32_t>((npix + kBlock - 1) / kBlock));
            const TileGrid tg(P);
            const dim3 gt((tg.count() + kBlock - 1) / kBlock);
            const dim3 gw((tg.count() * 64u + kBlock - 1) / kBlock);  // one wave per tile
            HIPCHECK(hipMemsetAsync(s->d_cost_hist, 0, kCostBuckets * sizeof(uint32_t), st));
            HIPCHECK(hipMemsetAsync(s->d_cost, 0, 2 * static_cast<size_t>(tg.count()) * sizeof(uint32_t), st));
            // full images below 400 samples per pixel probe one pixel per 2x2 block: the
            // probe's ~0.75 ms does not shrink with the samples while the frame does
            // (config 3, s=10: 26.89 -> 26.58 ms, profiles/r06_misc/); small shards keep
            // every pixel's probe (their pre-parking reads it), and so do s >= 20 frames
            // (neutral there, profiles/r02_misc/knob_probe_sub.log)
            const double fill_est = static_cast<double>(npix) / (static_cast<double>(s->n_cu > 0 ? s->n_cu : 256) * kPBlock);
            P.probe_sub = fill_est >= 1.5 && P.n_off < 400u ? 2u : 1u;
            if (const char *e = kn.get("RTW_PROBE_SUB")) P.probe_sub = static_cast<uint32_t>(std::max(1, std::atoi(e)));
            P.probe_cap = kProbeCap, P.hot_segs = kHotSegs;
            if (const char *e = kn.get("RTW_PROBE_CAP")) P.probe_cap = static_cast<uint32_t>(std::max(1, std::atoi(e)));
            if (const char *e = kn.get("RTW_HOT_SEGS")) P.hot_segs = static_cast<uint32_t>(std::max(1, std::atoi(e)));
            if (P.probe_sub > 1) HIPCHECK(hipMemsetAsync(s->d_pcost, 0, npix * sizeof(uint32_t), st));
            // probe: scene + per-lane walk stacks in LDS when they fit, one workgroup per CU
            KParams Q = P;
            Q.lane_lds_off = static_cast<uint32_t>((lds_bytes_for(P.n_sph, P.n_node, P.n_leaf, true, P.n_nbr) + 15) & ~size_t(15));
            const size_t lds_p = Q.lane_lds_off + static_cast<size_t>(kProbeBlock) * rtw_accel::kScratch * sizeof(uint16_t);
            const dim3 gp(static_cast<uint32_t>(std::min<uint64_t>(s->n_cu > 0 ? s->n_cu : 256, (npix + kProbeBlock - 1) / kProbeBlock)));
            if (lds_p <= kLdsCap) hipLaunchKernelGGL(rtw_cost_probe<true>, gp, dim3(kProbeBlock), lds_p, st, Q);
            else hipLaunchKernelGGL(rtw_cost_probe<false>, gp, dim3(kProbeBlock), 0, st, Q);
            // hot pixels only if the probe can reach hot_segs: with the default cap of 8
            // segments per sample (16 per pixel) and hot_segs 20 it cannot, and the two
            // per-pixel launches are skipped. Enabling them measured slower everywhere
            // (RTW_HOT_SEGS=16: N=1 +1.1 %, N=4 rank 60.7 -> 68.5 ms; a deeper probe,
            // RTW_PROBE_CAP=16/24/50: N=1 +0.3/+2.2/+2.7 %, N=4 68-69 ms;
            // profiles/r05_misc/knobs_probe_hot_REJECTED.log): long pixels promoted to
            // the front start together and queue for the drains.
            const bool hot = P.hot_segs <= kProbeSamples * P.probe_cap;
            hipLaunchKernelGGL(rtw_cost_bucket, gt, dim3(kBlock), 0, st, P);
            if (hot) hipLaunchKernelGGL(rtw_cost_hot_bucket, g1, dim3(kBlock), 0, st, P);
            hipLaunchKernelGGL(rtw_cost_scan, dim3(1), dim3(64), 0, st, P);
            hipLaunchKernelGGL(rtw_cost_place, gt, dim3(kBlock), 0, st, P);
            if (hot) hipLaunchKernelGGL(rtw_cost_hot_place, g1, dim3(kBlock), 0, st, P);
            hipLaunchKernelGGL(rtw_cost_scatter, gw, dim3(kBlock), 0, st, P);
            HIPCHECK(hipGetLastError());
        }
        const int pblock = kPBlock;
        int coop_g = 64;  // lanes per parked pixel in the persistent drain (RTW_COOPG=16: 4 per wave)
        if (const char *e = kn.get("RTW_COOPG")) coop_g = std::atoi(e) == 16 ? 16 : 64;
        // LDS: the scene view + pass-1 records when they fit beside the per-lane areas
        const size_t lane_b = lane_lds_bytes(kPBlock);
        bool lds_scene = use_lds && lds + lane_b <= kLdsCap;
        P.lane_lds_off = lds_scene ? static_cast<uint32_t>((lds + 15) & ~size_t(15)) : 0u;
        lds = P.lane_lds_off + lane_b;
        const void *fn = nullptr;
#define RTW_PFN(L, M) reinterpret_cast<const void *>(&rtw_render_persist<L, M, kPBlock>)
        if (coop_g == 64 && lds_scene && mode == kBvh) {
            fn = reinterpret_cast<const void *>(&rtw_render_persist<true, kBvh, kPBlock, 64>);
        } else if (lds_scene) {
            fn = mode == kBvh ? RTW_PFN(true, kBvh) : mode == kScanF32 ? RTW_PFN(true, kScanF32) : RTW_PFN(true, kScanF64);
        } else {
            fn = mode == kBvh ? RTW_PFN(false, kBvh) : mode == kScanF32 ? RTW_PFN(false, kScanF32) : RTW_PFN(false, kScanF64);
        }
#undef RTW_PFN
        int per_cu = 0;
        HIPCHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, pblock, lds));
        if (per_cu < 1) per_cu = 1;
        grid_p = static_cast<uint32_t>(per_cu) * static_cast<uint32_t>(s->n_cu > 0 ? s->n_cu : 256);
        // every CU gets a workgroup even when the shard has fewer pixels than the
        // launch has lanes: pixels then spread over all CUs (shorter per-lane
        // iterations), and the waves left without a pixel drain the park queue
        // heavy waves per workgroup (RTW_HEAVY, default 2): raised priority, parked
        // pixels only. A shard with fewer pixels than cursor lanes (strong scaling
        // at N >= 8) leaves whole waves without a pixel from the start; they drain
        // the park queue too, and no pixel is parked for being late (dry-cursor
        // parking off). Since draining waves raise their priority (drain_prio) the
        // priority waves pay there as well: N=8 rank 54.7 (0) -> 52.2 ms (2), and at
        // N=1 they are worth 15 % (1: 152 ms, 2: 128 ms; profiles/r03_drain1).
        const uint32_t wpb = static_cast<uint32_t>(pblock) / 64u;
        const bool small_shard = npix < static_cast<uint64_t>(grid_p) * (wpb - kHeavyPerBlock) * 64u;
        // A shard of about one pixel per lane (N=4 of the bench image) takes half its
        // waves as priority waves: every pixel starts at once, a cursor lane of a full
        // wave advances a segment every ~20 us, and the chains of more than ~4
        // segments per sample must move to drains early, so the drain needs the waves
        // (rank 67-68 -> 61.4-61.7 ms with the parking rules below; 3 waves: 66-69 ms;
        // N=1, 2, 8 lose with more: profiles/r03_misc/knobs_small_shard_parking.log,
        // knobs_heavy_rate_endgame.log)
        const double fill = static_cast<double>(npix) / (static_cast<double>(grid_p) * pblock);
        const bool small_fill = fill < 1.5;  // strong scaling at N >= 4 of the bench image
        // (fewer samples per pixel, shorter chains, fewer drains wanted: 4 at 100 spp,
        // rank 23.0 -> 17.9 ms at s=10 with the rate rule's earlier start below)
        uint32_t heavy = fill >= 0.75 && small_fill ? (P.n_off >= 400u ? kHeavyPerBlockFull : kHeavyPerBlockFullShort)
                                                    : kHeavyPerBlock;
        if (const char *e = kn.get("RTW_HEAVY")) heavy = static_cast<uint32_t>(std::atoi(e));
        if (heavy >= wpb) heavy = wpb - 1;
        P.heavy_per_block = heavy;
        // priority waves join the cursor once it has handed out kJoinPct % of the
        // pixels (RTW_JOIN=percent, 0 = never): the hot pixels (handed out first) have
        // parked and been drained by then, and the waves would idle (measured: 25-50 %
        // all 159-161 ms, never 168-171 ms, 10 % 173 ms)
        // Only shards of >= 4 x the cursor lanes: in smaller ones the first fill already
        // hands out most pixels, and parks keep coming while the waves would be gone
        // (N=2 rank: 93 -> 111 ms, N=4: 79 -> 103 ms with the join).
        const uint64_t cursor_lanes = static_cast<uint64_t>(grid_p) * (wpb - heavy) * 64u;
        double join_pct = npix >= 4u * cursor_lanes ? kJoinPct : 0.;
        if (const char *e = kn.get("RTW_JOIN")) join_pct = std::atof(e);
        P.join_at = join_pct > 0. ? static_cast<uint32_t>(std::min(npix, static_cast<uint64_t>(
                                        join_pct / 100. * static_cast<double>(npix))))
                                  : 0xffffffffu;
        // waves that signal the end of their cursor loop: priority waves too when they join
        P.n_cursor_waves = P.join_at != 0xffffffffu ? grid_p * wpb : grid_p * (wpb - heavy);
        // Park rules. Full images: after 16 samples above 16 segments per sample. Small
        // shards (spare or half the waves drain): above 10, and a pixel whose 2-sample
        // probe traced >= 16 segments goes to a drain before its first sample -- the
        // longest chains then start draining at once instead of after ~6 ms in a
        // cursor lane (N=8 rank 53.2-53.6 -> 48.3-50.8 ms, N=4 with the priority waves
        // above 61.3-61.8 ms; N=1 and N=2 lose 25-40 % with them: knobs_small_shard_
        // parking.log, knobs_tail_rate.log)
        // In small shards the rate rule starts after ~3 % of the samples (16 of 529, 4 of
        // 100: N=8 rank at s=10 16.3 -> 12.0-12.2 ms, knobs_s10_rate_heavy.log)
        P.rate_k = small_fill ? std::max(4u, static_cast<uint32_t>(std::lround(16. * P.n_off / 529.))) : 16u;
        P.rate_x = small_fill ? 10u : 16u;
        P.prepark = small_fill && P.order_map ? kSmallShardPrepark : 0u;
        // endgame parking: one pixel per drain group once the cursor is dry, in shards
        // of fewer than 2 pixels per lane of the launch (strong scaling at N >= 4: the
        // last chains set the time; N=8 rank 86 -> 65 ms). Full images lose by it (the
        // last pixels are cheap ones, handed out last on purpose: 152.6 -> 157.6 ms).
        // RTW_ENDGAME: the remaining-pixel threshold, 0 = off.
        const bool small_for_endgame = npix < 2u * static_cast<uint64_t>(grid_p) * pblock;
        P.endgame = small_for_endgame ? grid_p * wpb * (64u / static_cast<uint32_t>(coop_g)) : 0u;
        if (const char *e = kn.get("RTW_ENDGAME")) P.endgame = static_cast<uint32_t>(std::atoi(e));
        P.tail_segs = small_shard ? 0xffffffffu
                                  : static_cast<uint32_t>(std::max(64., std::round(kTailSegsPerSample * P.n_off)));
        if (const char *e = kn.get("RTW_TAIL")) P.tail_segs = static_cast<uint32_t>(std::atoi(e));
        if (const char *e = kn.get("RTW_RATE_X")) P.rate_x = static_cast<uint32_t>(std::atoi(e));
        if (const char *e = kn.get("RTW_RATE_K")) P.rate_k = static_cast<uint32_t>(std::atoi(e));
        if (const char *e = kn.get("RTW_DRAIN_OFF")) P.drain_off = std::atoi(e) != 0 ? 1u : 0u;
        // priority waves drain at raised issue priority only in small shards, where the
        // drained chains set the end; in a full image they have the time and their
        // issue-bound segments would take slots from the cursor waves (N=1 123.6 ->
        // 122.2 ms with 0; N=4 rank 60.0 -> 63.1 ms with 0: ab_heavy_prio.log)
        P.drain_prio = 3, P.heavy_prio = small_fill ? 3u : 0u;
        if (const char *e = kn.get("RTW_HEAVY_PRIO")) P.heavy_prio = static_cast<uint32_t>(std::min(3, std::max(0, std::atoi(e))));
        if (const char *e = kn.get("RTW_PREPARK")) P.prepark = static_cast<uint32_t>(std::atoi(e));
        // per-pixel drain priority in a shard of about one pixel per lane (N=4 of the
        // bench image, half the waves drain): only pixels estimated at >= 20 segments per
        // sample (the long serial chains) drain at the raised priority, the others at
        // the cursor waves' -- rank 60.2 -> 56.8 ms (mean of 3 maxima); at N=8 (fewer
        // pixels than lanes) it loses, 48.0 -> 49.4 ms, so it is off there
        // (profiles/r06_misc/knobs_prio_split.log, strong_repeats_prio_split.log)
        P.prio_split = fill >= 0.75 && small_fill ? kPrioSplit8 : 0u;
        // shards with fewer pixels than cursor lanes (N=8 of the bench image): the first
        // fill spreads them over every cursor wave (~40 per wave) instead of filling the
        // first waves and leaving the rest idle (profiles/r06_misc/ab_refill_chunk_wave_cap.log,
        // strong_repeats_wave_cap.log)
        {
            const uint64_t cw = static_cast<uint64_t>(grid_p) * (wpb - heavy);
            P.wave_cap = fill < 0.75 && cw ? static_cast<uint32_t>(std::min<uint64_t>(64u, (npix + cw - 1) / cw)) : 0u;
        }
        if (const char *e = kn.get("RTW_WAVE_CAP")) P.wave_cap = static_cast<uint32_t>(std::min(64, std::max(0, std::atoi(e))));
        if (const char *e = kn.get("RTW_PRIO_SPLIT")) P.prio_split = static_cast<uint32_t>(std::max(0., std::atof(e) * 8.));
        P.spread_q = 0;
        if (const char *e = kn.get("RTW_SPREAD"))
            if (std::atoi(e) != 0 && P.order_map) P.spread_q = static_cast<uint32_t>(npix / 64u);
        if (const char *e = kn.get("RTW_DRAIN_PRIO")) P.drain_prio = static_cast<uint32_t>(std::min(3, std::max(0, std::atoi(e))));
        if (P.rate_x == 0) P.rate_k = 0xffffffffu;  // rate-based parking off
        HIPCHECK(hipMemsetAsync(s->d_park_flag, 0, npix * sizeof(uint32_t), st));
        if (probe) HIPCHECK(hipStreamWaitEvent(st, s->ev_join, 0));  // the seeds are written
        void *args[] = {&P};
        HIPCHECK(hipEventRecord(s->ev_k0, st));
        HIPCHECK(hipLaunchKernel(fn, dim3(grid_p), dim3(pblock), args, lds, st));
        HIPCHECK(hipEventRecord(s->ev_k1, st));
        // entries no group claimed (only after guard exits); returns at once otherwise
        const size_t lds2 = lds_bytes_for(P.n_sph, 0, 0, false) + static_cast<size_t>(P.n_sph) * sizeof(float4);
        const dim3 grid_l(static_cast<uint32_t>(s->n_cu > 0 ? s->n_cu : 256));
        if (lds2 <= kLdsCap) hipLaunchKernelGGL((rtw_park_leftover<true, 64>), grid_l, dim3(kBlock), lds2, st, P);
        else hipLaunchKernelGGL((rtw_park_leftover<false, 64>), grid_l, dim3(kBlock), 0, st, P);
        HIPCHECK(hipGetLastError());
    }
    hipLaunchKernelGGL(rtw_latch_check<uint32_t>, dim3(1), dim3(64), 0, st,
                       static_cast<const uint32_t *>(P.pixels_done),
                       static_cast<uint32_t>(static_cast<uint64_t>(P.n_rows) * P.W), s->d_err);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipEventRecord(s->ev1, st));
    s->last_stream = st;
    s->pending = true;
    s->last = rtw_stats{};
    s->last.pixels = static_cast<uint64_t>(P.n_rows) * P.W;
    s->last.samples = s->last.pixels * P.n_off;
    s->last.grid_blocks = grid_p;
    s->last.block_threads = kPBlock;
    s->last.accel = static_cast<uint32_t>(mode);
    s->last.lds_bytes = static_cast<uint32_t>(lds);
    s->last_fast = false;
    s->main_ev = P.n_rows != 0;
}

// f32 fast mode (rtw_fast.hip): same camera, shard and validation as render().
void render_fast(rtw_session *s, const rtw_camera *cam, uint32_t samples_sqrt, rtw_u128 seed,
                 const rtw_shard *shard_in, float *out, hipStream_t stream) {
    if (!cam || !out) throw rtw::Error(RTW_E_ARG, "null argument");
    if (!s->scene_set) throw rtw::Error(RTW_E_ARG, "session has no scene");
    if (cam->img_height == 0 || cam->img_width == 0)
        throw rtw::Error(RTW_E_EMPTY_IMAGE, "image height and width must be > 0");  // camera.rs:267
    if (samples_sqrt > 65535) throw rtw::Error(RTW_E_UNSUPPORTED, "samples_sqrt > 65535");
    if (static_cast<uint64_t>(cam->img_height) * cam->img_width >= (1ull << 32))
        throw rtw::Error(RTW_E_UNSUPPORTED, "fast mode: image >= 2^32 pixels");
    const rtw_shard sh = resolve_shard(cam, shard_in);
    rtw_fast::FastParams F{};
    auto cp = [](float *d, const rtw_vec3 &v) {
        d[0] = static_cast<float>(v.x), d[1] = static_cast<float>(v.y), d[2] = static_cast<float>(v.z);
    };
    cp(F.p00, cam->pixel00);
    cp(F.du, cam->pixel_delta_u);
    cp(F.dv, cam->pixel_delta_v);
    cp(F.from, cam->look_from);
    cp(F.ddu, cam->defocus_disk_u);
    cp(F.ddv, cam->defocus_disk_v);
    // offset_lattice(&pixel_delta_v, &pixel_delta_u, s) (camera.rs:243-244), in f64 then rounded
    const rtw::Vec3 dxv = rtw::Vec3::of(cam->pixel_delta_v), dyv = rtw::Vec3::of(cam->pixel_delta_u);
    if (samples_sqrt == 0) {
        cp(F.pos0, (dxv / 2. + dyv / 2.).c());
    } else {
        const double n = static_cast<double>(samples_sqrt);
        const rtw::Vec3 dx = dxv / n, dy = dyv / n;
        cp(F.ldx, dx.c());
        cp(F.ldy, dy.c());
        cp(F.pos0, (dx / 2. + dy / 2.).c());
    }
    F.defocus = cam->defocus_angle > 0. ? 1u : 0u;
    F.W = cam->img_width;
    F.s = samples_sqrt;
    F.n_off = samples_sqrt ? samples_sqrt * samples_sqrt : 1;
    F.max_depth = cam->max_depth;
    F.row_begin = sh.row_begin, F.row_step = sh.row_step, F.n_rows = sh.n_rows;
    F.n_sph = s->n_sph;
    // the walk's per-lane stack bounds the BVH depth it can take; deeper trees scan
    const bool walk = s->has_bvh && rtw_fast::stack_slots(s->bvh_depth) <= rtw_fast::kMaxStack;
    F.n_node = walk ? s->n_node : 0;
    F.n_always = walk ? s->n_always : 0;
    F.nodes = s->d_nodes;
    F.always = s->d_always;
    F.n_stack = walk ? rtw_fast::stack_slots(s->bvh_depth) : 0;
    F.cmax = static_cast<float>(std::min(65536., 2147483648. / static_cast<double>(F.n_off)));
    F.seed_mix = seed.lo ^ (seed.hi * 0x9e3779b97f4a7c15ull);
    F.geo = s->d_fgeo, F.mat = s->d_fmat, F.kind = s->d_fkind;
    F.out = out;
    F.cursor = s->d_fcursor;
    F.counters = s->d_fcount;
    hipStream_t st = stream;
    HIPCHECK(hipSetDevice(s->device));
    order_after_last(s, st);
    HIPCHECK(hipEventRecord(s->ev0, st));
    HIPCHECK(hipEventRecord(s->ev_k0, st));
    const rtw::Knobs kn;  // tuning only under RTW_AB (rtw_internal.h)
    const char *lds_knob = kn.get("RTW_FAST_LDS");
    HIPCHECK(rtw_fast::launch(F, s->n_cu, st, !(lds_knob && !std::atoi(lds_knob))));
    HIPCHECK(hipEventRecord(s->ev_k1, st));
    hipLaunchKernelGGL(rtw_latch_check<unsigned long long>, dim3(1), dim3(64), 0, st,
                       static_cast<const unsigned long long *>(s->d_fcount + 2),
                       static_cast<unsigned long long>(F.n_rows) * F.W, s->d_err);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipEventRecord(s->ev1, st));
    s->last_stream = st;
    s->pending = true;
    s->last = rtw_stats{};
    s->last.pixels = static_cast<uint64_t>(F.n_rows) * F.W;
    s->last.samples = s->last.pixels * F.n_off;
    s->last.grid_blocks = static_cast<uint32_t>(std::min<uint64_t>(static_cast<uint64_t>(s->n_cu > 0 ? s->n_cu : 256) * 2,
                                                                   (s->last.pixels + 7) / 8));
    s->last.block_threads = rtw_fast::kBlock;
    s->last.accel = F.n_node ? 2u : 0u;
    bool in_lds = false;
    s->last.lds_bytes = static_cast<uint32_t>(rtw_fast::lds_bytes(F.n_sph, F.n_node, F.n_stack, &in_lds));
    s->last_fast = true;
    s->main_ev = true;
}

// Latched incomplete renders since the last check (rtw_latch_check): reported
// once, then cleared.
void check_latch(rtw_session *s) {
    uint32_t bad = 0;
    HIPCHECK(hipMemcpy(&bad, s->d_err, sizeof bad, hipMemcpyDeviceToHost));
    if (bad) {
        HIPCHECK(hipMemset(s->d_err, 0, sizeof bad));
        throw rtw::Error(RTW_E_HIP, std::to_string(bad) + " render(s) since the last check wrote fewer "
                                    "pixels than the image has (incomplete image)");
    }
}

void collect(rtw_session *s) {
    if (!s->pending) return;
    HIPCHECK(hipSetDevice(s->device));
    HIPCHECK(hipEventSynchronize(s->ev1));
    s->pending = false;
    check_latch(s);
    float main_ms = 0.f;
    if (s->main_ev) HIPCHECK(hipEventElapsedTime(&main_ms, s->ev_k0, s->ev_k1));
    if (s->last_fast) {
        unsigned long long c[5] = {};
        HIPCHECK(hipMemcpy(c, s->d_fcount, sizeof c, hipMemcpyDeviceToHost));
        float ms = 0.f;
        HIPCHECK(hipEventElapsedTime(&ms, s->ev0, s->ev1));
        s->last.segments = c[0];
        s->last.node_visits = c[1];
        s->last.wave_iterations = c[3];
        s->last.exact_wave_iterations = c[4];  // fast mode: wave-level walk iterations (RTW_FAST_DIAG builds)
        s->last.sphere_tests = c[0] * s->n_sph;
        s->last.kernel_ms = ms;
        s->last.main_kernel_ms = main_ms;
        if (c[2] != s->last.pixels)  // never a silently incomplete image
            throw rtw::Error(RTW_E_HIP, "fast render incomplete: " + std::to_string(c[2]) + " of " +
                                            std::to_string(s->last.pixels) + " pixels written");
        return;
    }
    unsigned long long c[kCounters] = {};
    HIPCHECK(hipMemcpy(c, s->d_counters, sizeof c, hipMemcpyDeviceToHost));
#ifdef RTW_WALK_DIAG
    std::fprintf(stderr, "walk_diag: wave-iters %llu, sum max visits all %llu, without camera rays %llu, "
                         "camera rays only %llu; camera-ray segments %llu, their visits %llu; cursor atomics %llu, "
                         "completion atomics %llu, spill-level pushes %llu\n",
                 c[1], c[11], c[12], c[13], c[14], c[15], c[16], c[17], c[18]);
#endif
    float ms = 0.f;
    HIPCHECK(hipEventElapsedTime(&ms, s->ev0, s->ev1));
    s->last.segments = c[0];
    s->last.wave_iterations = c[1];
    s->last.exact_tests = c[2];
    s->last.exact_wave_iterations = c[3];
    s->last.node_visits = c[4];
    s->last.brute_segments = c[5];
    s->last.parked_pixels = c[6];
    s->last.inside_segments = c[8];
    s->last.trap_segments = c[9];
    s->last.guard_exits = c[7];
    s->last.leftover_pixels = c[10];
    s->last.sphere_tests = c[0] * s->n_sph;
    s->last.kernel_ms = ms;
    s->last.main_kernel_ms = s->main_ev ? main_ms : ms;
    uint32_t ctl[8] = {};
    HIPCHECK(hipMemcpy(ctl, s->d_park_ctl, sizeof ctl, hipMemcpyDeviceToHost));
    if (ctl[4] != static_cast<uint32_t>(s->last.pixels))  // never a silently incomplete image
        throw rtw::Error(RTW_E_HIP, "render incomplete: " + std::to_string(ctl[4]) + " of " +
                                        std::to_string(s->last.pixels) + " pixels written");
}

int default_device() {
    const char *e = std::getenv("RTW_DEVICE");
    return e ? std::atoi(e) : 0;
}

void create_session(int device, rtw_session **out) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) throw rtw::Error(RTW_E_NO_DEVICE, "no HIP device");
    if (device < 0 || device >= n) throw rtw::Error(RTW_E_NO_DEVICE, "device index out of range");
    auto *s = new rtw_session();
    s->device = device;
    try {
        HIPCHECK(hipSetDevice(device));
        HIPCHECK(hipStreamCreateWithFlags(&s->own, hipStreamNonBlocking));
        HIPCHECK(hipEventCreate(&s->ev0));
        HIPCHECK(hipEventCreate(&s->ev1));
        HIPCHECK(hipEventCreate(&s->ev_k0));
        HIPCHECK(hipEventCreate(&s->ev_k1));
        HIPCHECK(hipStreamCreateWithFlags(&s->aux, hipStreamNonBlocking));
        HIPCHECK(hipEventCreateWithFlags(&s->ev_fork, hipEventDisableTiming));
        HIPCHECK(hipEventCreateWithFlags(&s->ev_join, hipEventDisableTiming));
        HIPCHECK(hipMalloc(&s->d_counters, kCounters * sizeof(unsigned long long)));
        HIPCHECK(hipMalloc(&s->d_park_ctl, 8 * sizeof(uint32_t)));
        HIPCHECK(hipMalloc(&s->d_err, sizeof(uint32_t)));
        HIPCHECK(hipMemset(s->d_err, 0, sizeof(uint32_t)));
        HIPCHECK(hipMalloc(&s->d_cost_hist, kCostBuckets * sizeof(uint32_t)));
        HIPCHECK(hipMalloc(&s->d_fcursor, sizeof(uint32_t)));
        HIPCHECK(hipMalloc(&s->d_fcount, 8 * sizeof(unsigned long long)));
        HIPCHECK(hipDeviceGetAttribute(&s->n_cu, hipDeviceAttributeMultiprocessorCount, device));
        upload_jump(s);
    } catch (...) {
        rtw_session_destroy(s);
        throw;
    }
    *out = s;
}

}  // namespace

#define RTW_GUARD_BEGIN try {
#define RTW_GUARD_END                         \
    }                                         \
    catch (const rtw::Error &e) {             \
        rtw::set_error(e.what());             \
        return e.code;                        \
    }                                         \
    catch (const std::exception &e) {         \
        rtw::set_error(e.what());             \
        return RTW_E_ARG;                     \
    }

// Sessions the library owns (rtw_shutdown frees them): the one-shot API's session
// of $RTW_DEVICE, and one per entry of rtw_threaded_render_multi's device list.
static std::mutex g_one_mu;
static rtw_session *g_one = nullptr;
static std::mutex g_multi_mu;
static std::vector<rtw_session *> g_multi;

// grow-only device framebuffer of a library-owned session
static void *session_out(rtw_session *s, size_t bytes) {
    bytes = std::max<size_t>(bytes, 8);
    if (bytes > s->out_cap) {
        dev_free(s->d_out);
        s->d_out = nullptr, s->out_cap = 0;
        HIPCHECK(hipMalloc(&s->d_out, bytes));
        s->out_cap = bytes;
    }
    return s->d_out;
}

// Host-buffer render on the cached session of $RTW_DEVICE (the blocking
// Camera::threaded_render shape): upload, enqueue `run`, wait, download.
template <typename T, typename Run>
int threaded(const rtw_camera *cam, const rtw_sphere *spheres, uint32_t n_spheres, const rtw_material *mats,
             uint32_t n_mats, const rtw_shard *shard, T *out_rgb, rtw_stats *stats, Run run) {
    if (!cam || !out_rgb) return rtw::set_error("null argument"), RTW_E_ARG;
    std::lock_guard<std::mutex> lock(g_one_mu);
    RTW_GUARD_BEGIN
    if (cam->img_height == 0 || cam->img_width == 0)
        throw rtw::Error(RTW_E_EMPTY_IMAGE, "image height and width must be > 0");
    validate_scene(spheres, n_spheres, mats, n_mats);
    const rtw_shard sh = resolve_shard(cam, shard);
    const int dev = default_device();
    if (g_one && g_one->device != dev) rtw_session_destroy(g_one), g_one = nullptr;
    if (!g_one) create_session(dev, &g_one);
    set_scene(g_one, spheres, n_spheres, mats, n_mats);
    const size_t bytes = static_cast<size_t>(sh.n_rows) * cam->img_width * 3 * sizeof(T);
    T *d_out = static_cast<T *>(session_out(g_one, bytes));
    run(g_one, &sh, d_out, g_one->own);
    collect(g_one);
    if (bytes) HIPCHECK(hipMemcpy(out_rgb, d_out, bytes, hipMemcpyDeviceToHost));
    if (stats) *stats = g_one->last;
    return RTW_OK;
    RTW_GUARD_END
}

// rtw_threaded_render_multi(_fast): one host thread per device entry, rows r = i mod n.
template <typename T, typename Run>
static int threaded_multi(const rtw_camera *cam, const rtw_sphere *spheres, uint32_t n_spheres, const rtw_material *mats,
                          uint32_t n_mats, const int *devices, uint32_t n_devices, T *out_rgb, rtw_stats *stats,
                          Run run) {
    if (!cam || !out_rgb || (n_devices && !devices)) return rtw::set_error("null argument"), RTW_E_ARG;
    std::lock_guard<std::mutex> lock(g_multi_mu);
    RTW_GUARD_BEGIN
    if (cam->img_height == 0 || cam->img_width == 0)
        throw rtw::Error(RTW_E_EMPTY_IMAGE, "image height and width must be > 0");
    validate_scene(spheres, n_spheres, mats, n_mats);
    int visible = 0;
    if (hipGetDeviceCount(&visible) != hipSuccess || visible == 0) throw rtw::Error(RTW_E_NO_DEVICE, "no HIP device");
    std::vector<int> devs;
    if (n_devices == 0) {
        for (int d = 0; d < visible; ++d) devs.push_back(d);
    } else {
        devs.assign(devices, devices + n_devices);
    }
    for (int d : devs)
        if (d < 0 || d >= visible) throw rtw::Error(RTW_E_NO_DEVICE, "device index out of range");
    const uint32_t H = cam->img_height, W = cam->img_width;
    const uint32_t n = static_cast<uint32_t>(std::min<size_t>(devs.size(), H));  // extra entries: no rows
    if (g_multi.size() < n) g_multi.resize(n, nullptr);
    std::vector<std::thread> workers;
    std::vector<std::exception_ptr> errs(n);
    std::vector<rtw_stats> st(n);
    for (uint32_t i = 0; i < n; ++i) {
        workers.emplace_back([&, i] {
            try {
                rtw_session *&s = g_multi[i];
                if (s && s->device != devs[i]) rtw_session_destroy(s), s = nullptr;
                if (!s) create_session(devs[i], &s);
                HIPCHECK(hipSetDevice(s->device));
                set_scene(s, spheres, n_spheres, mats, n_mats);
                const rtw_shard sh{i, n, (H - i + n - 1) / n, 0};
                const size_t row = static_cast<size_t>(W) * 3 * sizeof(T);
                T *d_out = static_cast<T *>(session_out(s, sh.n_rows * row));
                run(s, &sh, d_out, s->own);
                collect(s);
                // the gather: tile row k -> image row i + k n, one strided copy
                HIPCHECK(hipMemcpy2D(out_rgb + static_cast<size_t>(i) * W * 3, n * row, d_out, row, row, sh.n_rows,
                                     hipMemcpyDeviceToHost));
                st[i] = s->last;
            } catch (...) {
                errs[i] = std::current_exception();
            }
        });
    }
    for (auto &w : workers) w.join();
    for (auto &e : errs)
        if (e) std::rethrow_exception(e);
    if (stats) {
        rtw_stats acc{};
        for (uint32_t i = 0; i < n; ++i) rtw::add_stats(acc, st[i], i == 0);
        *stats = acc;
    }
    return RTW_OK;
    RTW_GUARD_END
}

extern "C" {

int rtw_device_count(int *count) {
    if (!count) return rtw::set_error("null argument"), RTW_E_ARG;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return RTW_OK;
}

int rtw_session_create(int device, rtw_session **out) {
    if (!out) return rtw::set_error("null argument"), RTW_E_ARG;
    RTW_GUARD_BEGIN
    create_session(device, out);
    return RTW_OK;
    RTW_GUARD_END
}

int rtw_session_destroy(rtw_session *s) {
    if (!s) return RTW_OK;
    (void)hipSetDevice(s->device);
    if (s->pending && s->ev1) (void)hipEventSynchronize(s->ev1);
    dev_free(s->d_arena), dev_free(s->d_out);  // the scene tables point into the arena
    dev_free(s->d_jump), dev_free(s->d_tries), dev_free(s->d_counters), dev_free(s->d_spill);
    dev_free(s->d_park), dev_free(s->d_park_ctl), dev_free(s->d_seeds), dev_free(s->d_diag);
    dev_free(s->d_park_flag), dev_free(s->d_order), dev_free(s->d_cost), dev_free(s->d_cost_hist);
    dev_free(s->d_pcost), dev_free(s->d_err);
    dev_free(s->d_fcursor), dev_free(s->d_fcount);
    if (s->ev0) (void)hipEventDestroy(s->ev0);
    if (s->ev1) (void)hipEventDestroy(s->ev1);
    if (s->ev_k0) (void)hipEventDestroy(s->ev_k0);
    if (s->ev_k1) (void)hipEventDestroy(s->ev_k1);
    if (s->own) (void)hipStreamDestroy(s->own);
    if (s->ev_fork) (void)hipEventDestroy(s->ev_fork);
    if (s->ev_join) (void)hipEventDestroy(s->ev_join);
    if (s->aux) (void)hipStreamDestroy(s->aux);
    delete s;
    return RTW_OK;
}

int rtw_session_set_scene(rtw_session *s, const rtw_sphere *spheres, uint32_t n_spheres,
                          const rtw_material *mats, uint32_t n_mats) {
    if (!s) return rtw::set_error("null session"), RTW_E_ARG;
    RTW_GUARD_BEGIN
    set_scene(s, spheres, n_spheres, mats, n_mats);
    return RTW_OK;
    RTW_GUARD_END
}

int rtw_session_render(rtw_session *s, const rtw_camera *cam, uint32_t samples_sqrt,
                       rtw_u128 seed, const rtw_shard *shard, double *out_rgb_device,
                       void *hip_stream) {
    if (!s) return rtw::set_error("null session"), RTW_E_ARG;
    RTW_GUARD_BEGIN
    render(s, cam, samples_sqrt, seed, shard, out_rgb_device, static_cast<hipStream_t>(hip_stream));
    return RTW_OK;
    RTW_GUARD_END
}

int rtw_session_render_fast(rtw_session *s, const rtw_camera *cam, uint32_t samples_sqrt,
                            rtw_u128 seed, const rtw_shard *shard, float *out_rgb_device,
                            void *hip_stream) {
    if (!s) return rtw::set_error("null session"), RTW_E_ARG;
    RTW_GUARD_BEGIN
    render_fast(s, cam, samples_sqrt, seed, shard, out_rgb_device, static_cast<hipStream_t>(hip_stream));
    return RTW_OK;
    RTW_GUARD_END
}

int rtw_session_stats(rtw_session *s, rtw_stats *out) {
    if (!s || !out) return rtw::set_error("null argument"), RTW_E_ARG;
    RTW_GUARD_BEGIN
    collect(s);
    *out = s->last;
    return RTW_OK;
    RTW_GUARD_END
}

int rtw_session_diag(rtw_session *s, uint32_t *out, uint64_t cap) {
    if (!s || (!out && cap)) return rtw::set_error("null argument"), RTW_E_ARG;
    RTW_GUARD_BEGIN
    collect(s);
    if (cap < s->diag_n) throw rtw::Error(RTW_E_CAPACITY, "diag buffer too small");
    if (s->diag_n)
        HIPCHECK(hipMemcpy(out, s->d_diag, s->diag_n * sizeof(uint32_t), hipMemcpyDeviceToHost));
    return RTW_OK;
    RTW_GUARD_END
}

int rtw_threaded_render(const rtw_camera *cam, const rtw_sphere *spheres, uint32_t n_spheres,
                        const rtw_material *mats, uint32_t n_mats, uint32_t samples_sqrt,
                        rtw_u128 seed, const rtw_shard *shard, double *out_rgb, rtw_stats *stats) {
    return threaded(cam, spheres, n_spheres, mats, n_mats, shard, out_rgb, stats,
                    [&](rtw_session *s, const rtw_shard *sh, double *d, hipStream_t st) {
                        render(s, cam, samples_sqrt, seed, sh, d, st);
                    });
}

int rtw_threaded_render_multi(const rtw_camera *cam, const rtw_sphere *spheres, uint32_t n_spheres,
                              const rtw_material *mats, uint32_t n_mats, uint32_t samples_sqrt,
                              rtw_u128 seed, const int *devices, uint32_t n_devices, double *out_rgb,
                              rtw_stats *stats) {
    return threaded_multi(cam, spheres, n_spheres, mats, n_mats, devices, n_devices, out_rgb, stats,
                          [&](rtw_session *s, const rtw_shard *sh, double *d, hipStream_t st) {
                              render(s, cam, samples_sqrt, seed, sh, d, st);
                          });
}

int rtw_threaded_render_multi_fast(const rtw_camera *cam, const rtw_sphere *spheres, uint32_t n_spheres,
                                   const rtw_material *mats, uint32_t n_mats, uint32_t samples_sqrt,
                                   rtw_u128 seed, const int *devices, uint32_t n_devices, float *out_rgb,
                                   rtw_stats *stats) {
    return threaded_multi(cam, spheres, n_spheres, mats, n_mats, devices, n_devices, out_rgb, stats,
                          [&](rtw_session *s, const rtw_shard *sh, float *d, hipStream_t st) {
                              render_fast(s, cam, samples_sqrt, seed, sh, d, st);
                          });
}

int rtw_shutdown(void) {
    std::lock_guard<std::mutex> l1(g_one_mu);
    std::lock_guard<std::mutex> l2(g_multi_mu);
    rtw_session_destroy(g_one);
    g_one = nullptr;
    for (auto *s : g_multi) rtw_session_destroy(s);
    g_multi.clear();
    return RTW_OK;
}

int rtw_threaded_render_fast(const rtw_camera *cam, const rtw_sphere *spheres, uint32_t n_spheres,
                             const rtw_material *mats, uint32_t n_mats, uint32_t samples_sqrt,
                             rtw_u128 seed, const rtw_shard *shard, float *out_rgb, rtw_stats *stats) {
    return threaded(cam, spheres, n_spheres, mats, n_mats, shard, out_rgb, stats,
                    [&](rtw_session *s, const rtw_shard *sh, float *d, hipStream_t st) {
                        render_fast(s, cam, samples_sqrt, seed, sh, d, st);
                    });
}

int rtw_probe_device_seeds(int device, rtw_u128 seed, uint64_t first_pixel, uint64_t count,
                           rtw_u128 *out) {
    if (!out && count) return rtw::set_error("null argument"), RTW_E_ARG;
    rtw_session *s = nullptr;
    U128 *d = nullptr;
    RTW_GUARD_BEGIN
    if (!count) return RTW_OK;
    const uint32_t bits = bit_length(first_pixel + count - 1);
    if (bits > static_cast<uint32_t>(rtw::kJumpBits)) throw rtw::Error(RTW_E_UNSUPPORTED, "pixel index beyond 2^40");
    create_session(device, &s);
    HIPCHECK(hipMalloc(&d, count * sizeof(U128)));
    const unsigned blocks = static_cast<unsigned>((count + 255) / 256);
    hipLaunchKernelGGL(probe_seeds, dim3(blocks), dim3(256), 0, s->own, U128{seed.lo, seed.hi},
                       first_pixel, count, s->d_jump, bits, d);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipStreamSynchronize(s->own));
    HIPCHECK(hipMemcpy(out, d, count * sizeof(U128), hipMemcpyDeviceToHost));
    HIPCHECK(hipFree(d));
    rtw_session_destroy(s);
    return RTW_OK;
    }
    catch (const rtw::Error &e) {
        if (d) (void)hipFree(d);
        rtw_session_destroy(s);
        rtw::set_error(e.what());
        return e.code;
    }
}

#ifdef RTW_STAMPS
// Diagnostic: copies the per-wave stamp rows of the last render (8 u64 each).
int rtw_diag_stamps(uint64_t *out, uint64_t cap_rows, uint64_t *n_rows) {
    *n_rows = stamp_n();
    if (!out || cap_rows < stamp_n()) return RTW_E_CAPACITY;
    (void)hipDeviceSynchronize();
    return hipMemcpy(out, stamp_buf(), stamp_n() * kStampRow * 8, hipMemcpyDeviceToHost) == hipSuccess ? RTW_OK : RTW_E_HIP;
}
#endif

int rtw_probe_f64_ops(int device, const double *a, const double *b, uint64_t n, double *out_sqrt,
                      double *out_div) {
    if ((!a || !b || !out_sqrt || !out_div) && n) return rtw::set_error("null argument"), RTW_E_ARG;
    double *d = nullptr;
    RTW_GUARD_BEGIN
    if (!n) return RTW_OK;
    int cnt = 0;
    if (hipGetDeviceCount(&cnt) != hipSuccess || device < 0 || device >= cnt)
        throw rtw::Error(RTW_E_NO_DEVICE, "no such HIP device");
    HIPCHECK(hipSetDevice(device));
    HIPCHECK(hipMalloc(&d, 4 * n * sizeof(double)));
    HIPCHECK(hipMemcpy(d, a, n * sizeof(double), hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(d + n, b, n * sizeof(double), hipMemcpyHostToDevice));
    const unsigned blocks = static_cast<unsigned>((n + 255) / 256);
    hipLaunchKernelGGL(probe_f64, dim3(blocks), dim3(256), 0, nullptr, d, d + n, n, d + 2 * n, d + 3 * n);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipDeviceSynchronize());
    HIPCHECK(hipMemcpy(out_sqrt, d + 2 * n, n * sizeof(double), hipMemcpyDeviceToHost));
    HIPCHECK(hipMemcpy(out_div, d + 3 * n, n * sizeof(double), hipMemcpyDeviceToHost));
    HIPCHECK(hipFree(d));
    return RTW_OK;
    }
    catch (const rtw::Error &e) {
        if (d) (void)hipFree(d);
        rtw::set_error(e.what());
        return e.code;
    }
}

}  // extern "C"
