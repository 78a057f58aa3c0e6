// rtw_fast.h -- the f32 "fast mode" render: the same camera,
// scene, materials and depth rule as the reference's ray_color (camera.rs:376-398),
// computed in f32 with independent random streams per (pixel, sample), so that a
// pixel's samples run in parallel instead of as one serial chain. Not bit-exact
// by design: its gate is statistical against the f64 parity render.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace rtw_fast {

// Launch parameters (host-derived camera values as f32; scene tables on device).
struct FastParams {
    float p00[3], du[3], dv[3];  // get_ray: pixel_loc = (pixel00 + i du) + j dv
    float from[3], ddu[3], ddv[3];  // look_from, defocus disk basis
    float pos0[3], ldx[3], ldy[3];  // offset_lattice (camera.rs:422-450)
    uint32_t defocus;               // 1: origins on the defocus disk (camera.rs:406-410)
    uint32_t W, s, n_off, max_depth;
    uint32_t row_begin, row_step, n_rows;
    uint32_t n_sph, n_node, n_always;
    uint32_t n_stack;  // per-lane stack slots (stack_slots(depth)); 0 with n_node = 0
    float cmax;        // per-sample colour clamp of the fixed-point sum (2^32 n_off cmax < 2^63)
    uint64_t seed_mix; // render seed folded to 64 bits
    const float4 *geo;      // {cx, cy, cz, r} per sphere
    const float4 *mat;      // Lambertian/Metal {albedo, fuzz}; Dielectric {1/ir, ir, r0^2, 0}
    const uint32_t *kind;   // RTW_LAMBERTIAN / RTW_METAL / RTW_DIELECTRIC per sphere
    const float4 *nodes;    // rtw_accel.h 4-wide nodes (n_node = 0: brute-force scan)
    const uint32_t *always; // spheres tested before the walk (rtw_accel.h)
    float *out;             // n_rows x W x 3 f32
    uint32_t *cursor;       // pixel hand-out counter (zeroed by the launcher)
    unsigned long long *counters;  // [0] segments, [1] node visits, [2] pixels written, [3] wave iterations,
                                   // [4] wave-level walk iterations
};

constexpr uint32_t kBlock = 512;   // 8 waves per workgroup, two per CU (LDS-bound: 640 measured 25% slower)
constexpr uint32_t kMaxStack = 32;  // per-lane BVH stack cap (u16 node ids)
constexpr uint32_t kLdsCap = 79 * 1024;  // two workgroups per CU (160 KB), with the static ring sums

// Stack slots a walk of a BVH of this depth needs: 3 pending siblings per level
// + the top write (the root is level 0). Deeper trees than kMaxStack allows scan.
// The scene tables follow the stacks: n_stack x kBlock x 2 bytes stays 16-aligned.
static_assert(kBlock % 8 == 0, "stack area alignment");
constexpr uint32_t stack_slots(uint32_t depth) { return 3 * depth + 2; }

// Dynamic LDS bytes of a launch: the stacks, plus the scene tables when they fit
// (*scene_in_lds); otherwise the kernel reads the scene from global memory.
size_t lds_bytes(uint32_t n_sph, uint32_t n_node, uint32_t n_stack, bool *scene_in_lds);

// Enqueues the render (zeroes the cursor and counters first).
hipError_t launch(const FastParams &P, int n_cu, hipStream_t st, bool scene_lds = true);

}  // namespace rtw_fast
