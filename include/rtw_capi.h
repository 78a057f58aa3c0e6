/*
 * rtw_capi.h -- C ABI of the MI355X-native sampling path (librtw.so).
 *
 * Drop-in boundary for NicoElbers/Raytracing_in_a_weekend_rust's per-pixel hot
 * path. The reference has no FFI; its swappable seam is
 *   Camera::threaded_render(cam: &Arc<Camera>, world: &Arc<dyn Hittable>,
 *                           samples_sqrt: usize) -> Result<(), Box<dyn Error>>
 *   (src/raytracing/camera.rs:223-227, called from src/raytracing/mod.rs:123)
 * whose per-ray trait calls (Hittable::hit, hittable.rs:12-14; Material::scatter,
 * materials.rs:7-9) are far too fine-grained to cross a device boundary. So the
 * boundary is at whole-image granularity: the host flattens the scene (spheres +
 * material table) and the derived Camera, and one call renders all pixels.
 * The Rust-side binding a maintainer would add (bindgen + cc) is shown in
 * INTEGRATION.md.
 *
 * All structs are POD and bindgen-clean. All calls are synchronous unless noted,
 * return RTW_OK (0) or a negative RTW_E_* code, never abort, and leave a
 * thread-local message in rtw_last_error(). The caller owns every host buffer for
 * the duration of a call; nothing is retained after return.
 */
#ifndef RTW_CAPI_H
#define RTW_CAPI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RTW_ABI_VERSION 7

/* ---- error codes ---- */
#define RTW_OK 0
#define RTW_E_ARG (-1)          /* null pointer / bad size / bad shard                 */
#define RTW_E_EMPTY_IMAGE (-2)  /* height or width 0: assert!, camera.rs:267           */
#define RTW_E_FUZZ (-3)         /* Metal fuzz > 1: assert!, materials.rs:47            */
#define RTW_E_MAT_INDEX (-4)    /* sphere refers to a material that does not exist     */
#define RTW_E_HIP (-5)          /* HIP runtime error (message in rtw_last_error)       */
#define RTW_E_UNSUPPORTED (-6)  /* limits of this build (max_depth, table sizes)       */
#define RTW_E_NO_DEVICE (-7)    /* no usable gfx950 device                             */
#define RTW_E_CAPACITY (-8)     /* caller buffer too small (count written anyway)      */

/* ---- plain data ---- */
typedef struct rtw_vec3 { double x, y, z; } rtw_vec3;           /* Vec3/Point3/Color, vec3.rs:9-14 */
typedef struct rtw_u128 { uint64_t lo, hi; } rtw_u128;          /* XorShift state, random.rs:3-6   */

/* Camera after Camera::new (camera.rs:138-221): the derived values the path reads. */
typedef struct rtw_camera {
    uint32_t img_height, img_width, max_depth, _pad0;
    double focal_length, fov;                 /* stored, unused by the path (as in the reference) */
    rtw_vec3 look_from, look_to, vup;
    rtw_vec3 u, v, w;                         /* BasisVecs, camera.rs:96-100                  */
    double viewport_height, viewport_width;
    rtw_vec3 pixel00, pixel_delta_u, pixel_delta_v;
    double defocus_angle, focus_dist;
    rtw_vec3 defocus_disk_u, defocus_disk_v;
} rtw_camera;

/* Material table row: Lambertian{albedo} (materials.rs:11-14), Metal{albedo,fuzz}
 * (39-43), Dielectric{ir} (65-68). Unused fields are ignored. */
enum { RTW_LAMBERTIAN = 0, RTW_METAL = 1, RTW_DIELECTRIC = 2 };
typedef struct rtw_material {
    uint32_t kind, _pad;
    double albedo[3];
    double fuzz;
    double ir;
} rtw_material;

/* Sphere{center, radius, mat} (sphere.rs:11-16); mat indexes the material table. */
typedef struct rtw_sphere {
    double center[3];
    double radius;
    uint32_t mat, _pad;
} rtw_sphere;

/* Rows row_begin + k*row_step for k < n_rows (row-cyclic multi-GPU shards).
 * NULL shard = the whole image. Output row k of a shard is image row
 * row_begin + k*row_step; per-pixel RNG streams depend only on the global pixel
 * index, so any shard reproduces the unsharded pixels bit-for-bit. */
typedef struct rtw_shard { uint32_t row_begin, row_step, n_rows, _pad; } rtw_shard;

typedef struct rtw_stats {
    uint64_t pixels;          /* pixels rendered                                       */
    uint64_t samples;         /* pixels x lattice offsets (samples_sqrt^2, or 1 if 0)  */
    uint64_t segments;        /* traced segments = Scene::hit calls                    */
    uint64_t sphere_tests;    /* segments x n_spheres (brute force, as the reference)  */
    uint64_t wave_iterations; /* sum over waves of the wave's loop trip count          */
    uint64_t exact_tests;     /* f64 sphere tests run after the conservative filter    */
    uint64_t exact_wave_iterations; /* wave-level iterations of the exact-test loop
                                       (fast mode: of the BVH walk loop, diagnostic
                                       builds with -DRTW_FAST_DIAG; else 0)           */
    double kernel_ms;         /* render kernel time, HIP events on the launch stream   */
    uint32_t grid_blocks, block_threads;
    uint64_t node_visits;     /* BVH walk iterations (inner-node or leaf tests), lanes  */
    uint64_t brute_segments;  /* segments the BVH path re-did by brute-force scan      */
    uint32_t accel;           /* 0 brute-force f64, 1 f32-filtered scan, 2 BVH         */
    uint32_t lds_bytes;       /* dynamic LDS per workgroup                             */
    uint64_t parked_pixels;   /* pixels finished by the cooperative second kernel      */
    uint64_t inside_segments; /* segments resolved by the inside cut (rtw_accel.h)     */
    uint64_t trap_segments;   /* segments skipped by the trapped-path fast-forward      */
    /* ABI 5: */
    uint64_t guard_exits;     /* idle waits of the persistent kernel ended by its
                                 no-progress guard ($RTW_SPIN_GUARD_MS, default 100)   */
    uint64_t leftover_pixels; /* parked pixels finished by the follow-up launch (after
                                 guard exits; 0 on an exclusive device)                 */
    /* ABI 6: */
    double main_kernel_ms;    /* the main render kernel alone (persistent / fast kernel),
                                 HIP events around its launch; kernel_ms spans every
                                 launch of the render (seeds, cost order, main, leftover) */
} rtw_stats;

/* ---- library ---- */
const char *rtw_version(void);
/* RTW_ABI_VERSION the library was built with. A client compares it with the
 * RTW_ABI_VERSION of the header it was compiled against before passing any struct
 * (rtw_stats grew in ABI 5 and ABI 6). */
int rtw_abi_version(void);
/* Hash of the library's sources and device flags (profiles/ counter files are
 * stamped with it). */
const char *rtw_build_id(void);
const char *rtw_last_error(void);
int rtw_device_count(int *count);
/* Frees every device resource the library owns: the sessions behind
 * rtw_threaded_render(_fast) and rtw_threaded_render_multi. Sessions the caller
 * created with rtw_session_create stay the caller's. The next one-shot call
 * re-creates what it needs. Not to be called while another thread renders. */
int rtw_shutdown(void);

/* ---- host mirror of the reference types (bit-exact f64, no FMA) ---- */
/* Camera::new(img_height, img_width, max_depth, focal_length, fov, look_from,
 * look_to, vup, defocus_angle, focus_dist, None) -- camera.rs:138-150.
 * Note the reference's argument order: height before width. */
int rtw_camera_new(uint32_t img_height, uint32_t img_width, uint32_t max_depth,
                   double focal_length, double fov, const rtw_vec3 *look_from,
                   const rtw_vec3 *look_to, const rtw_vec3 *vup, double defocus_angle,
                   double focus_dist, rtw_camera *out);

/* Camera::offset_lattice(dx, dy, num_layers) -- camera.rs:422-450 (the render
 * calls it as (pixel_delta_v, pixel_delta_u, s), camera.rs:243-244). */
int rtw_offset_lattice(const rtw_vec3 *dx, const rtw_vec3 *dy, uint32_t samples_sqrt,
                       rtw_vec3 *out, uint32_t cap, uint32_t *count);

/* Interval::contains_inc / contains_ex -- interval.rs:55-62 */
int rtw_interval_contains_inc(double min, double max, double x);
int rtw_interval_contains_ex(double min, double max, double x);

/* XorShift::next_int / next_01 streams from `seed` (random.rs:33-52). */
int rtw_xorshift_next_int(rtw_u128 seed, uint32_t n, rtw_u128 *out);
int rtw_xorshift_next_01(rtw_u128 seed, uint32_t n, double *out);
/* Children handed to pixels first_pixel .. first_pixel+count-1 by the row-major
 * copy_reset chain of threaded_render (camera.rs:255, 269-272; random.rs:61-69),
 * computed by GF(2) jump-ahead (no serial walk). */
int rtw_seed_children(rtw_u128 seed, uint64_t first_pixel, uint64_t count, rtw_u128 *out);

/* Built-in scenes (raytracing/mod.rs). name: "complex" (54-126, the book's final
 * scene; `seed` replaces the wall-clock XorShift::default at mod.rs:67),
 * "simple" (129-173), "threads" (176-202), "super_simple" (205-238), and
 * "three_lambertian" (BASELINE config 1: simple() with the dielectric dropped and
 * the metal sphere made Lambertian). img_height/img_width/max_depth override the
 * builder's hard-coded values when non-zero. Writes up to `cap` spheres and
 * materials; *n_spheres / *n_mats receive the full counts. */
int rtw_scene_builtin(const char *name, rtw_u128 seed, uint32_t img_height, uint32_t img_width,
                      uint32_t max_depth, rtw_camera *cam, rtw_sphere *spheres,
                      rtw_material *mats, uint32_t cap, uint32_t *n_spheres, uint32_t *n_mats);

/* Color::wire_full_file (color.rs:196-247) on an H*W*3 f64 framebuffer (row 0 =
 * top). rtw_format_ppm returns the byte count (writes only if buf && cap
 * suffice); rtw_write_ppm writes the file. */
int64_t rtw_format_ppm(const double *rgb, uint32_t width, uint32_t height, char *buf,
                       uint64_t cap);
int rtw_write_ppm(const char *path, const double *rgb, uint32_t width, uint32_t height);

/* ---- the hot path ---- */
/* Camera::threaded_render equivalent: renders `shard` (NULL = all rows) of the
 * scene into out_rgb (host, n_rows*W*3 f64, row-major), on device 0 (or
 * $RTW_DEVICE). Per-pixel RNG: child p of `seed` (random.rs:61-69). Validation
 * mirrors the reference's asserts. stats may be NULL. */
int rtw_threaded_render(const rtw_camera *cam, const rtw_sphere *spheres, uint32_t n_spheres,
                        const rtw_material *mats, uint32_t n_mats, uint32_t samples_sqrt,
                        rtw_u128 seed, const rtw_shard *shard, double *out_rgb,
                        rtw_stats *stats);

/* Camera::threaded_render on several GPUs of this node (camera.rs:223-227; the
 * reference's pool takes every core, camera.rs:253 -- this takes every listed GPU).
 * `devices` holds n_devices device indices; NULL or 0 = every visible device. An
 * index may repeat: every entry gets its own session, stream and host thread.
 * Rows are dealt cyclically -- image row r goes to entry r % n_devices (sky rows
 * are cheap, ground rows are not) -- and each entry copies its rows straight into
 * their places in out_rgb (host, H*W*3 f64) with one strided device-to-host copy:
 * the gather needs no collective because the result is a host buffer. Pixels and
 * their RNG streams depend only on the global pixel index, so the image is
 * bit-identical to rtw_threaded_render's. stats (nullable): counters summed over
 * the entries, kernel_ms = the slowest entry's render. */
int rtw_threaded_render_multi(const rtw_camera *cam, const rtw_sphere *spheres, uint32_t n_spheres,
                              const rtw_material *mats, uint32_t n_mats, uint32_t samples_sqrt,
                              rtw_u128 seed, const int *devices, uint32_t n_devices, double *out_rgb,
                              rtw_stats *stats);

/* rtw_threaded_render_multi in f32 fast mode (ABI 7; see rtw_session_render_fast):
 * same device list, row dealing and strided gather into out_rgb (host, H*W*3 f32). */
int rtw_threaded_render_multi_fast(const rtw_camera *cam, const rtw_sphere *spheres,
                                   uint32_t n_spheres, const rtw_material *mats, uint32_t n_mats,
                                   uint32_t samples_sqrt, rtw_u128 seed, const int *devices,
                                   uint32_t n_devices, float *out_rgb, rtw_stats *stats);

/* rtw_threaded_render in f32 fast mode (see rtw_session_render_fast). */
int rtw_threaded_render_fast(const rtw_camera *cam, const rtw_sphere *spheres, uint32_t n_spheres,
                             const rtw_material *mats, uint32_t n_mats, uint32_t samples_sqrt,
                             rtw_u128 seed, const rtw_shard *shard, float *out_rgb,
                             rtw_stats *stats);

/* Device-resident sessions: scene uploaded once, renders enqueued on a caller
 * stream into a caller device buffer (inputs already in HBM when timing). */
typedef struct rtw_session rtw_session;
int rtw_session_create(int device, rtw_session **out);
int rtw_session_destroy(rtw_session *s);
int rtw_session_set_scene(rtw_session *s, const rtw_sphere *spheres, uint32_t n_spheres,
                          const rtw_material *mats, uint32_t n_mats);
/* Asynchronous: enqueues the render of `shard` on `hip_stream` (a hipStream_t;
 * NULL = HIP's null stream, as everywhere in HIP) writing out_rgb_device (device
 * pointer, n_rows*W*3 f64).
 * Concurrency: all renders of one session share its device buffers, so at most
 * one runs at a time -- a render enqueued on a different stream than the
 * session's previous render waits for it (hipStreamWaitEvent). Use one session
 * per concurrent render. Completeness (one write per pixel) is checked on the
 * device after EVERY render and latched: rtw_session_stats fails if any render
 * since its previous call was incomplete, even if later renders were enqueued
 * before it was called.
 * Residency: the persistent kernel (one workgroup per CU) is fastest with the
 * device to itself, but never depends on all of its workgroups being resident at
 * once: waves that wait for parked pixels leave after $RTW_SPIN_GUARD_MS (default
 * 100) without progress anywhere, and a follow-up launch finishes any parked
 * pixel they left (rtw_stats.guard_exits / leftover_pixels). */
int rtw_session_render(rtw_session *s, const rtw_camera *cam, uint32_t samples_sqrt,
                       rtw_u128 seed, const rtw_shard *shard, double *out_rgb_device,
                       void *hip_stream);
/* f32 fast mode (SURVEY 8(c) "Fast mode"; the ABI sketch's rtw_mode FAST_F32):
 * the same camera, scene, materials and depth rule in f32, with independent
 * xoroshiro64** streams per (pixel, lattice sample) instead of the reference's
 * per-pixel XorShift chain. NOT bit-exact: statistically equal to the parity
 * render (tests/test_gpu_fast.py). Deterministic, and any shard reproduces the
 * unsharded pixels bit-for-bit. Output: n_rows*W*3 f32. Per-sample colours are
 * clamped to [0, min(65536, 2^31 / spp)] (NaN -> 0). */
int rtw_session_render_fast(rtw_session *s, const rtw_camera *cam, uint32_t samples_sqrt,
                            rtw_u128 seed, const rtw_shard *shard, float *out_rgb_device,
                            void *hip_stream);
/* Waits for the session's last render and reports its statistics. */
int rtw_session_stats(rtw_session *s, rtw_stats *out);
/* Diagnostic (not part of the reference surface): per-pixel records of the last
 * render when it ran with RTW_DIAG=1 in the environment -- for pixel p of the
 * shard (row-major), out[2p] = traced segments of the pixel in the one-lane
 * kernel, out[2p+1] = low 32 bits of the 100 MHz device real-time clock when
 * the pixel completed (0 = never ran); out[2 x pixels] = the clock at the persistent
 * launch's start. Returns RTW_E_CAPACITY if cap < 2 x pixels + 4. */
int rtw_session_diag(rtw_session *s, uint32_t *out, uint64_t cap);

/* ---- device-resident multi-GPU renders (ABI 7) ----
 * A group is the node-level Camera::threaded_render (camera.rs:223-352; the
 * reference's pool takes every core, camera.rs:253 -- a group takes every listed
 * GPU) with the image left in HBM: one session per entry of `devices` (NULL or 0
 * entries = every visible device; an index may repeat), image row r rendered by
 * entry r % n, the row tiles gathered on the root device (entry 0) and
 * un-permuted there into the caller's device buffer. The gather is one ncclGather
 * over xGMI (RCCL communicators from ncclCommInitAll) when the entries are
 * distinct GPUs, device-to-device copies otherwise (a repeated device, or
 * RTW_GROUP_COPY_GATHER). If RCCL cannot be loaded or its communicators fail to
 * come up, the group falls back to the copy gather (peer access over xGMI) and
 * says why (rtw_group_info.fallback, rtw_group_note); only RTW_GROUP_RCCL_ALWAYS
 * makes that an error. Renders are blocking: on return the image is complete in
 * out_rgb_device. The root device's first write to out_rgb_device is ordered
 * after the work already queued on that device's null stream (or on the caller's
 * stream: rtw_group_render_on). Every rtw_group_*
 * call restores the caller's current HIP device. Bit-identical to a one-device
 * render. */
typedef struct rtw_group rtw_group;
#define RTW_GROUP_COPY_GATHER 1u /* flags: never RCCL, gather by device copies          */
#define RTW_GROUP_RCCL_ALWAYS 2u /* flags: RCCL gather even for a one-entry group; no
                                    fallback: an RCCL failure is an error (tests)      */
#define RTW_GROUP_RCCL_TRY 4u    /* flags: RCCL gather for a one-entry group too, with
                                    the fallback (tests of the fallback on one GPU)    */
enum { RTW_GATHER_NONE = 0, RTW_GATHER_COPY = 1, RTW_GATHER_RCCL = 2 };
enum { RTW_FALLBACK_NONE = 0, RTW_FALLBACK_NO_RCCL = 1, RTW_FALLBACK_COMM_INIT = 2 };
typedef struct rtw_group_info {
    uint32_t n_entries;     /* entries that rendered rows in the last render (min(n, H)) */
    uint32_t gather;        /* RTW_GATHER_* the last render used                        */
    double wall_ms;         /* host wall time of the last rtw_group_render(_fast)       */
    double render_ms_max;   /* slowest entry's render (HIP events on its own stream)     */
    double root_gather_ms;  /* root stream, from its own tile rendered to the image
                               complete: waiting for the other entries + gather +
                               un-permute                                               */
    uint32_t fast;          /* the last render was f32 fast mode                        */
    uint32_t fallback;      /* RTW_FALLBACK_*: why the group gathers by copies although
                               its entries are distinct GPUs (RCCL unloadable, or
                               ncclCommInitAll failed); text in rtw_group_note       */
} rtw_group_info;
int rtw_group_create(const int *devices, uint32_t n_devices, uint32_t flags, rtw_group **out);
int rtw_group_destroy(rtw_group *g);
int rtw_group_set_scene(rtw_group *g, const rtw_sphere *spheres, uint32_t n_spheres,
                        const rtw_material *mats, uint32_t n_mats);
/* out_rgb_device: H*W*3 f64 on the root device. */
int rtw_group_render(rtw_group *g, const rtw_camera *cam, uint32_t samples_sqrt, rtw_u128 seed,
                     double *out_rgb_device);
/* f32 fast mode; out_rgb_device: H*W*3 f32 on the root device. */
int rtw_group_render_fast(rtw_group *g, const rtw_camera *cam, uint32_t samples_sqrt,
                          rtw_u128 seed, float *out_rgb_device);
/* The same, ordered after the work queued on caller_stream (a hipStream_t of the root
 * device; NULL = its null stream, what rtw_group_render does) instead of the null
 * stream: a caller inside torch.cuda.stream(s), or on a per-thread default stream,
 * passes that stream. Still blocking. */
int rtw_group_render_on(rtw_group *g, const rtw_camera *cam, uint32_t samples_sqrt, rtw_u128 seed,
                        double *out_rgb_device, void *caller_stream);
int rtw_group_render_fast_on(rtw_group *g, const rtw_camera *cam, uint32_t samples_sqrt,
                             rtw_u128 seed, float *out_rgb_device, void *caller_stream);
/* Last render: total (counters summed, times the slowest entry's; nullable),
 * per_entry[0..n_entries) (nullable; RTW_E_CAPACITY if cap < n_entries) and info
 * (nullable). */
int rtw_group_stats(rtw_group *g, rtw_stats *total, rtw_stats *per_entry, uint32_t cap,
                    rtw_group_info *info);
/* Why the group fell back from RCCL to the copy gather ("" if it did not). Owned by
 * the group, valid until rtw_group_destroy. */
const char *rtw_group_note(rtw_group *g);
/* 1 if RCCL (librccl.so.1 with ncclCommInitAll/ncclGather) can be loaded, else 0 with
 * the reason in why[0..cap) (nullable). Needs no GPU. */
int rtw_rccl_available(char *why, size_t cap);

/* ---- device probes (tests) ---- */
/* Device jump-ahead seeds (the kernel's own code path) for a pixel range. */
int rtw_probe_device_seeds(int device, rtw_u128 seed, uint64_t first_pixel, uint64_t count,
                           rtw_u128 *out);
/* Device f64 sqrt(a) and a/b, to check correct rounding against the host. */
int rtw_probe_f64_ops(int device, const double *a, const double *b, uint64_t n,
                      double *out_sqrt, double *out_div);

#ifdef __cplusplus
}
#endif
#endif /* RTW_CAPI_H */
