/*
 * rtw_oracle.h -- TEST INFRASTRUCTURE ONLY (the parity checker and the CPU
 * baseline). Never linked into, loaded by, or called from the product path.
 *
 * Plain-C restatement of the reference's per-pixel sampling path
 * (NicoElbers/Raytracing_in_a_weekend_rust @ 2025-12-05). Every function in
 * rtw_oracle.c cites the reference file:line it restates.
 *
 * Parity status: the reference publishes no pixel/RNG fixtures. Its own tests
 * pin only Interval::contains_inc/contains_ex (src/util/interval.rs:65-145) and
 * the offset_lattice sizes (src/raytracing/camera.rs:481-488); both are
 * re-checked here (tests/test_oracle.py). Render values are otherwise
 * "parity unpinned" by reference fixtures; they are cross-checked bit-for-bit
 * against a second, independent restatement (oracle/pyoracle.py, pure Python).
 *
 * Struct layouts are plain data, identical byte-for-byte to include/rtw_capi.h
 * so a test can pass the same buffers to both (the oracle does not include the
 * product header on purpose).
 */
#ifndef RTW_ORACLE_H
#define RTW_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { double x, y, z; } orc_vec3;

typedef struct {                 /* derived Camera values, camera.rs:138-221 */
    uint32_t img_height, img_width, max_depth, _pad0;
    double focal_length, fov;
    orc_vec3 look_from, look_to, vup;
    orc_vec3 u, v, w;
    double viewport_height, viewport_width;
    orc_vec3 pixel00, pixel_delta_u, pixel_delta_v;
    double defocus_angle, focus_dist;
    orc_vec3 defocus_disk_u, defocus_disk_v;
} orc_camera;

enum { ORC_LAMBERTIAN = 0, ORC_METAL = 1, ORC_DIELECTRIC = 2 };

typedef struct {                 /* materials.rs:11-111 */
    uint32_t kind, _pad;
    double albedo[3];
    double fuzz;
    double ir;
} orc_material;

typedef struct {                 /* sphere.rs:11-16 */
    double center[3];
    double radius;
    uint32_t mat, _pad;
} orc_sphere;

/* XorShift (random.rs:3-70). u128 passed as (lo, hi) halves. */
void orc_xs_next_int(uint64_t lo, uint64_t hi, uint32_t n, uint64_t *out /*2n*/);
void orc_xs_next_01(uint64_t lo, uint64_t hi, uint32_t n, double *out);
void orc_xs_copy_reset_chain(uint64_t lo, uint64_t hi, uint64_t n, uint64_t *out /*2n*/);

/* Interval (interval.rs:55-62) */
int orc_interval_contains_inc(double min, double max, double x);
int orc_interval_contains_ex(double min, double max, double x);

/* Camera::new (camera.rs:138-221) */
void orc_camera_new(uint32_t h, uint32_t w, uint32_t max_depth, double focal_length,
                    double fov, const double from[3], const double to[3], const double vup[3],
                    double defocus_angle, double focus_dist, orc_camera *out);

/* Camera::offset_lattice (camera.rs:422-450). Returns count (s==0 -> 1, else s*s). */
uint32_t orc_offset_lattice(const double dx[3], const double dy[3], uint32_t s, double *out /*3*count*/);

/* raytracing::complex scene (mod.rs:62-103). Returns sphere count (== material count). */
uint32_t orc_scene_complex(uint64_t lo, uint64_t hi, orc_sphere *sph, orc_material *mat, uint32_t cap);

/* Render rows {row_begin + k*row_step : k < n_rows} of the image.
 * scheduler 0 = "ref-faithful": one job per pixel pulled by nthreads workers,
 *   function-pointer dispatch per object (dyn Hittable / dyn Material) and an
 *   atomic refcount bump per candidate hit (Arc clone, sphere.rs:69).
 * scheduler 1 = "clean": rows pulled by nthreads workers, direct calls.
 * out: n_rows*W*3 f64 (row-major). segments (nullable): traced segments total.
 * Returns 0 on success, <0 on bad arguments. */
int orc_render(const orc_camera *cam, const orc_sphere *sph, uint32_t n_sph,
               const orc_material *mat, uint32_t n_mat, uint32_t samples_sqrt,
               uint64_t seed_lo, uint64_t seed_hi, uint32_t row_begin, uint32_t row_step,
               uint32_t n_rows, uint32_t nthreads, int scheduler, double *out,
               uint64_t *segments);

/* Render an explicit ascending list of image rows (same schedulers, same per-pixel
 * children as a whole-image render). row_segments (nullable): traced segments per
 * listed row. */
int orc_render_rows(const orc_camera *cam, const orc_sphere *sph, uint32_t n_sph,
                    const orc_material *mat, uint32_t n_mat, uint32_t samples_sqrt,
                    uint64_t seed_lo, uint64_t seed_hi, const uint32_t *rows, uint32_t n_rows,
                    uint32_t nthreads, int scheduler, double *out, uint64_t *segments,
                    uint64_t *row_segments);

/* Color::wire_full_file (color.rs:196-247). Writes into buf (cap bytes); returns
 * bytes needed (call with buf=NULL to size). */
uint64_t orc_format_ppm(const double *rgb, uint32_t w, uint32_t h, char *buf, uint64_t cap);

#ifdef __cplusplus
}
#endif
#endif
