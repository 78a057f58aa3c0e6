// rtw_host.h -- C++ host mirror of the reference's trait surface for the sampling
// path (NicoElbers/Raytracing_in_a_weekend_rust, src/raytracing + src/space +
// src/util). Same names, argument order and error behaviour; arithmetic is f64 in
// the reference's operation order (built with -ffp-contract=off, no FMA).
//
// What crosses the device boundary is the flattened scene (rtw_sphere[] +
// rtw_material[]) and the derived camera; Hittable::flatten / Material::flatten
// are the trait extension a Rust drop-in would add.
#pragma once

#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "rtw_capi.h"
#include "rtw_internal.h"  // rtw::Error

namespace rtw {

using u128 = unsigned __int128;

inline u128 to_u128(rtw_u128 v) { return (static_cast<u128>(v.hi) << 64) | v.lo; }
inline rtw_u128 from_u128(u128 v) {
    return rtw_u128{static_cast<uint64_t>(v), static_cast<uint64_t>(v >> 64)};
}

// ---- Vec3 / Point3 / Color (src/space/vec3.rs, point3.rs, raytracing/color.rs) ----
struct Vec3 {
    double x = 0, y = 0, z = 0;
    constexpr Vec3() = default;
    constexpr Vec3(double x_, double y_, double z_) : x(x_), y(y_), z(z_) {}
    Vec3 operator+(const Vec3 &o) const { return {x + o.x, y + o.y, z + o.z}; }  // vec3.rs:28-42
    Vec3 operator-(const Vec3 &o) const { return {x - o.x, y - o.y, z - o.z}; }  // vec3.rs:44-58
    Vec3 operator-() const { return {-x, -y, -z}; }                              // vec3.rs:60-70
    Vec3 operator*(double s) const { return {x * s, y * s, z * s}; }             // vec3.rs:72-82
    Vec3 operator/(double s) const { return {x / s, y / s, z / s}; }             // vec3.rs:110-120
    Vec3 operator*(const Vec3 &o) const { return {x * o.x, y * o.y, z * o.z}; }  // color.rs:60-70
    double len_squared() const { return x * x + y * y + z * z; }                 // vec3.rs:150-152
    double len() const;                                                          // vec3.rs:155-157
    static double dot(const Vec3 &a, const Vec3 &b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
    Vec3 cross(const Vec3 &r) const {                                            // vec3.rs:170-180
        return {y * r.z - z * r.y, z * r.x - x * r.z, x * r.y - y * r.x};
    }
    Vec3 unit() const { return *this / len(); }                                  // vec3.rs:183-185
    rtw_vec3 c() const { return rtw_vec3{x, y, z}; }
    static Vec3 of(const rtw_vec3 &v) { return {v.x, v.y, v.z}; }
};
inline Vec3 operator*(double s, const Vec3 &v) { return v * s; }  // `f64 * Vec3` = vec * self
using Point3 = Vec3;
using Color = Vec3;

// ---- XorShift (src/util/random.rs:3-70) ----
class XorShift {
   public:
    explicit constexpr XorShift(u128 seed) : state_(seed) {}  // XorShift::new, random.rs:29-31
    u128 next_int();                                          // random.rs:33-38
    double next_01();                                         // random.rs:40-52
    double next_bound(double min, double max);                // random.rs:54-59
    XorShift copy_reset();                                    // random.rs:61-69
    u128 state() const { return state_; }

   private:
    u128 state_;
};
Color color_random(XorShift &r);  // color.rs:249-255

// GF(2) jump-ahead for the copy_reset chain: state_p = T^p(seed), T = next_int.
// cols[k*128 + j] = T^(2^k)(e_j), k < kJumpBits.
constexpr int kJumpBits = 40;
const std::vector<u128> &jump_table();
// The trapped-path replay's lane table (rtw_render.hip trap_forward): for each bit b of
// a 128-bit state (b < 64: lo bit b, else hi bit b - 64) and lane j < 64,
// tries[b * 64 + j] = T^(3 j)(e_b) -- lane j's RNG state at the start of the j-th
// 3-draw try after a wave-uniform state s is the XOR over s's set bits. Row 128 is zero.
constexpr int kTryLanes = 64;
const std::vector<u128> &try_table();
u128 jump(u128 state, uint64_t p);
u128 copy_reset_of(u128 parent_state);  // child handed out by copy_reset at this parent state

// ---- materials (src/raytracing/materials.rs) ----
struct Material {
    virtual ~Material() = default;
    virtual rtw_material flatten() const = 0;
};
struct Lambertian final : Material {  // materials.rs:11-20
    Color albedo;
    explicit Lambertian(Color a) : albedo(a) {}
    rtw_material flatten() const override;
};
struct Metal final : Material {  // materials.rs:39-50: assert!(fuzz <= 1.)
    Color albedo;
    double fuzz;
    Metal(Color a, double f);
    rtw_material flatten() const override;
};
struct Dielectric final : Material {  // materials.rs:65-73
    double ir;
    explicit Dielectric(double i) : ir(i) {}
    rtw_material flatten() const override;
};

// ---- hittables (src/raytracing/hittable.rs, shapes/sphere.rs) ----
struct FlatScene {
    std::vector<rtw_sphere> spheres;
    std::vector<rtw_material> materials;
    std::unordered_map<const Material *, uint32_t> mat_index;  // Arc identity -> table row
    uint32_t intern(const std::shared_ptr<Material> &m);
};
struct Hittable {
    virtual ~Hittable() = default;
    virtual void flatten(FlatScene &out) const = 0;  // trait extension
};
struct Sphere final : Hittable {  // sphere.rs:11-37
    Point3 center;
    double radius;
    std::shared_ptr<Material> mat;
    Sphere(Point3 c, double r, std::shared_ptr<Material> m) : center(c), radius(r), mat(std::move(m)) {}
    static std::shared_ptr<Sphere> new_world_obj(double x, double y, double z, double radius,
                                                 std::shared_ptr<Material> m);
    void flatten(FlatScene &out) const override;
};
struct Scene final : Hittable {  // hittable.rs:119-143 (objects in insertion order)
    std::vector<std::shared_ptr<Hittable>> objects;
    void flatten(FlatScene &out) const override;
};
class SceneBuilder {  // hittable.rs:86-117
   public:
    void add(std::shared_ptr<Hittable> obj) { objects_.push_back(std::move(obj)); }
    // An empty builder yields a scene holding only `Empty` (always misses),
    // which flattens to zero spheres (hittable.rs:98-106, 145-152).
    std::shared_ptr<Scene> build();

   private:
    std::vector<std::shared_ptr<Hittable>> objects_;
};

// ---- camera (src/raytracing/camera.rs) ----
struct Camera {
    rtw_camera d{};
    // Camera::new, camera.rs:138-221 (height first, as in the reference)
    static Camera new_(uint32_t img_height, uint32_t img_width, uint32_t max_depth,
                       double focal_length, double fov, Point3 look_from, Point3 look_to,
                       Vec3 vup, double defocus_angle, double focus_dist);
    uint32_t width() const { return d.img_width; }
    uint32_t height() const { return d.img_height; }
    // camera.rs:422-450
    static std::vector<Vec3> offset_lattice(const Vec3 &dx, const Vec3 &dy, uint32_t num_layers);
    // camera.rs:223-352: renders on the GPUs of this node and writes `ppm_path`
    // ("img.ppm" in the reference); returns the f64 framebuffer (H*W*3). The
    // reference's pool takes every core (camera.rs:253): an empty `devices` takes
    // every visible GPU (rtw_threaded_render_multi), else the listed ones (an index
    // may repeat). Throws on error.
    static std::vector<double> threaded_render(const Camera &cam, const Scene &world,
                                               uint32_t samples_sqrt, rtw_u128 seed,
                                               const char *ppm_path = "img.ppm",
                                               rtw_stats *stats = nullptr,
                                               const std::vector<int> &devices = {});
};

// ---- scenes (src/raytracing/mod.rs) ----
struct BuiltScene {
    Camera cam;
    std::shared_ptr<Scene> world;
};
// name: complex | simple | threads | super_simple | three_lambertian
BuiltScene build_scene(const std::string &name, rtw_u128 seed, uint32_t h, uint32_t w,
                       uint32_t max_depth);

// ---- output (color.rs:196-247) ----
std::string format_ppm(const double *rgb, uint32_t w, uint32_t h);
// the same text as the header followed by row-block chunks (no concatenation)
std::vector<std::string> format_ppm_parts(const double *rgb, uint32_t w, uint32_t h);

}  // namespace rtw
