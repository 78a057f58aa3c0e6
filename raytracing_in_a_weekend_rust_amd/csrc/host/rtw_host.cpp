// rtw_host.cpp -- host mirror of the reference types + the host-side half of the
// C ABI (include/rtw_capi.h). Compiled with -O2 -ffp-contract=off: every f64
// expression below is evaluated in the reference's order, without contraction,
// so Camera::new and the scene builders produce the reference's bits.
#include "rtw_host.h"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <exception>
#include <thread>

#include "rtw_internal.h"

namespace rtw {

// ------------------------------------------------------------------ errors --
static thread_local std::string g_last_error;
void set_error(const std::string &m) { g_last_error = m; }
const char *last_error() { return g_last_error.c_str(); }

// -------------------------------------------------------------------- math --
double Vec3::len() const { return std::sqrt(len_squared()); }

u128 XorShift::next_int() {
    state_ ^= state_ << 23;
    state_ ^= state_ >> 17;
    state_ ^= state_ << 26;
    return state_;
}
double XorShift::next_01() {
    const u128 next = next_int();
    const uint32_t b = static_cast<uint32_t>(next % static_cast<u128>(0xFFFFFFFFu));
    return static_cast<double>(b) / 4294967295.0;
}
double XorShift::next_bound(double min, double max) {
    const double diff = max - min;
    const double next = next_01();
    return min + diff * next;
}
XorShift XorShift::copy_reset() {
    const u128 self_state = state_;
    u128 r = self_state ^ next_int();
    r ^= r >> 13;
    r ^= r << 5;
    r ^= r >> 11;
    return XorShift(r);
}
Color color_random(XorShift &r) {
    const double a = r.next_01();
    const double b = r.next_01();
    const double c = r.next_01();
    return {a, b, c};
}

u128 copy_reset_of(u128 parent_state) {
    XorShift p(parent_state);
    return p.copy_reset().state();
}

// GF(2) matrices of T^(2^k); T (one next_int step) is linear over GF(2)^128.
static u128 apply_cols(const u128 *cols, u128 v) {
    u128 r = 0;
    for (int j = 0; j < 128; ++j)
        if ((v >> j) & 1) r ^= cols[j];
    return r;
}
const std::vector<u128> &jump_table() {
    static std::vector<u128> table;
    static std::once_flag once;
    std::call_once(once, [] {
        table.resize(static_cast<size_t>(kJumpBits) * 128);
        for (int j = 0; j < 128; ++j) {
            XorShift x(static_cast<u128>(1) << j);
            table[j] = x.next_int();
        }
        for (int k = 1; k < kJumpBits; ++k)
            for (int j = 0; j < 128; ++j)
                table[k * 128 + j] = apply_cols(&table[(k - 1) * 128], table[(k - 1) * 128 + j]);
    });
    return table;
}
u128 jump(u128 state, uint64_t p) {
    const auto &t = jump_table();
    for (int k = 0; k < kJumpBits && p; ++k, p >>= 1)
        if (p & 1) state = apply_cols(&t[k * 128], state);
    if (p) throw Error(RTW_E_UNSUPPORTED, "pixel index beyond 2^40");
    return state;
}

// --------------------------------------------------------------- materials --
Metal::Metal(Color a, double f) : albedo(a), fuzz(f) {
    if (!(f <= 1.)) throw Error(RTW_E_FUZZ, "Fuzz cannot be more than 1");  // materials.rs:47
}
rtw_material Lambertian::flatten() const {
    rtw_material m{};
    m.kind = RTW_LAMBERTIAN;
    m.albedo[0] = albedo.x, m.albedo[1] = albedo.y, m.albedo[2] = albedo.z;
    return m;
}
rtw_material Metal::flatten() const {
    rtw_material m{};
    m.kind = RTW_METAL;
    m.albedo[0] = albedo.x, m.albedo[1] = albedo.y, m.albedo[2] = albedo.z;
    m.fuzz = fuzz;
    return m;
}
rtw_material Dielectric::flatten() const {
    rtw_material m{};
    m.kind = RTW_DIELECTRIC;
    m.ir = ir;
    return m;
}

// --------------------------------------------------------------- hittables --
uint32_t FlatScene::intern(const std::shared_ptr<Material> &m) {
    auto it = mat_index.find(m.get());
    if (it != mat_index.end()) return it->second;
    const uint32_t idx = static_cast<uint32_t>(materials.size());
    materials.push_back(m->flatten());
    mat_index.emplace(m.get(), idx);
    return idx;
}
std::shared_ptr<Sphere> Sphere::new_world_obj(double x, double y, double z, double radius,
                                              std::shared_ptr<Material> m) {
    return std::make_shared<Sphere>(Point3(x, y, z), radius, std::move(m));
}
void Sphere::flatten(FlatScene &out) const {
    rtw_sphere s{};
    s.center[0] = center.x, s.center[1] = center.y, s.center[2] = center.z;
    s.radius = radius;
    s.mat = out.intern(mat);
    out.spheres.push_back(s);
}
void Scene::flatten(FlatScene &out) const {
    for (const auto &o : objects) o->flatten(out);
}
std::shared_ptr<Scene> SceneBuilder::build() {
    auto s = std::make_shared<Scene>();
    s->objects = std::move(objects_);  // empty -> `Empty`: flattens to nothing
    return s;
}

// ------------------------------------------------------------------ camera --
static inline double to_radians(double deg) { return deg * (M_PI / 180.0); }  // f64::to_radians

Camera Camera::new_(uint32_t img_height, uint32_t img_width, uint32_t max_depth,
                    double focal_length, double fov, Point3 look_from, Point3 look_to, Vec3 vup,
                    double defocus_angle, double focus_dist) {
    // camera.rs:151-191
    const double theta = to_radians(fov);
    const double h = std::tan(theta / 2.);
    const double viewport_height = 2. * h * focus_dist;
    const double viewport_width =
        viewport_height * (static_cast<double>(img_width) / static_cast<double>(img_height));
    const Vec3 w = (look_from - look_to).unit();
    const Vec3 u = vup.cross(w).unit();
    const Vec3 v = w.cross(u);
    const Vec3 viewport_u = viewport_width * u;
    const Vec3 viewport_v = viewport_height * -v;
    const Vec3 pixel_delta_u = viewport_u / static_cast<double>(img_width);
    const Vec3 pixel_delta_v = viewport_v / static_cast<double>(img_height);
    const Point3 pixel00 = look_from - (focus_dist * w) - viewport_u / 2. - viewport_v / 2.;
    const double defocus_radius = focus_dist * std::tan(to_radians(defocus_angle / 2.));

    Camera c;
    c.d.img_height = img_height;
    c.d.img_width = img_width;
    c.d.max_depth = max_depth;
    c.d.focal_length = focal_length;
    c.d.fov = fov;
    c.d.look_from = look_from.c();
    c.d.look_to = look_to.c();
    c.d.vup = vup.c();
    c.d.u = u.c();
    c.d.v = v.c();
    c.d.w = w.c();
    c.d.viewport_height = viewport_height;
    c.d.viewport_width = viewport_width;
    c.d.pixel00 = pixel00.c();
    c.d.pixel_delta_u = pixel_delta_u.c();
    c.d.pixel_delta_v = pixel_delta_v.c();
    c.d.defocus_angle = defocus_angle;
    c.d.focus_dist = focus_dist;
    c.d.defocus_disk_u = (u * defocus_radius).c();
    c.d.defocus_disk_v = (v * defocus_radius).c();
    return c;
}

std::vector<Vec3> Camera::offset_lattice(const Vec3 &dx_in, const Vec3 &dy_in,
                                         uint32_t num_layers) {
    if (num_layers == 0) return {dx_in / 2. + dy_in / 2.};
    const double n = static_cast<double>(num_layers);
    const Vec3 dx = dx_in / n;
    const Vec3 dy = dy_in / n;
    const Vec3 pos0 = dx / 2. + dy / 2.;
    std::vector<Vec3> offsets;
    offsets.reserve(static_cast<size_t>(num_layers) * num_layers);
    for (uint32_t y = 0; y < num_layers; ++y) {
        const Vec3 pos = pos0 + dy * static_cast<double>(y);
        for (uint32_t x = 0; x < num_layers; ++x) offsets.push_back(pos + dx * static_cast<double>(x));
    }
    return offsets;
}

std::vector<double> Camera::threaded_render(const Camera &cam, const Scene &world,
                                            uint32_t samples_sqrt, rtw_u128 seed,
                                            const char *ppm_path, rtw_stats *stats) {
    FlatScene flat;
    world.flatten(flat);
    std::vector<double> fb(static_cast<size_t>(cam.width()) * cam.height() * 3);
    const int rc = rtw_threaded_render(&cam.d, flat.spheres.data(),
                                       static_cast<uint32_t>(flat.spheres.size()),
                                       flat.materials.data(),
                                       static_cast<uint32_t>(flat.materials.size()), samples_sqrt,
                                       seed, nullptr, fb.data(), stats);
    if (rc != RTW_OK) throw Error(rc, last_error());
    if (ppm_path && rtw_write_ppm(ppm_path, fb.data(), cam.width(), cam.height()) != RTW_OK)
        throw Error(RTW_E_ARG, last_error());
    return fb;
}

// ------------------------------------------------------------------ scenes --
// raytracing/mod.rs:38-51
static constexpr double FOCAL_LENGTH = 1.0;
static constexpr double FOV = 20.;
static constexpr uint32_t MAX_DEPTH = 10;
static constexpr Point3 LOOK_FROM{13., 2., 3.};
static constexpr Point3 LOOK_TO{0., 0., 0.};
static constexpr Vec3 VUP{0., 1., 0.};
static constexpr double DEFOCUS_ANGLE = 0.6;
static constexpr double FOCUS_DIST = 10.0;

static uint32_t pick(uint32_t v, uint32_t dflt) { return v ? v : dflt; }

BuiltScene build_scene(const std::string &name, rtw_u128 seed, uint32_t h, uint32_t w,
                       uint32_t max_depth) {
    BuiltScene out;
    SceneBuilder world;
    if (name == "complex") {  // mod.rs:54-126; Config defaults 1080x1920 (main.rs:20-29)
        world.add(Sphere::new_world_obj(0., -1000., 0., 1000.,
                                        std::make_shared<Lambertian>(Color(0.5, 0.5, 0.5))));
        XorShift rand(to_u128(seed));  // replaces XorShift::default() (mod.rs:67)
        for (int a = -11; a < 11; ++a) {
            for (int b = -11; b < 11; ++b) {
                const double choose_mat = rand.next_01();
                const double cx = static_cast<double>(a) + 0.9 * rand.next_01();
                const double cz = static_cast<double>(b) + 0.9 * rand.next_01();
                const Point3 center(cx, 0.2, cz);
                const Vec3 point_vec = center - Point3(4., 0.2, 0.);
                if (point_vec.len() > 0.9) {
                    std::shared_ptr<Material> mat;
                    if (choose_mat < 0.34) {
                        const Color c1 = color_random(rand);
                        const Color c2 = color_random(rand);
                        mat = std::make_shared<Lambertian>(c1 * c2);
                    } else if (choose_mat < 0.67) {
                        const Color c1 = color_random(rand);
                        const Color c2 = color_random(rand);
                        const double fuzz = rand.next_bound(0., 1.);
                        mat = std::make_shared<Metal>(c1 * c2, fuzz);
                    } else {
                        mat = std::make_shared<Dielectric>(1.5);
                    }
                    world.add(std::make_shared<Sphere>(center, 0.2, mat));
                }
            }
        }
        world.add(Sphere::new_world_obj(0., 1., 0., 1., std::make_shared<Dielectric>(1.5)));
        world.add(Sphere::new_world_obj(-4., 1., 0., 1.,
                                        std::make_shared<Lambertian>(Color(0.4, 0.2, 0.1))));
        world.add(Sphere::new_world_obj(4., 1., 0., 1.,
                                        std::make_shared<Metal>(Color(0.7, 0.6, 0.5), 0.0)));
        out.cam = Camera::new_(pick(h, 1080), pick(w, 1920), pick(max_depth, MAX_DEPTH),
                               FOCAL_LENGTH, FOV, LOOK_FROM, LOOK_TO, VUP, DEFOCUS_ANGLE,
                               FOCUS_DIST);
    } else if (name == "simple" || name == "three_lambertian") {  // mod.rs:129-173
        const bool three = name == "three_lambertian";
        out.cam = Camera::new_(pick(h, three ? 225 : 1080), pick(w, three ? 400 : 1920),
                               pick(max_depth, three ? 8 : 25), 1.0, 20.0, Point3(-2., 2., 1.),
                               Point3(0., 0., -1.), Vec3(0., 1., 0.), 10.0, 3.4);
        auto ground = std::make_shared<Lambertian>(Color(0.8, 0.8, 0.0));
        auto center = std::make_shared<Lambertian>(Color(0.1, 0.2, 0.5));
        world.add(Sphere::new_world_obj(0., -100.5, -1., 100., ground));
        world.add(Sphere::new_world_obj(0., 0., -1., 0.5, center));
        if (three) {  // BASELINE config 1: dielectric dropped, metal -> Lambertian
            world.add(Sphere::new_world_obj(1., 0., -1., 0.5,
                                            std::make_shared<Lambertian>(Color(0.8, 0.6, 0.2))));
        } else {
            world.add(Sphere::new_world_obj(-1., 0., -1., 0.5, std::make_shared<Dielectric>(1.5)));
            world.add(Sphere::new_world_obj(1., 0., -1., 0.5,
                                            std::make_shared<Metal>(Color(0.8, 0.6, 0.2), 0.)));
        }
    } else if (name == "threads" || name == "super_simple") {  // mod.rs:176-238
        out.cam = Camera::new_(pick(h, 1000), pick(w, 1000), pick(max_depth, 50), 1.0, 50.0,
                               Point3(0., 0., 0.), Point3(0., 0., -0.3), Vec3(0., 1., 0.), 0.6,
                               10.0);
        world.add(Sphere::new_world_obj(0., -100.5, -1., 100.,
                                        std::make_shared<Lambertian>(Color(0.8, 0.8, 0.0))));
    } else {
        throw Error(RTW_E_ARG, "unknown scene '" + name + "'");
    }
    out.world = world.build();
    return out;
}

// ------------------------------------------------------------------ output --
// Rust `f64 as u64`: saturating, NaN -> 0
static inline uint64_t sat_u64(double v) {
    if (!(v > 0.)) return 0;
    if (v >= 18446744073709551616.0) return UINT64_MAX;
    return static_cast<uint64_t>(v);
}
// gamma_correct + quantise (color.rs:241-247): (c.powf(1/2.2) * 255.0) as u64.
static inline uint64_t quantise_pow(double c) { return sat_u64(std::pow(c, 1. / 2.2) * 255.); }
static inline uint64_t bits_of(double x) {
    uint64_t u;
    std::memcpy(&u, &x, 8);
    return u;
}
// The same value without a pow call for c in (0, 1): c's value is the number of
// thresholds T_1..T_255 it reaches, T_k = the smallest double with quantise_pow >= k
// (found once by bisection over the bit patterns of [0, 1], with the library pow
// itself). pow is accurate to < 1 ulp, and near T_k the true c^(1/2.2) x 255 moves
// by ~0.45 ulp per ulp of c, so any wobble of the rounded result around k stays
// within a few ulps of T_k: inputs within kNear ulps of a threshold, c >= 1 and
// c <= 0 / NaN take quantise_pow itself. Equal to quantise_pow for every input
// (tests/test_host_abi.py checks millions of them and every threshold's neighbourhood).
struct GammaTable {
    static constexpr uint64_t kNear = 64;
    uint64_t t[257];  // t[0] = 0, t[k] = bits of T_k, t[256] = bits of 1.0
    GammaTable() {
        t[0] = 0;
        for (uint32_t k = 1; k <= 255; ++k) {
            uint64_t lo = t[k - 1], hi = bits_of(1.0);  // quantise_pow(lo) < k <= quantise_pow(hi)
            while (hi - lo > 1) {
                const uint64_t mid = lo + (hi - lo) / 2;
                double m;
                std::memcpy(&m, &mid, 8);
                if (quantise_pow(m) >= k) hi = mid;
                else lo = mid;
            }
            t[k] = hi;
        }
        t[256] = bits_of(1.0);
    }
    uint64_t operator()(double c) const {
        if (!(c > 0.) || !(c < 1.)) return quantise_pow(c);
        const uint64_t b = bits_of(c);
        uint32_t k = 0;  // largest k with t[k] <= b (t[0] = 0 <= b)
        for (uint32_t step = 128; step; step >>= 1)
            if (k + step <= 255 && t[k + step] <= b) k += step;
        if (b - t[k] < kNear || (k < 255 && t[k + 1] - b <= kNear)) return quantise_pow(c);
        return k;
    }
};
static const GammaTable &gamma_table() {
    static const GammaTable g;
    return g;
}
uint64_t quantise_channel(double c, bool direct) { return direct ? quantise_pow(c) : gamma_table()(c); }

// Decimal text of 0..255 (the values of a [0, 1] channel): length + digits.
struct SmallDigits {
    char d[256][4];
    uint8_t n[256];
    SmallDigits() {
        for (uint32_t v = 0; v < 256; ++v) n[v] = static_cast<uint8_t>(std::snprintf(d[v], 4, "%u", v));
    }
};
static void format_rows(const double *rgb, uint32_t w, uint32_t y0, uint32_t y1, std::string &s) {
    static const SmallDigits sd;
    const GammaTable &gt = gamma_table();
    std::vector<char> line(static_cast<size_t>(w) * 3 * 21 + 1);  // 20 digits + separator each
    for (uint32_t y = y0; y < y1; ++y) {
        const double *row = rgb + static_cast<size_t>(y) * w * 3;
        char *o = line.data();
        for (uint64_t i = 0; i < 3ull * w; ++i) {
            uint64_t v = gt(row[i]);  // gamma_correct, color.rs:241-247
            if (v < 256) {
                std::memcpy(o, sd.d[v], 4);  // 4 bytes copied, n[v] kept
                o += sd.n[v];
            } else {
                char tmp[24];
                char *e = tmp + sizeof tmp, *b = e;  // decimal digits, right to left
                do {
                    *--b = static_cast<char>('0' + v % 10u);
                    v /= 10u;
                } while (v);
                std::memcpy(o, b, static_cast<size_t>(e - b));
                o += e - b;
            }
            *o++ = ' ';
        }
        if (o != line.data()) o[-1] = '\n';  // color.rs:226-233: one text line per image row
        s.append(line.data(), static_cast<size_t>(o - line.data()));
    }
}
// color.rs:196-239. Rows are formatted in parallel chunks (the reference's
// single-threaded fold is the output edge's cost at 4096x2304).
std::vector<std::string> format_ppm_parts(const double *rgb, uint32_t w, uint32_t h) {
    unsigned nt = std::thread::hardware_concurrency();
    nt = nt ? (nt > 16 ? 16 : nt) : 1;
    if (static_cast<uint64_t>(w) * h < 65536) nt = 1;
    std::vector<std::string> parts(nt + 1);
    parts[0] = "P3\n" + std::to_string(w) + " " + std::to_string(h) + "\n255\n";
    // Exception safety: a worker's exception (bad_alloc of a ~100 MB part) is
    // caught into its slot and rethrown after every thread has joined; the joiner
    // also runs when this thread throws (thread creation, its own chunk), so no
    // joinable std::thread is ever destroyed (which would std::terminate).
    std::vector<std::exception_ptr> errs(nt);
    std::vector<std::thread> th;
    struct Joiner {
        std::vector<std::thread> &t;
        ~Joiner() {
            for (auto &x : t)
                if (x.joinable()) x.join();
        }
    } joiner{th};
    th.reserve(nt);
    for (unsigned t = 0; t < nt; ++t) {
        const uint32_t y0 = static_cast<uint32_t>(static_cast<uint64_t>(h) * t / nt);
        const uint32_t y1 = static_cast<uint32_t>(static_cast<uint64_t>(h) * (t + 1) / nt);
        std::string &part = parts[t + 1];
        std::exception_ptr &err = errs[t];
        auto work = [=, &part, &err] {
            try {
                part.reserve(static_cast<size_t>(y1 - y0) * w * 12);  // allocated in the worker
                format_rows(rgb, w, y0, y1, part);
            } catch (...) {
                err = std::current_exception();
            }
        };
        if (t + 1 == nt) work();
        else th.emplace_back(work);
    }
    for (auto &x : th) x.join();
    for (auto &e : errs)
        if (e) std::rethrow_exception(e);
    return parts;
}
std::string format_ppm(const double *rgb, uint32_t w, uint32_t h) {
    std::string s;
    for (const auto &p : format_ppm_parts(rgb, w, h)) s += p;
    return s;
}

}  // namespace rtw

// ===================================================================== C ABI ==
using namespace rtw;

#define RTW_GUARD_BEGIN try {
#define RTW_GUARD_END                                  \
    }                                                  \
    catch (const rtw::Error &e) {                      \
        rtw::set_error(e.what());                      \
        return e.code;                                 \
    }                                                  \
    catch (const std::exception &e) {                  \
        rtw::set_error(e.what());                      \
        return RTW_E_ARG;                              \
    }

extern "C" {

const char *rtw_version(void) { return "rtw-mi355x 0.5.0 (abi 5, gfx950)"; }
const char *rtw_last_error(void) { return rtw::last_error(); }

int rtw_camera_new(uint32_t img_height, uint32_t img_width, uint32_t max_depth,
                   double focal_length, double fov, const rtw_vec3 *look_from,
                   const rtw_vec3 *look_to, const rtw_vec3 *vup, double defocus_angle,
                   double focus_dist, rtw_camera *out) {
    if (!look_from || !look_to || !vup || !out) return set_error("null argument"), RTW_E_ARG;
    RTW_GUARD_BEGIN
    *out = Camera::new_(img_height, img_width, max_depth, focal_length, fov, Vec3::of(*look_from),
                        Vec3::of(*look_to), Vec3::of(*vup), defocus_angle, focus_dist)
               .d;
    return RTW_OK;
    RTW_GUARD_END
}

int rtw_offset_lattice(const rtw_vec3 *dx, const rtw_vec3 *dy, uint32_t samples_sqrt,
                       rtw_vec3 *out, uint32_t cap, uint32_t *count) {
    if (!dx || !dy || !count) return set_error("null argument"), RTW_E_ARG;
    RTW_GUARD_BEGIN
    const auto v = Camera::offset_lattice(Vec3::of(*dx), Vec3::of(*dy), samples_sqrt);
    *count = static_cast<uint32_t>(v.size());
    if (!out || cap < v.size()) return set_error("lattice buffer too small"), RTW_E_CAPACITY;
    for (size_t i = 0; i < v.size(); ++i) out[i] = v[i].c();
    return RTW_OK;
    RTW_GUARD_END
}

int rtw_interval_contains_inc(double min, double max, double x) { return min <= x && x <= max; }
int rtw_interval_contains_ex(double min, double max, double x) { return min < x && x < max; }

int rtw_xorshift_next_int(rtw_u128 seed, uint32_t n, rtw_u128 *out) {
    if (!out && n) return set_error("null argument"), RTW_E_ARG;
    XorShift x(to_u128(seed));
    for (uint32_t i = 0; i < n; ++i) out[i] = from_u128(x.next_int());
    return RTW_OK;
}
int rtw_xorshift_next_01(rtw_u128 seed, uint32_t n, double *out) {
    if (!out && n) return set_error("null argument"), RTW_E_ARG;
    XorShift x(to_u128(seed));
    for (uint32_t i = 0; i < n; ++i) out[i] = x.next_01();
    return RTW_OK;
}
int rtw_seed_children(rtw_u128 seed, uint64_t first_pixel, uint64_t count, rtw_u128 *out) {
    if (!out && count) return set_error("null argument"), RTW_E_ARG;
    RTW_GUARD_BEGIN
    XorShift parent(jump(to_u128(seed), first_pixel));
    for (uint64_t i = 0; i < count; ++i) out[i] = from_u128(parent.copy_reset().state());
    return RTW_OK;
    RTW_GUARD_END
}

int rtw_scene_builtin(const char *name, rtw_u128 seed, uint32_t img_height, uint32_t img_width,
                      uint32_t max_depth, rtw_camera *cam, rtw_sphere *spheres,
                      rtw_material *mats, uint32_t cap, uint32_t *n_spheres, uint32_t *n_mats) {
    if (!name || !n_spheres || !n_mats) return set_error("null argument"), RTW_E_ARG;
    RTW_GUARD_BEGIN
    BuiltScene b = build_scene(name, seed, img_height, img_width, max_depth);
    FlatScene flat;
    b.world->flatten(flat);
    *n_spheres = static_cast<uint32_t>(flat.spheres.size());
    *n_mats = static_cast<uint32_t>(flat.materials.size());
    if (cam) *cam = b.cam.d;
    if (flat.spheres.size() > cap || flat.materials.size() > cap) {
        set_error("scene buffers too small");
        return RTW_E_CAPACITY;
    }
    if (spheres) std::memcpy(spheres, flat.spheres.data(), flat.spheres.size() * sizeof(rtw_sphere));
    if (mats) std::memcpy(mats, flat.materials.data(), flat.materials.size() * sizeof(rtw_material));
    return RTW_OK;
    RTW_GUARD_END
}

int64_t rtw_format_ppm(const double *rgb, uint32_t width, uint32_t height, char *buf,
                       uint64_t cap) {
    if (!rgb && width && height) return set_error("null argument"), RTW_E_ARG;
    try {
        const auto parts = format_ppm_parts(rgb, width, height);
        size_t n = 0;
        for (const auto &p : parts) n += p.size();
        if (buf && cap >= n)
            for (const auto &p : parts) std::memcpy(buf, p.data(), p.size()), buf += p.size();
        return static_cast<int64_t>(n);
    } catch (const std::exception &e) {
        set_error(e.what());
        return RTW_E_ARG;
    }
}

int rtw_write_ppm(const char *path, const double *rgb, uint32_t width, uint32_t height) {
    if (!path || (!rgb && width && height)) return set_error("null argument"), RTW_E_ARG;
    if (width == 0 || height == 0) return set_error("empty image"), RTW_E_EMPTY_IMAGE;
    RTW_GUARD_BEGIN
    const auto parts = format_ppm_parts(rgb, width, height);
    FILE *f = std::fopen(path, "wb");
    if (!f) return set_error(std::string("cannot create ") + path), RTW_E_ARG;
    bool short_write = false;
    for (const auto &p : parts) short_write |= std::fwrite(p.data(), 1, p.size(), f) != p.size();
    const int rc = std::fclose(f);
    if (short_write || rc != 0) return set_error("short write"), RTW_E_ARG;
    return RTW_OK;
    RTW_GUARD_END
}

}  // extern "C"
