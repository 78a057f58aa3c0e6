// rtw_cli -- host driver mirroring the reference's main.rs (flags main.rs:32-87,
// defaults main.rs:20-29) and raytracing::complex (raytracing/mod.rs:54-126):
// builds the scene, runs Camera::threaded_render on the GPU, writes img.ppm.
//
// Extra flags (the reference hard-codes or time-seeds these): --depth (MAX_DEPTH,
// mod.rs:43), --seed (both XorShift::default seeds, mod.rs:67 / camera.rs:255),
// --scene (the other builders of mod.rs), --out, --mode parity|fast (fast: the
// f32 statistical mode), --gpus N|LIST (N: the first N devices; LIST: comma-
// separated device indices, repeats allowed; default: every visible device -- the
// reference's pool takes every core, camera.rs:253). --preview is accepted and
// ignored: the winit preview window (application/mod.rs) is out of scope.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "rtw_host.h"

namespace {

struct Config {  // main.rs:13-29
    uint32_t height = 1080, width = 1920, sample_sqrt = 10, depth = 0;
    bool preview = false;
    std::string scene = "complex", out = "img.ppm";
    unsigned __int128 seed = 0;
    bool seed_set = false;
    bool fast = false;
    std::vector<int> devices;  // empty: every visible device
};

bool parse_u32(const char *s, uint32_t &v);

// --gpus N (the first N devices) or a comma-separated device list ("0,0,1")
bool parse_gpus(const char *s, std::vector<int> &out) {
    if (!s || !*s) return false;
    out.clear();
    const bool list = std::strchr(s, ',') != nullptr;
    std::string cur;
    for (const char *p = s;; ++p) {
        if (*p == ',' || !*p) {
            uint32_t v = 0;
            if (!parse_u32(cur.c_str(), v) || v > 65535) return false;
            out.push_back(static_cast<int>(v));
            cur.clear();
            if (!*p) break;
        } else {
            cur.push_back(*p);
        }
    }
    if (!list) {  // a count
        const int n = out[0];
        if (n == 0) return false;
        out.clear();
        for (int d = 0; d < n; ++d) out.push_back(d);
    }
    return true;
}

// Rust's str::parse::<usize>() (main.rs:37-39): an optional '+', then decimal
// digits only (no whitespace, no sign '-', no base prefix).
bool parse_dec(const char *s, unsigned __int128 max, unsigned __int128 &v) {
    if (!s) return false;
    if (*s == '+') ++s;
    if (!*s) return false;
    unsigned __int128 x = 0;
    for (; *s; ++s) {
        if (*s < '0' || *s > '9') return false;
        const unsigned d = static_cast<unsigned>(*s - '0');
        if (x > (max - d) / 10) return false;
        x = x * 10 + d;
    }
    v = x;
    return true;
}
bool parse_u32(const char *s, uint32_t &v) {
    unsigned __int128 x = 0;
    if (!parse_dec(s, 0xffffffffu, x)) return false;
    v = static_cast<uint32_t>(x);
    return true;
}

Config parse_args(int argc, char **argv) {
    Config c;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        const char *next = i + 1 < argc ? argv[i + 1] : nullptr;
        auto need = [&](uint32_t &dst, const char *usage) {
            if (!parse_u32(next, dst)) {
                std::fprintf(stderr, "Usage: %s <number>\n", usage);
                std::exit(1);
            }
        };
        if (a == "--height" || a == "-h") need(c.height, "--height");
        else if (a == "--width" || a == "-w") need(c.width, "--width");
        else if (a == "--samplesqrt" || a == "-s") need(c.sample_sqrt, "--samplesqrt");
        else if (a == "--depth" || a == "-d") need(c.depth, "--depth");
        else if (a == "--preview" || a == "-p") c.preview = true;
        else if (a == "--seed") {  // decimal, up to 2^128 - 1 (XorShift state is a u128)
            if (!parse_dec(next, ~static_cast<unsigned __int128>(0), c.seed)) {
                std::fprintf(stderr, "Usage: --seed <decimal number>\n");
                std::exit(1);
            }
            c.seed_set = true;
        }
        else if (a == "--scene" && next) c.scene = next;
        else if (a == "--out" && next) c.out = next;
        else if (a == "--mode" && next) {
            if (std::strcmp(next, "fast") && std::strcmp(next, "parity")) {
                std::fprintf(stderr, "Usage: --mode parity|fast\n");
                std::exit(1);
            }
            c.fast = !std::strcmp(next, "fast");
        }
        else if (a == "--gpus") {
            if (!parse_gpus(next, c.devices)) {
                std::fprintf(stderr, "Usage: --gpus <count> | <device,device,...>\n");
                std::exit(1);
            }
        }
        else if (a == "--help") {
            std::printf("Use the application like this:\n");
            std::printf("\t-h --height\t:\tSet the height of the image\n");
            std::printf("\t--width -w\t:\tSet the width of the image\n");
            std::printf("\t--samplesqrt -s\t:\tSet the sqrt of the samples used for the image\n");
            std::printf("\t--preview -p\t:\tSet whether a preview window is displayed (ignored)\n");
            std::printf("\t--depth -d\t:\tMax bounce depth (reference: 10)\n");
            std::printf("\t--seed N\t:\tXorShift seed (decimal) for scene and render (reference: wall-clock ms)\n");
            std::printf("\t--scene NAME\t:\tcomplex | simple | threads | super_simple | three_lambertian\n");
            std::printf("\t--out PATH\t:\tOutput PPM (reference: img.ppm)\n");
            std::printf("\t--mode M\t:\tparity (f64, bit-exact; default) | fast (f32, statistical)\n");
            std::printf("\t--gpus N|LIST\t:\tthe first N GPUs, or device indices 0,1,.. (default: every GPU)\n");
            std::exit(0);
        }
    }
    if (!c.seed_set)  // XorShift::default(): milliseconds since the Unix epoch
        c.seed = static_cast<unsigned long long>(
            std::chrono::duration_cast<std::chrono::milliseconds>(
                std::chrono::system_clock::now().time_since_epoch())
                .count());
    return c;
}

std::string dec(unsigned __int128 v) {
    std::string r;
    do {
        r.insert(r.begin(), static_cast<char>('0' + static_cast<int>(v % 10)));
        v /= 10;
    } while (v);
    return r;
}

}  // namespace

int main(int argc, char **argv) {
    const Config cfg = parse_args(argc, argv);
    if (cfg.preview) std::fprintf(stderr, "note: --preview is not supported; rendering headless\n");
    try {
        const rtw_u128 seed{static_cast<uint64_t>(cfg.seed), static_cast<uint64_t>(cfg.seed >> 64)};
        rtw::BuiltScene b = rtw::build_scene(cfg.scene, seed, cfg.height, cfg.width, cfg.depth);
        std::printf(
            "\n            Multithreaded rendering\n            Making an image of format:\n"
            "                %u by %u\n                %u samples\n                %u max depth\n\n",
            b.cam.width(), b.cam.height(), cfg.sample_sqrt * cfg.sample_sqrt, b.cam.d.max_depth);
        rtw_stats st{};
        const auto t0 = std::chrono::steady_clock::now();
        if (cfg.fast) {
            rtw::FlatScene flat;
            b.world->flatten(flat);
            std::vector<float> f32(static_cast<size_t>(b.cam.width()) * b.cam.height() * 3);
            int rc = rtw_threaded_render_multi_fast(
                &b.cam.d, flat.spheres.data(), static_cast<uint32_t>(flat.spheres.size()), flat.materials.data(),
                static_cast<uint32_t>(flat.materials.size()), cfg.sample_sqrt, seed,
                cfg.devices.empty() ? nullptr : cfg.devices.data(), static_cast<uint32_t>(cfg.devices.size()),
                f32.data(), &st);
            if (rc != RTW_OK) throw rtw::Error(rc, rtw_last_error());
            const std::vector<double> fb(f32.begin(), f32.end());
            rc = rtw_write_ppm(cfg.out.c_str(), fb.data(), b.cam.width(), b.cam.height());
            if (rc != RTW_OK) throw rtw::Error(rc, rtw_last_error());
        } else {
            rtw::Camera::threaded_render(b.cam, *b.world, cfg.sample_sqrt, seed, cfg.out.c_str(), &st, cfg.devices);
        }
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        std::printf("Finished succesfully: %s (%.3f s wall, kernel %.3f ms, %.1f Msamples/s, seed %s)\n",
                    cfg.out.c_str(), s, st.kernel_ms, st.samples / st.kernel_ms / 1e3, dec(cfg.seed).c_str());
    } catch (const rtw::Error &e) {
        // main.rs:106-110: the render thread's error is printed, and main still
        // returns Ok(()) -- exit status 0, as the reference
        std::fprintf(stderr, "\nRender thread errored with %s\n", e.what());
    }
    return 0;
}
