// rtw_group.hip -- device-resident multi-GPU renders of one image (rtw_group_*,
// include/rtw_capi.h), the node-level form of Camera::threaded_render
// (src/raytracing/camera.rs:223-352; its pool takes every core, camera.rs:253 --
// a group takes every listed GPU).
//
// Rows are dealt cyclically (image row r -> entry r % n: sky rows are cheap,
// ground rows are not). Each entry is an rtw_session on its own
// device and stream and renders its rows into a padded tile of ceil(H/n) rows.
// The tiles are then gathered on the root device (entry 0):
//   RTW_GATHER_RCCL -- entries are distinct GPUs: one ncclGather over xGMI
//                      (communicators from ncclCommInitAll, one process, one
//                      comm per device), root's own tile rendered in place;
//   RTW_GATHER_COPY -- some device repeats (or RTW_GROUP_COPY_GATHER): one
//                      device copy per tile on the root stream (peer access
//                      enabled between distinct devices);
// and un-permuted on the root device (rtw_unpermute_rows) into the caller's
// image buffer. Both gathers fill the same slot layout (tile i at slot i; the
// root renders straight into slot 0), so the un-permute is one code path.
// Pixels and RNG streams depend only on the global pixel index, so the image is
// bit-identical to a one-device render.
//
// Built only on the public session ABI. RCCL is opened with dlopen when a group
// first needs it (a process that already holds torch's librccl.so.1 reuses that
// copy), so single-GPU users of librtw.so never load it.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "rtw_capi.h"
#include "rtw_internal.h"

namespace {

// un-permute of the gathered tiles: image row r = entry (r % n), tile row (r / n).
// One workgroup row per image row; consecutive lanes copy consecutive elements
// (both sides contiguous: coalesced 8 B (f64) / 4 B (f32) per lane).
template <typename T>
__global__ __launch_bounds__(256) void rtw_unpermute_rows(const T *__restrict__ gathered, T *__restrict__ out,
                                                          uint32_t n, uint32_t tile_rows, uint32_t row_elems) {
    const uint32_t r = blockIdx.y;
    const T *src = gathered + (static_cast<size_t>(r % n) * tile_rows + r / n) * row_elems;
    T *dst = out + static_cast<size_t>(r) * row_elems;
    for (uint32_t e = blockIdx.x * 256 + threadIdx.x; e < row_elems; e += gridDim.x * 256) dst[e] = src[e];
}

struct Rccl {
    void *so = nullptr;
    ncclResult_t (*comm_init_all)(ncclComm_t *, int, const int *) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*gather)(const void *, void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
    const char *(*error_string)(ncclResult_t) = nullptr;
};

// RCCL, opened on first use. The soname list can be replaced under RTW_AB
// (RTW_RCCL_SONAME, ':'-separated) so tests can make RCCL unloadable.
Rccl &rccl_handle(std::string *why) {
    static Rccl r;
    static std::string err;
    static std::once_flag once;
    std::call_once(once, [] {
        std::vector<std::string> names = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
        if (const char *e = rtw::Knobs().get("RTW_RCCL_SONAME")) {
            names.clear();
            std::string v(e);
            for (size_t a = 0; a <= v.size();) {
                const size_t b = std::min(v.find(':', a), v.size());
                if (b > a) names.push_back(v.substr(a, b - a));
                a = b + 1;
            }
        }
        for (const auto &name : names) {
            if ((r.so = dlopen(name.c_str(), RTLD_NOW | RTLD_GLOBAL))) break;
        }
        if (!r.so) {
            std::string tried;
            for (const auto &name : names) tried += (tried.empty() ? "" : ", ") + name;
            err = "RCCL not loadable (dlopen of " + tried + " failed)";
            return;
        }
        r.comm_init_all = reinterpret_cast<decltype(r.comm_init_all)>(dlsym(r.so, "ncclCommInitAll"));
        r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(dlsym(r.so, "ncclCommDestroy"));
        r.gather = reinterpret_cast<decltype(r.gather)>(dlsym(r.so, "ncclGather"));
        r.group_start = reinterpret_cast<decltype(r.group_start)>(dlsym(r.so, "ncclGroupStart"));
        r.group_end = reinterpret_cast<decltype(r.group_end)>(dlsym(r.so, "ncclGroupEnd"));
        r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(r.so, "ncclGetErrorString"));
        if (!r.comm_init_all || !r.comm_destroy || !r.gather || !r.group_start || !r.group_end) {
            err = "RCCL loaded but lacks ncclCommInitAll/ncclGather/ncclGroupStart/End";
            r.so = nullptr;
        }
    });
    if (why) *why = err;
    return r;
}

bool rccl_ok(std::string *why) { return rccl_handle(why).so != nullptr; }

Rccl &rccl() {
    std::string why;
    Rccl &r = rccl_handle(&why);
    if (!r.so) throw rtw::Error(RTW_E_HIP, why);
    return r;
}

void nccl_check(ncclResult_t rc, const char *what) {
    if (rc != ncclSuccess) {
        const Rccl &r = rccl_handle(nullptr);
        throw rtw::Error(RTW_E_HIP, std::string(what) + ": " + (r.error_string ? r.error_string(rc) : ""));
    }
}

void hip_check(hipError_t e, const char *what) {
    if (e != hipSuccess) throw rtw::Error(RTW_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

void api_check(int rc) {
    if (rc != RTW_OK) throw rtw::Error(rc, rtw_last_error());
}

struct Entry {
    int device = 0;
    rtw_session *sess = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;  // around the entry's render, on its stream
    void *tile = nullptr;                     // padded row tile (entries > 0)
    size_t tile_cap = 0;
    ncclComm_t comm = nullptr;
    rtw_stats last{};
};

}  // namespace

struct rtw_group {
    std::vector<Entry> e;
    uint32_t gather = RTW_GATHER_NONE;  // for n > 1 entries
    bool force_rccl = false;            // RTW_GROUP_RCCL_ALWAYS: RCCL even for one entry (strict)
    bool single_rccl = false;           // a one-entry group gathers through RCCL (ALWAYS, or TRY that worked)
    std::string note;                   // why the group fell back from RCCL to device copies ("" = it did not)
    void *gathered = nullptr;           // root: n x tile, tile i at slot i
    size_t gathered_cap = 0;
    hipEvent_t g0 = nullptr, g1 = nullptr;  // root stream: root tile ready -> image complete
    hipEvent_t caller = nullptr;            // root device's null stream at the call (ordering)
    rtw_group_info info{};
    std::mutex mu;
};

namespace {

void grow(void *&p, size_t &cap, size_t need, int device) {
    if (need <= cap) return;
    hip_check(hipSetDevice(device), "hipSetDevice");
    if (p) (void)hipFree(p);
    p = nullptr, cap = 0;
    hip_check(hipMalloc(&p, need), "hipMalloc (group tile)");
    cap = need;
}

void destroy(rtw_group *g) {
    for (auto &x : g->e) {
        (void)hipSetDevice(x.device);
        if (x.stream) (void)hipStreamSynchronize(x.stream);
        if (x.comm) (void)rccl_handle(nullptr).comm_destroy(x.comm);
        if (x.tile) (void)hipFree(x.tile);
        if (x.ev0) (void)hipEventDestroy(x.ev0);
        if (x.ev1) (void)hipEventDestroy(x.ev1);
        if (x.stream) (void)hipStreamDestroy(x.stream);
        rtw_session_destroy(x.sess);
    }
    if (!g->e.empty()) (void)hipSetDevice(g->e[0].device);
    if (g->gathered) (void)hipFree(g->gathered);
    if (g->g0) (void)hipEventDestroy(g->g0);
    if (g->g1) (void)hipEventDestroy(g->g1);
    if (g->caller) (void)hipEventDestroy(g->caller);
    delete g;
}

void create(const int *devices, uint32_t n_devices, uint32_t flags, rtw_group **out) {
    int visible = 0;
    if (hipGetDeviceCount(&visible) != hipSuccess || visible == 0) throw rtw::Error(RTW_E_NO_DEVICE, "no HIP device");
    std::vector<int> devs;
    if (n_devices == 0)
        for (int d = 0; d < visible; ++d) devs.push_back(d);
    else
        devs.assign(devices, devices + n_devices);
    for (int d : devs)
        if (d < 0 || d >= visible) throw rtw::Error(RTW_E_NO_DEVICE, "device index out of range");
    auto *g = new rtw_group();
    try {
        g->e.resize(devs.size());
        for (size_t i = 0; i < devs.size(); ++i) {
            Entry &x = g->e[i];
            x.device = devs[i];
            api_check(rtw_session_create(x.device, &x.sess));
            hip_check(hipSetDevice(x.device), "hipSetDevice");
            hip_check(hipStreamCreateWithFlags(&x.stream, hipStreamNonBlocking), "hipStreamCreate");
            hip_check(hipEventCreate(&x.ev0), "hipEventCreate");
            hip_check(hipEventCreate(&x.ev1), "hipEventCreate");
        }
        hip_check(hipSetDevice(devs[0]), "hipSetDevice");
        hip_check(hipEventCreate(&g->g0), "hipEventCreate");
        hip_check(hipEventCreate(&g->g1), "hipEventCreate");
        hip_check(hipEventCreateWithFlags(&g->caller, hipEventDisableTiming), "hipEventCreate");
        std::vector<int> sorted = devs;
        std::sort(sorted.begin(), sorted.end());
        const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
        g->force_rccl = (flags & RTW_GROUP_RCCL_ALWAYS) != 0;
        if (g->force_rccl && (!distinct || (flags & RTW_GROUP_COPY_GATHER)))
            throw rtw::Error(RTW_E_ARG, "RTW_GROUP_RCCL_ALWAYS needs distinct devices and no RTW_GROUP_COPY_GATHER");
        const bool try_single = (flags & RTW_GROUP_RCCL_TRY) != 0 && !(flags & RTW_GROUP_COPY_GATHER);
        if (devs.size() > 1 || g->force_rccl || try_single) {
            g->gather = (distinct && !(flags & RTW_GROUP_COPY_GATHER)) ? RTW_GATHER_RCCL : RTW_GATHER_COPY;
            if (g->gather == RTW_GATHER_RCCL) {
                // RCCL when it loads and its communicators come up; otherwise the
                // device-copy gather (same slots, same image), with the reason kept in
                // rtw_group_note -- unless the caller asked for RCCL strictly
                std::string why;
                if (rccl_ok(&why)) {
                    std::vector<ncclComm_t> comms(devs.size());
                    const ncclResult_t rc =
                        rccl().comm_init_all(comms.data(), static_cast<int>(devs.size()), devs.data());
                    if (rc == ncclSuccess) {
                        for (size_t i = 0; i < devs.size(); ++i) g->e[i].comm = comms[i];
                    } else {
                        const char *m = rccl().error_string ? rccl().error_string(rc) : "";
                        why = std::string("ncclCommInitAll failed: ") + m;
                        g->info.fallback = RTW_FALLBACK_COMM_INIT;
                    }
                } else {
                    g->info.fallback = RTW_FALLBACK_NO_RCCL;
                }
                if (g->info.fallback != RTW_FALLBACK_NONE) {
                    if (g->force_rccl) throw rtw::Error(RTW_E_HIP, why);
                    g->note = why;
                    g->gather = RTW_GATHER_COPY;
                }
            }
            if (g->gather == RTW_GATHER_COPY) {
                // copies from other devices' tiles: peer access where the pair allows it
                hip_check(hipSetDevice(devs[0]), "hipSetDevice");
                for (size_t i = 1; i < devs.size(); ++i) {
                    int ok = 0;
                    if (devs[i] != devs[0] && hipDeviceCanAccessPeer(&ok, devs[0], devs[i]) == hipSuccess && ok) {
                        const hipError_t pe = hipDeviceEnablePeerAccess(devs[i], 0);
                        if (pe != hipSuccess && pe != hipErrorPeerAccessAlreadyEnabled)
                            hip_check(pe, "hipDeviceEnablePeerAccess");
                        (void)hipGetLastError();
                    }
                }
            }
            g->single_rccl = devs.size() == 1 && g->gather == RTW_GATHER_RCCL;
            if (devs.size() == 1 && g->gather == RTW_GATHER_COPY) g->gather = RTW_GATHER_NONE;  // TRY fell back
        }
        g->info.n_entries = static_cast<uint32_t>(devs.size());
        g->info.gather = g->gather;
    } catch (...) {
        destroy(g);
        throw;
    }
    *out = g;
}

template <typename T>
void render(rtw_group *g, const rtw_camera *cam, uint32_t samples_sqrt, rtw_u128 seed, bool fast, T *out,
            hipStream_t caller) {
    const auto t0 = std::chrono::steady_clock::now();
    if (!cam || !out) throw rtw::Error(RTW_E_ARG, "null argument");
    const uint32_t H = cam->img_height, W = cam->img_width;
    if (H == 0 || W == 0) throw rtw::Error(RTW_E_EMPTY_IMAGE, "image height and width must be > 0");
    // entries beyond the row count get no rows (and take no part in this render)
    const uint32_t n = static_cast<uint32_t>(std::min<size_t>(g->e.size(), H));
    const uint32_t tile_rows = (H + n - 1) / n;
    const size_t row_elems = static_cast<size_t>(W) * 3, row_bytes = row_elems * sizeof(T);
    const size_t tile_bytes = tile_rows * row_bytes;
    const bool all_entries = n == g->e.size();
    const bool use_rccl = all_entries && g->gather == RTW_GATHER_RCCL && (n > 1 || g->single_rccl);
    const uint32_t gather = use_rccl ? RTW_GATHER_RCCL : n == 1 ? RTW_GATHER_NONE : RTW_GATHER_COPY;
    Entry &root = g->e[0];
    if (gather != RTW_GATHER_NONE) grow(g->gathered, g->gathered_cap, n * tile_bytes, root.device);
    // The root stream is non-blocking, so order it after the work the caller already
    // queued on its stream on the root device (`caller`: NULL = the null stream, torch's
    // default stream; rtw_group_render_on passes a torch.cuda.stream's or a per-thread
    // stream), which may still read or write `out`: the root stream's first write to
    // `out` (the one-entry render, or the un-permute) waits for it.
    hip_check(hipSetDevice(root.device), "hipSetDevice");
    hip_check(hipEventRecord(g->caller, caller), "hipEventRecord (caller stream)");
    hip_check(hipStreamWaitEvent(root.stream, g->caller, 0), "hipStreamWaitEvent");

    // 1. every entry's rows, enqueued on its own stream (asynchronous)
    for (uint32_t i = 0; i < n; ++i) {
        Entry &x = g->e[i];
        const rtw_shard sh{i, n, (H - i + n - 1) / n, 0};
        void *dst;
        if (gather == RTW_GATHER_NONE) dst = out;          // one entry: the whole image in place
        else if (i == 0) dst = g->gathered;                // root's slot of the gather buffer
        else grow(x.tile, x.tile_cap, tile_bytes, x.device), dst = x.tile;
        hip_check(hipSetDevice(x.device), "hipSetDevice");
        hip_check(hipEventRecord(x.ev0, x.stream), "hipEventRecord");
        if (fast)
            api_check(rtw_session_render_fast(x.sess, cam, samples_sqrt, seed, &sh, static_cast<float *>(dst), x.stream));
        else
            api_check(rtw_session_render(x.sess, cam, samples_sqrt, seed, &sh, static_cast<double *>(dst), x.stream));
        hip_check(hipEventRecord(x.ev1, x.stream), "hipEventRecord");
    }
    // 2. the gather of the tiles into the root's buffer (tile i at slot i), then the
    //    un-permute into the image
    hip_check(hipSetDevice(root.device), "hipSetDevice");
    hip_check(hipEventRecord(g->g0, root.stream), "hipEventRecord");
    if (gather == RTW_GATHER_RCCL) {
        // root's send buffer is its own slot: RCCL's in-place gather
        const ncclDataType_t dt = sizeof(T) == 8 ? ncclFloat64 : ncclFloat32;
        const size_t count = tile_rows * row_elems;
        nccl_check(rccl().group_start(), "ncclGroupStart");
        for (uint32_t i = 0; i < n; ++i) {
            Entry &x = g->e[i];
            const ncclResult_t rc = rccl().gather(i == 0 ? g->gathered : x.tile, i == 0 ? g->gathered : nullptr,
                                                  count, dt, 0, x.comm, x.stream);
            if (rc != ncclSuccess) {
                (void)rccl().group_end();
                nccl_check(rc, "ncclGather");
            }
        }
        nccl_check(rccl().group_end(), "ncclGroupEnd");
    } else if (gather == RTW_GATHER_COPY) {
        for (uint32_t i = 1; i < n; ++i) {
            Entry &x = g->e[i];
            hip_check(hipStreamWaitEvent(root.stream, x.ev1, 0), "hipStreamWaitEvent");
            const size_t rows = (H - i + n - 1) / n;
            hip_check(hipMemcpyAsync(static_cast<char *>(g->gathered) + i * tile_bytes, x.tile, rows * row_bytes,
                                     hipMemcpyDefault, root.stream),
                      "hipMemcpyAsync (gather)");
        }
    }
    if (gather != RTW_GATHER_NONE) {
        hipLaunchKernelGGL(rtw_unpermute_rows<T>, dim3(static_cast<uint32_t>(std::min<size_t>((row_elems + 255) / 256, 64)), H),
                           dim3(256), 0, root.stream, static_cast<const T *>(g->gathered), out, n, tile_rows,
                           static_cast<uint32_t>(row_elems));
        hip_check(hipGetLastError(), "rtw_unpermute_rows");
    }
    hip_check(hipEventRecord(g->g1, root.stream), "hipEventRecord");
    // 3. wait, then every entry's counters (each session checks its completeness latch)
    float render_max = 0.f;
    for (uint32_t i = 0; i < n; ++i) {
        Entry &x = g->e[i];
        hip_check(hipSetDevice(x.device), "hipSetDevice");
        hip_check(hipStreamSynchronize(x.stream), "hipStreamSynchronize");
        api_check(rtw_session_stats(x.sess, &x.last));
        float ms = 0.f;
        hip_check(hipEventElapsedTime(&ms, x.ev0, x.ev1), "hipEventElapsedTime");
        render_max = std::max(render_max, ms);
    }
    float gms = 0.f;
    hip_check(hipEventElapsedTime(&gms, g->g0, g->g1), "hipEventElapsedTime");
    g->info.n_entries = n;
    g->info.gather = gather;
    g->info.render_ms_max = render_max;
    g->info.root_gather_ms = gms;
    g->info.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    g->info.fast = fast ? 1u : 0u;
}

}  // namespace

// The caller's current device is restored on every exit of an rtw_group_* call
// (the calls switch devices per entry; a torch caller's allocations must not move).
struct DeviceGuard {
    int dev = -1;
    DeviceGuard() {
        if (hipGetDevice(&dev) != hipSuccess) dev = -1;
    }
    ~DeviceGuard() {
        if (dev >= 0) (void)hipSetDevice(dev);
    }
};

#define RTW_GROUP_GUARD(body)                 \
    DeviceGuard device_guard_;                \
    try {                                     \
        body;                                 \
        return RTW_OK;                        \
    } catch (const rtw::Error &e) {           \
        rtw::set_error(e.what());             \
        return e.code;                        \
    } catch (const std::exception &e) {       \
        rtw::set_error(e.what());             \
        return RTW_E_ARG;                     \
    }

extern "C" {

int rtw_group_create(const int *devices, uint32_t n_devices, uint32_t flags, rtw_group **out) {
    if (!out || (n_devices && !devices)) return rtw::set_error("null argument"), RTW_E_ARG;
    RTW_GROUP_GUARD(create(devices, n_devices, flags, out))
}

int rtw_group_destroy(rtw_group *g) {
    DeviceGuard guard;
    if (g) destroy(g);
    return RTW_OK;
}

const char *rtw_group_note(rtw_group *g) { return g ? g->note.c_str() : ""; }

int rtw_rccl_available(char *why, size_t cap) {
    std::string w;
    const bool ok = rccl_ok(&w);
    if (why && cap) {
        const size_t k = std::min(cap - 1, w.size());
        std::memcpy(why, w.data(), k);
        why[k] = '\0';
    }
    return ok ? 1 : 0;
}

int rtw_group_set_scene(rtw_group *g, const rtw_sphere *spheres, uint32_t n_spheres, const rtw_material *mats,
                        uint32_t n_mats) {
    if (!g) return rtw::set_error("null group"), RTW_E_ARG;
    std::lock_guard<std::mutex> lock(g->mu);
    RTW_GROUP_GUARD(for (auto &x : g->e) api_check(rtw_session_set_scene(x.sess, spheres, n_spheres, mats, n_mats)))
}

int rtw_group_render_on(rtw_group *g, const rtw_camera *cam, uint32_t samples_sqrt, rtw_u128 seed,
                        double *out_rgb_device, void *caller_stream) {
    if (!g) return rtw::set_error("null group"), RTW_E_ARG;
    std::lock_guard<std::mutex> lock(g->mu);
    RTW_GROUP_GUARD(render<double>(g, cam, samples_sqrt, seed, false, out_rgb_device,
                                   static_cast<hipStream_t>(caller_stream)))
}

int rtw_group_render_fast_on(rtw_group *g, const rtw_camera *cam, uint32_t samples_sqrt, rtw_u128 seed,
                             float *out_rgb_device, void *caller_stream) {
    if (!g) return rtw::set_error("null group"), RTW_E_ARG;
    std::lock_guard<std::mutex> lock(g->mu);
    RTW_GROUP_GUARD(render<float>(g, cam, samples_sqrt, seed, true, out_rgb_device,
                                  static_cast<hipStream_t>(caller_stream)))
}

int rtw_group_render(rtw_group *g, const rtw_camera *cam, uint32_t samples_sqrt, rtw_u128 seed,
                     double *out_rgb_device) {
    return rtw_group_render_on(g, cam, samples_sqrt, seed, out_rgb_device, nullptr);
}

int rtw_group_render_fast(rtw_group *g, const rtw_camera *cam, uint32_t samples_sqrt, rtw_u128 seed,
                          float *out_rgb_device) {
    return rtw_group_render_fast_on(g, cam, samples_sqrt, seed, out_rgb_device, nullptr);
}

int rtw_group_stats(rtw_group *g, rtw_stats *total, rtw_stats *per_entry, uint32_t cap, rtw_group_info *info) {
    if (!g) return rtw::set_error("null group"), RTW_E_ARG;
    std::lock_guard<std::mutex> lock(g->mu);
    const uint32_t n = g->info.n_entries;
    if (per_entry && cap < n) return rtw::set_error("per_entry buffer too small"), RTW_E_CAPACITY;
    if (total) {
        rtw_stats a{};
        for (uint32_t i = 0; i < n; ++i) rtw::add_stats(a, g->e[i].last, i == 0);
        *total = a;
    }
    if (per_entry)
        for (uint32_t i = 0; i < n; ++i) per_entry[i] = g->e[i].last;
    if (info) *info = g->info;
    return RTW_OK;
}

}  // extern "C"
