// rtw_internal.h -- shared between the host mirror (rtw_host.cpp) and the device
// half of the C ABI (rtw_render.hip, rtw_group.hip). Not part of the public ABI.
#pragma once

#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "rtw_capi.h"

namespace rtw {
void set_error(const std::string &m);
const char *last_error();

// Counters of several shards of one image: sums; the times are the slowest shard's.
inline void add_stats(rtw_stats &a, const rtw_stats &b, bool first) {
    if (first) {
        a = b;
        return;
    }
    a.pixels += b.pixels, a.samples += b.samples, a.segments += b.segments;
    a.sphere_tests += b.sphere_tests, a.wave_iterations += b.wave_iterations;
    a.exact_tests += b.exact_tests, a.exact_wave_iterations += b.exact_wave_iterations;
    a.kernel_ms = std::max(a.kernel_ms, b.kernel_ms);
    a.main_kernel_ms = std::max(a.main_kernel_ms, b.main_kernel_ms);
    a.node_visits += b.node_visits, a.brute_segments += b.brute_segments;
    a.parked_pixels += b.parked_pixels, a.inside_segments += b.inside_segments;
    a.trap_segments += b.trap_segments, a.guard_exits += b.guard_exits;
    a.leftover_pixels += b.leftover_pixels;
}

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

// Scheduling, strategy and diagnostic switches (RTW_ACCEL, RTW_HEAVY, RTW_DIAG, ...)
// are read from the environment only when RTW_AB is set to a non-zero value: A/B
// runs, the developer tools and the strategy tests. A production render reads
// RTW_AB once and nothing else, so its schedule cannot change with the caller's
// environment (the reference's Camera::threaded_render takes no tuning either,
// camera.rs:223-227). Results are identical either way; only the schedule moves.
struct Knobs {
    bool on;
    Knobs() {
        const char *e = std::getenv("RTW_AB");
        on = e && *e && !(e[0] == '0' && e[1] == '\0');
    }
    const char *get(const char *name) const { return on ? std::getenv(name) : nullptr; }
};
}  // namespace rtw
