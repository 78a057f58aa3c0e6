// next01_check.cpp -- test infrastructure: exhaustive check of rtw_num::next01_of
// (csrc/rtw_numeric.h, the device's division-free XorShift::next_01 tail) against
// the IEEE division m / 4294967295.0 of random.rs:40-52, for every m in
// [0, 2^32-2]. Prints the mismatch count; exit 1 on any mismatch.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "rtw_numeric.h"

// "tir" mode: rtw_num::tir_exceeds against the reference's sqrt-and-multiply test
// on random (ratio, cos) pairs, cos near the critical angle, and edge values.
static int tir_check(uint64_t n) {
    uint64_t x = 0x9E3779B97F4A7C15ull, bad = 0, checked = 0;
    auto next = [&] {
        x ^= x << 13, x ^= x >> 7, x ^= x << 17;
        return x;
    };
    auto u01 = [&] { return static_cast<double>(next() >> 11) * 0x1p-53; };
    const double ratios[] = {1. / 1.5, 1.5, 1. / 1.33, 1.33, 2.4, 1. / 2.4, 1.0, 0.5, 3.0, 1e-3, 1e3,
                             0., -1.5, 1e120, 1e-120, __builtin_inf(), __builtin_nan("")};
    const double edge[] = {1.0, -1.0, 0.0, -0.0, 1.0 + 0x1p-52, -1.0 - 0x1p-52, __builtin_nan(""),
                           __builtin_inf(), -__builtin_inf(), 0x1p-1074, 1e-300};
    for (double thr : {1.0, 1.0 + 1e-9}) {
        auto one = [&](double ratio, double c) {
            const double xx = 1.0 - c * c;
            const bool ref = ratio * __builtin_sqrt(xx) > thr;
            bad += rtw_num::tir_exceeds(ratio, xx, thr) != ref;
            ++checked;
        };
        for (double r : ratios)
            for (double c : edge) one(r, c);
        for (uint64_t i = 0; i < n; ++i) {
            double r = ratios[next() % 11];
            if (next() & 1) r *= 1. + (u01() - 0.5) * 1e-3;
            double c;
            const uint64_t mode = next() % 3;
            if (mode == 0) {
                c = u01() * 2. - 1.;
            } else {  // around the critical cosine sqrt(1 - (thr/r)^2), ulps to 1e-6 away
                const double s = thr / r;
                const double cc = s < 1. ? __builtin_sqrt(1. - s * s) : u01();
                const double d = mode == 1 ? (u01() - 0.5) * 1e-6 : static_cast<double>(static_cast<int64_t>(next() % 64) - 32) * 0x1p-52;
                c = (next() & 1 ? cc : -cc) + d;
            }
            one(r, c);
        }
    }
    printf("{\"tir_checked\": %llu, \"mismatches\": %llu}\n", (unsigned long long)checked, (unsigned long long)bad);
    return bad ? 1 : 0;
}

int main(int argc, char **argv) {
    if (argc > 2 && std::strcmp(argv[1], "tir") == 0) return tir_check(std::strtoull(argv[2], nullptr, 10));
    const unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<uint64_t> bad(nt, 0);
    std::vector<std::thread> th;
    const uint64_t total = 4294967295ull;
    for (unsigned t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
            const uint64_t b = total * t / nt, e = total * (t + 1) / nt;
            uint64_t nb = 0;
            for (uint64_t m = b; m < e; ++m) {
                const double ref = static_cast<double>(static_cast<uint32_t>(m)) / 4294967295.0;
                const double f = rtw_num::next01_of(static_cast<uint32_t>(m));
                nb += std::memcmp(&ref, &f, 8) != 0;
            }
            bad[t] = nb;
        });
    for (auto &x : th) x.join();
    uint64_t nb = 0;
    for (uint64_t v : bad) nb += v;
    printf("{\"checked\": %llu, \"mismatches\": %llu}\n", (unsigned long long)total, (unsigned long long)nb);
    return nb ? 1 : 0;
}
