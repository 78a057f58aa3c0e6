// next01_check.cpp -- test infrastructure: exhaustive check of rtw_num::next01_of
// (csrc/rtw_numeric.h, the device's division-free XorShift::next_01 tail) against
// the IEEE division m / 4294967295.0 of random.rs:40-52, for every m in
// [0, 2^32-2]. Prints the mismatch count; exit 1 on any mismatch.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "rtw_numeric.h"

int main() {
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
