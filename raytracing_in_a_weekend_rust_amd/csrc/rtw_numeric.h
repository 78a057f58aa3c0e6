// rtw_numeric.h -- exact replacements for expensive f64 operations on the hot
// path, shared by the device kernel and the host self-check
// (tools/next01_check.cpp verifies them exhaustively against IEEE arithmetic).
#pragma once

#include <cstdint>
#include <cstring>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define RTW_NHD __host__ __device__ __forceinline__
#else
#define RTW_NHD inline
#endif

namespace rtw_num {

// XorShift::next_01's last step, random.rs:40-52: m / 4294967295.0 with m the
// u128 state folded mod 2^32-1 (m <= 2^32-2), correctly rounded -- without the
// ~12-instruction IEEE f64 division sequence.
// m / (2^32-1) = A + B + T with A = m 2^-32, B = m 2^-64 (both exact) and
// 0 <= T < 2^-64 A. A and B have disjoint bit ranges, so A + B is exact when m
// has <= 21 significant bits, and otherwise RN(A + B) drops exactly the low
// k = bitlen(m) - 21 bits of m; T > 0 only matters when those bits are a tie
// (10...0), where the true value lies above the midpoint and the result must
// round up -- RN-even rounds down there iff bit k of m is 0.
RTW_NHD double next01_of(uint32_t m) {
    const double A = static_cast<double>(m) * 0x1p-32;
    const double B = static_cast<double>(m) * 0x1p-64;
    double s = A + B;
    const uint32_t b = 32u - static_cast<uint32_t>(__builtin_clz(m | 1u));
    if (b >= 22u) {
        const uint32_t k = b - 21u;
        const uint32_t low = m & ((1u << k) - 1u), half = 1u << (k - 1u);
        if (low == half && !((m >> k) & 1u)) {
            uint64_t u;
            memcpy(&u, &s, 8);
            ++u;
            memcpy(&s, &u, 8);
        }
    }
    return s;
}

}  // namespace rtw_num
