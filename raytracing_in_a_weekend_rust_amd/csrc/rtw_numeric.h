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
// Branch-free (a wave runs it for a few lanes at a time): k is clamped to >= 1 and
// the tie test is masked by b >= 22 instead of branched on.
RTW_NHD double next01_of(uint32_t m) {
    const double A = static_cast<double>(m) * 0x1p-32;
    const double B = static_cast<double>(m) * 0x1p-64;
    const double s = A + B;
    const uint32_t b = 32u - static_cast<uint32_t>(__builtin_clz(m | 1u));
    const uint32_t k = (b >= 22u ? b : 22u) - 21u;
    const uint32_t low = m & ((1u << k) - 1u), half = 1u << (k - 1u);
    const bool up = b >= 22u && low == half && !((m >> k) & 1u);
    uint64_t u;
    memcpy(&u, &s, 8);
    u += up ? 1u : 0u;
    double r;
    memcpy(&r, &u, 8);
    return r;
}

// ---- f64 divisions by one divisor sharing its reciprocal (device) ----------
// The compiler's IEEE f64 division x / d is: v_div_scale of d and of x, v_rcp_f64
// of the scaled d, two Newton steps r <- r + r (1 - d r), q0 = x r, the correction
// q = q0 + r (x - d q0) (v_div_fmas) and v_div_fixup. With |x| and |d| in
// [2^-256, 2^256] both scale steps are the identity (v_div_scale scales only for
// exponent gaps >= 768, denormal or near-overflow operands, or a numerator exponent
// <= 53) and so is the fixup (finite nonzero quotient, sign already right). Then
// divisions by the same d can share the reciprocal and its Newton steps: the same
// operations in the same order, the same bits. Outside the range: plain division.
// (Biased exponent e in [1023 - 256, 1023 + 256]: (e - 767) < 513 unsigned.)
RTW_NHD uint32_t div_exp_off(double v) {
    uint64_t u;
    memcpy(&u, &v, 8);
    return (static_cast<uint32_t>(u >> 52) & 0x7ffu) - 767u;
}
RTW_NHD bool div_range(double v) { return div_exp_off(v) < 513u; }
// d's reciprocal after the two Newton steps, or 0 when d is out of range
RTW_NHD double div_rcp(double d) {
#if defined(__HIP_DEVICE_COMPILE__)
    if (!div_range(d)) return 0.;
    const double r0 = __builtin_amdgcn_rcp(d);
    const double r1 = __builtin_fma(r0, __builtin_fma(-d, r0, 1.), r0);
    return __builtin_fma(r1, __builtin_fma(-d, r1, 1.), r1);
#else
    (void)d;
    return 0.;
#endif
}
// x / d given r = div_rcp(d) != 0 and div_range(x)
RTW_NHD double div_q(double x, double d, double r) {
    const double q0 = x * r;
    return __builtin_fma(__builtin_fma(-d, q0, x), r, q0);
}
// (x, y, z) / d, one range test for the three
RTW_NHD void div3(double &x, double &y, double &z, double d) {
#if defined(__HIP_DEVICE_COMPILE__)
    const double r = div_rcp(d);
    const uint32_t m = div_exp_off(x) > div_exp_off(y) ? div_exp_off(x) : div_exp_off(y);
    if (r != 0. && (m > div_exp_off(z) ? m : div_exp_off(z)) < 513u) {
        x = div_q(x, d, r), y = div_q(y, d, r), z = div_q(z, d, r);
        return;
    }
#endif
    x = x / d, y = y / d, z = z / d;
}

// Dielectric::scatter's "cannot refract" test, materials.rs:94-98:
//   ratio * sqrt(1 - cos^2) > thr   (thr = 1; the trapped-path hint uses 1 + 1e-9)
// decided without the square root when the squared comparison is clear by a
// relative margin of 2^-30 -- the operations here err by a few 2^-53 each -- and
// exactly as the reference (the square root, the product) otherwise, or when ratio
// is not a moderate positive number. x = 1 - cos*cos is the reference's own operand.
// Same decision for every input (tools/next01_check.cpp "tir" checks it).
RTW_NHD bool tir_exceeds(double ratio, double x, double thr) {
    if (ratio > 1e-100 && ratio < 1e100) {
        const double q = (ratio * ratio) * x, t2 = thr * thr;
        if (q > t2 * (1. + 0x1p-30)) return true;
        if (q < t2 * (1. - 0x1p-30)) return false;
    }
    return ratio * __builtin_sqrt(x) > thr;
}

}  // namespace rtw_num
