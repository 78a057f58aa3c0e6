// Test infrastructure (tests/test_accel.py): the drain groups' trapped-path replay
// (rtw_render.hip unit_vec_round / trap_forward<true>) emulated on the host against the
// serial random_unit_vec loop (vec3.rs:219-232): lane j of a round takes its RNG state
// as the XOR of rtw::try_table's columns over the round's base state, draws one try,
// and the accepted tries in lane order must be the serial loop's unit vectors, with the
// serial loop's RNG state after each. Prints {"checked": N, "mismatches": M}.
#include <cstdint>
#include <cstdio>
#include <cmath>
#include <random>
#include <vector>
#include "rtw_numeric.h"
#include "rtw_host.h"
struct U128 { uint64_t lo, hi; };
static void xs_step(U128 &s) {
    uint64_t hi = s.hi ^ ((s.hi << 23) | (s.lo >> 41));
    uint64_t lo = s.lo ^ (s.lo << 23);
    lo ^= (lo >> 17) | (hi << 47);
    hi ^= hi >> 17;
    hi ^= (hi << 26) | (lo >> 38);
    lo ^= lo << 26;
    s.lo = lo; s.hi = hi;
}
static uint32_t xs_next_m(U128 &s) {
    xs_step(s);
    unsigned __int128 t = (uint64_t)(uint32_t)s.lo + (uint64_t)(uint32_t)(s.lo >> 32) + (uint64_t)(uint32_t)s.hi + (uint64_t)(uint32_t)(s.hi >> 32);
    uint64_t v = (uint64_t)t;
    v = (v & 0xffffffffu) + (v >> 32);
    v = (v & 0xffffffffu) + (v >> 32);
    uint32_t r = (uint32_t)v;
    return r == 0xffffffffu ? 0u : r;
}
static float coord32(uint32_t m) { return fmaf((float)m, 4.656612873077393e-10f, -1.f); }
static double coord64(uint32_t m) { return -1. + rtw_num::next01_of(m) * 2.; }
const float kRejBand = 7.62939453125e-06f;
static void ruv(U128 &rng, double &ux, double &uy, double &uz) {
    double x, y, z, l2;
    for (;;) {
        uint32_t m0 = xs_next_m(rng), m1 = xs_next_m(rng), m2 = xs_next_m(rng);
        float x32 = coord32(m0), y32 = coord32(m1), z32 = coord32(m2);
        float l32 = fmaf(x32, x32, fmaf(y32, y32, z32 * z32));
        if (l32 > 1.f + kRejBand) continue;
        x = coord64(m0), y = coord64(m1), z = coord64(m2);
        l2 = x * x + y * y + z * z;
        if (l32 < 1.f - kRejBand || l2 <= 1.) break;
    }
    double l = sqrt(l2);
    ux = x / l, uy = y / l, uz = z / l;
}
int main() {
    const auto &tt = rtw::try_table();
    std::mt19937_64 g(7);
    int bad = 0;
    for (int trial = 0; trial < 2000; ++trial) {
        U128 s{g(), g()};
        // serial: the first 70 unit vectors and the states after them
        U128 r = s;
        std::vector<double> sv; std::vector<U128> ss;
        for (int i = 0; i < 70; ++i) { double a, b, c; ruv(r, a, b, c); sv.push_back(a); sv.push_back(b); sv.push_back(c); ss.push_back(r); }
        // rounds
        U128 base = s; int k = 0;
        while (k < 70) {
            U128 st[64]; double ux[64], uy[64], uz[64]; bool ok[64];
            for (int j = 0; j < 64; ++j) {
                unsigned __int128 v = 0;
                for (int b = 0; b < 128; ++b) {
                    bool bit = b < 64 ? (base.lo >> b) & 1 : (base.hi >> (b - 64)) & 1;
                    if (bit) v ^= tt[(size_t)b * 64 + j];
                }
                U128 x{(uint64_t)v, (uint64_t)(v >> 64)};
                uint32_t m0 = xs_next_m(x), m1 = xs_next_m(x), m2 = xs_next_m(x);
                float x32 = coord32(m0), y32 = coord32(m1), z32 = coord32(m2);
                float l32 = fmaf(x32, x32, fmaf(y32, y32, z32 * z32));
                double X = coord64(m0), Y = coord64(m1), Z = coord64(m2), l2 = X * X + Y * Y + Z * Z;
                ok[j] = !(l32 > 1.f + kRejBand) && (l32 < 1.f - kRejBand || l2 <= 1.);
                double l = sqrt(l2); ux[j] = X / l, uy[j] = Y / l, uz[j] = Z / l; st[j] = x;
            }
            for (int j = 0; j < 64 && k < 70; ++j) if (ok[j]) {
                if (ux[j] != sv[3*k] || uy[j] != sv[3*k+1] || uz[j] != sv[3*k+2] || st[j].lo != ss[k].lo || st[j].hi != ss[k].hi) { ++bad; if (bad < 5) fprintf(stderr, "mismatch trial %d k %d\n", trial, k); }
                ++k;
            }
            base = st[63];
        }
    }
    printf("{\"checked\": %d, \"mismatches\": %d}\n", 2000 * 70, bad);
    return bad != 0;
}
