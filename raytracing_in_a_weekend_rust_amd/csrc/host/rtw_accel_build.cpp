// rtw_accel_build.cpp -- host builder of the exact-result sphere BVH
// (csrc/rtw_accel.h). Replaces nothing in the reference: Scene::hit
// (hittable.rs:131-143) scans every object; this structure only lets the kernel
// skip spheres it can prove irrelevant, and the kernel still returns the scan's
// (t, first index) result.
//
// 4-wide nodes built top-down: a set of more than 4 spheres is cut into 4 parts
// by two levels of object-median splits on the longest centroid axis; each node
// holds the padded boxes of its (up to) 4 children -- inner nodes or single
// spheres -- and per ray-octant near-to-far child orders. Boxes are inflated by kPadK * M_b and rounded outward
// to f32 (rtw_accel.h "Padding").
#include <algorithm>
#include <cmath>
#include <cstring>
#include <numeric>
#include <cstdlib>
#include <vector>

#include "rtw_accel.h"
#include "rtw_internal.h"

namespace rtw_accel {
namespace {

float down_f32(double x) {
    float f = static_cast<float>(x);
    if (static_cast<double>(f) > x) f = std::nextafter(f, -INFINITY);
    return f;
}
float up_f32(double x) {
    float f = static_cast<float>(x);
    if (static_cast<double>(f) < x) f = std::nextafter(f, INFINITY);
    return f;
}

struct Builder {
    const double *c, *r;
    const float *r2p;
    std::vector<uint32_t> idx;
    Bvh *out;
    uint32_t n_leaf = 0;
    bool median = false;

    void bounds(uint32_t b, uint32_t e, double lo[3], double hi[3]) const {
        for (int k = 0; k < 3; ++k) lo[k] = INFINITY, hi[k] = -INFINITY;
        for (uint32_t j = b; j < e; ++j) {
            const uint32_t i = idx[j];
            const double rad = std::fabs(r[i]);
            for (int k = 0; k < 3; ++k) {
                lo[k] = std::min(lo[k], c[3 * i + k] - rad);
                hi[k] = std::max(hi[k], c[3 * i + k] + rad);
            }
        }
    }

    // Surface-area-heuristic split of idx[b, e): for each axis, sort by centroid
    // and sweep every cut, cost = area(left) |left| + area(right) |right|; the
    // range is left sorted on the best axis. Returns the cut. (Object median on
    // the longest axis when RTW_BVH_MEDIAN is set: A/B only.)
    static double box_area(const double lo[3], const double hi[3]) {
        const double dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
        return dx * dy + dy * dz + dz * dx;
    }
    void sort_axis(uint32_t b, uint32_t e, uint32_t axis) {
        std::sort(idx.begin() + b, idx.begin() + e, [&](uint32_t x, uint32_t y) {
            const double cx = c[3 * x + axis], cy = c[3 * y + axis];
            return cx < cy || (cx == cy && x < y);
        });
    }
    uint32_t split(uint32_t b, uint32_t e) {
        const uint32_t n = e - b;
        if (median) {
            double clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
            for (uint32_t j = b; j < e; ++j)
                for (int k = 0; k < 3; ++k) {
                    clo[k] = std::min(clo[k], c[3 * idx[j] + k]);
                    chi[k] = std::max(chi[k], c[3 * idx[j] + k]);
                }
            uint32_t axis = 0;
            for (uint32_t k = 1; k < 3; ++k)
                if (chi[k] - clo[k] > chi[axis] - clo[axis]) axis = k;
            sort_axis(b, e, axis);
            return b + n / 2;
        }
        double best = INFINITY;
        uint32_t best_axis = 0, best_cut = b + n / 2;
        std::vector<double> right(n + 1);
        for (uint32_t axis = 0; axis < 3; ++axis) {
            sort_axis(b, e, axis);
            double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
            for (uint32_t j = n; j-- > 0;) {  // right[j] = area of idx[b + j, e)
                const uint32_t i = idx[b + j];
                const double rad = std::fabs(r[i]);
                for (int k = 0; k < 3; ++k) {
                    lo[k] = std::min(lo[k], c[3 * i + k] - rad);
                    hi[k] = std::max(hi[k], c[3 * i + k] + rad);
                }
                right[j] = box_area(lo, hi);
            }
            for (int k = 0; k < 3; ++k) lo[k] = INFINITY, hi[k] = -INFINITY;
            for (uint32_t j = 0; j + 1 < n; ++j) {  // cut after j: left = [b, b+j]
                const uint32_t i = idx[b + j];
                const double rad = std::fabs(r[i]);
                for (int k = 0; k < 3; ++k) {
                    lo[k] = std::min(lo[k], c[3 * i + k] - rad);
                    hi[k] = std::max(hi[k], c[3 * i + k] + rad);
                }
                const double cost = box_area(lo, hi) * (j + 1) + right[j + 1] * (n - j - 1);
                if (cost < best) best = cost, best_axis = axis, best_cut = b + j + 1;
            }
        }
        sort_axis(b, e, best_axis);
        return best_cut;
    }

    // leaf id = sphere index: a candidate is its sphere (no index lookup after the walk)
    uint32_t leaf_record(uint32_t i) {
        const uint32_t k = i;
        ++n_leaf;
        float *L = &out->leaves[8 * static_cast<size_t>(k)];
        L[0] = static_cast<float>(c[3 * i]), L[1] = static_cast<float>(c[3 * i + 1]);
        L[2] = static_cast<float>(c[3 * i + 2]), L[3] = r2p[i];
        const double rr = r[i] * r[i];
        L[4] = up_f32((2. * (static_cast<double>(r2p[i]) - rr)) * (1. + 1e-6));
        L[5] = as_f32(i), L[6] = 0.f, L[7] = 0.f;
        return k;
    }

    // Emits the 4-wide node over idx[b, e) (pre-order ids); returns its id. Up to
    // 4 spheres become sphere children; more are cut into 4 parts by two levels
    // of median splits, each part a sphere child (1 sphere) or an inner child.
    uint32_t wide(uint32_t b, uint32_t e, uint32_t depth) {
        out->depth = std::max(out->depth, depth);
        std::vector<std::pair<uint32_t, uint32_t>> part;
        if (e - b <= 4) {
            for (uint32_t j = b; j < e; ++j) part.push_back({j, j + 1});
        } else {
            const uint32_t m = split(b, e);
            const uint32_t m0 = split(b, m), m1 = split(m, e);
            part = {{b, m0}, {m0, m}, {m, m1}, {m1, e}};
        }
        const uint32_t id = static_cast<uint32_t>(out->nodes.size() / kNodeFloats);
        out->nodes.resize(out->nodes.size() + kNodeFloats, 0.f);
        uint32_t ref[4] = {kEmpty, kEmpty, kEmpty, kEmpty}, masks = 0;
        double cen[4][3] = {};
        float box[6][4];
        for (int q = 0; q < 6; ++q)
            for (int j = 0; j < 4; ++j) box[q][j] = INFINITY;  // empty slot (masked by its ref)
        for (size_t j = 0; j < part.size(); ++j) {
            double lo[3], hi[3];
            bounds(part[j].first, part[j].second, lo, hi);
            double m = 0.;
            for (int k = 0; k < 3; ++k) m = std::max(m, std::max(std::fabs(lo[k]), std::fabs(hi[k])));
            const double pad = kPadKd * m + 1e-30;
            for (int k = 0; k < 3; ++k) {
                box[2 * k][j] = down_f32(lo[k] - pad);
                box[2 * k + 1][j] = up_f32(hi[k] + pad);
                cen[j][k] = 0.5 * (lo[k] + hi[k]);
            }
        }
        for (size_t j = 0; j < part.size(); ++j) {
            const uint32_t pb = part[j].first, pe = part[j].second;
            const bool leaf = pe - pb == 1;
            ref[j] = leaf ? leaf_record(idx[pb]) : wide(pb, pe, depth + 1);
            masks |= (1u << j) | (leaf ? 1u << (4 + j) : 0u);
        }
        // near-to-far child order per ray octant (bit k set: direction k < 0)
        uint32_t ord[2] = {0, 0};
        for (uint32_t o = 0; o < 8; ++o) {
            int perm[4] = {0, 1, 2, 3};
            std::stable_sort(perm, perm + 4, [&](int a, int b2) {
                if ((ref[a] == kEmpty) != (ref[b2] == kEmpty)) return ref[b2] == kEmpty;
                double ka = 0., kb = 0.;
                for (int k = 0; k < 3; ++k) {
                    const double s = (o >> k) & 1u ? -1. : 1.;
                    ka += s * cen[a][k], kb += s * cen[b2][k];
                }
                return ka < kb;
            });
            uint32_t byte = 0;
            for (int t = 0; t < 4; ++t) byte |= static_cast<uint32_t>(perm[t]) << (2 * t);
            ord[o >> 2] |= byte << (8 * (o & 3));
        }
        float *N = &out->nodes[kNodeFloats * static_cast<size_t>(id)];
        for (int q = 0; q < 6; ++q)
            for (int j = 0; j < 4; ++j) N[4 * q + j] = box[q][j];
        uint32_t packed[2] = {0, 0};
        for (int j = 0; j < 4; ++j)
            if (ref[j] != kEmpty) packed[j >> 1] |= (ref[j] & 0xffffu) << (16 * (j & 1));
        N[24] = as_f32(packed[0]), N[25] = as_f32(packed[1]), N[26] = as_f32(masks), N[27] = 0.f;
        N[28] = as_f32(ord[0]), N[29] = as_f32(ord[1]), N[30] = 0.f, N[31] = 0.f;
        return id;
    }
};

}  // namespace

bool build(const double *centers, const double *radii, const float *r2p, uint32_t n, Bvh &out) {
    out = Bvh{};
    if (n > kMaxSpheres) return false;
    // "always": non-finite or far-out spheres, and huge radii (ground planes)
    std::vector<double> ar;
    for (uint32_t i = 0; i < n; ++i)
        if (std::isfinite(radii[i])) ar.push_back(std::fabs(radii[i]));
    double med = 0.;
    if (!ar.empty()) {
        std::nth_element(ar.begin(), ar.begin() + ar.size() / 2, ar.end());
        med = ar[ar.size() / 2];
    }
    std::vector<uint32_t> rest;
    for (uint32_t i = 0; i < n; ++i) {
        const double *ci = centers + 3 * i;
        const double rad = std::fabs(radii[i]);
        double m = std::max(std::max(std::fabs(ci[0]), std::fabs(ci[1])), std::fabs(ci[2]));
        const bool finite = std::isfinite(m) && std::isfinite(rad) && std::isfinite(r2p[i]);
        if (!finite || m + rad > 1e7 || rad > kHugeRatio * med)
            out.always.push_back(i);
        else
            rest.push_back(i);
    }
    if (out.always.size() > kMaxAlways) return false;
    const uint32_t m = static_cast<uint32_t>(rest.size());
    // indexed by sphere; the walk never reaches an "always" slot, but every slot holds
    // its sphere's pass-1 record: the drain groups read them as their filter records
    out.leaves.assign(8 * static_cast<size_t>(n), 0.f);
    out.n_leaf = n;
    for (uint32_t i : out.always) {
        float *L = &out.leaves[8 * static_cast<size_t>(i)];
        L[0] = static_cast<float>(centers[3 * i]), L[1] = static_cast<float>(centers[3 * i + 1]);
        L[2] = static_cast<float>(centers[3 * i + 2]), L[3] = r2p[i];
        L[5] = as_f32(i);
    }
    if (m == 0) return true;
    Builder b{centers, radii, r2p, rest, &out};
    b.median = rtw::Knobs().get("RTW_BVH_MEDIAN") != nullptr;  // A/B only (RTW_AB)
    b.wide(0, m, 1);
    out.n_node = static_cast<uint32_t>(out.nodes.size() / kNodeFloats);
    return true;
}

// Inside-cut lists (rtw_accel.h): for every sphere S the spheres T whose gap to S
// is within delta(S, T); lists longer than kMaxNbr (e.g. a ground sphere with
// every small sphere resting on it) get no cut. O(n^2) pairs, scenes of up to
// 8192 spheres; larger ones (and any non-finite sphere) get no cuts.
void build_inside(const double *centers, const double *radii, uint32_t n, std::vector<uint32_t> &info,
                  std::vector<uint16_t> &ids, const uint8_t *trap_ok, std::vector<TrapRec> *trap) {
    info.assign(n, kNbrNone);
    ids.clear();
    if (trap) trap->assign(n, TrapRec{0., 0., 0., kTrapNever});
    if (n > 8192) return;
    std::vector<double> m(n);
    for (uint32_t i = 0; i < n; ++i) {
        const double *ci = centers + 3 * i;
        m[i] = std::max(std::max(std::fabs(ci[0]), std::fabs(ci[1])), std::fabs(ci[2]));
        if (!std::isfinite(m[i]) || !std::isfinite(radii[i]) || m[i] > 1e12 || std::fabs(radii[i]) > 1e12) return;
    }
    std::vector<uint32_t> nb;
    std::vector<double> nb_delta;
    for (uint32_t s = 0; s < n; ++s) {
        nb.clear(), nb_delta.clear();
        const double rs = std::fabs(radii[s]);
        for (uint32_t t = 0; t < n; ++t) {
            if (t == s) continue;
            const double rt = std::fabs(radii[t]);
            double d2 = 0.;
            for (int k = 0; k < 3; ++k) {
                const double q = centers[3 * s + k] - centers[3 * t + k];
                d2 += q * q;
            }
            const double D = std::sqrt(d2);
            const double delta = kNbrMargin * (5. * rs + 2. * rt + D + m[s] + m[t]);
            if (D - rs - rt <= delta) nb.push_back(t), nb_delta.push_back(delta);
        }
        if (nb.size() <= kMaxNbr) {
            info[s] = (static_cast<uint32_t>(ids.size()) << 8) | static_cast<uint32_t>(nb.size());
            for (uint32_t t : nb) ids.push_back(static_cast<uint16_t>(t));
        }
        if (!trap || !trap_ok || !trap_ok[s] || !(radii[s] >= 0.02)) continue;
        TrapRec &tr = (*trap)[s];
        if (nb.empty()) {
            tr = TrapRec{0., 0., 0., 1.};
            continue;
        }
        // w: mean direction towards the neighbours; every neighbour point x has
        // (x - c_S).w >= (c_T - c_S).w - r_T, so chords with both ends below
        // m = the minimum of that less delta stay delta clear of all of them
        double w[3] = {0., 0., 0.};
        bool ok = true;
        for (uint32_t t : nb) {
            double q[3], D = 0.;
            for (int k = 0; k < 3; ++k) q[k] = centers[3 * t + k] - centers[3 * s + k], D += q[k] * q[k];
            D = std::sqrt(D);
            if (!(D > 1e-9 * (rs + 1.))) ok = false;
            for (int k = 0; k < 3; ++k) w[k] += q[k] / D;
        }
        const double wl = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
        if (!ok || !(wl > 1e-6)) continue;
        for (double &x : w) x /= wl;
        double mm = INFINITY;
        for (size_t j = 0; j < nb.size(); ++j) {
            const uint32_t t = nb[j];
            double proj = 0.;
            for (int k = 0; k < 3; ++k) proj += (centers[3 * t + k] - centers[3 * s + k]) * w[k];
            mm = std::min(mm, proj - std::fabs(radii[t]) - nb_delta[j]);
        }
        const double cap = mm / rs - 1e-9;
        if (cap > -0.999) tr = TrapRec{w[0], w[1], w[2], std::min(cap, 1.)};
    }
}

}  // namespace rtw_accel
