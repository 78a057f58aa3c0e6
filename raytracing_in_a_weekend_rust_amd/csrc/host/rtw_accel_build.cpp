// rtw_accel_build.cpp -- host builder of the exact-result sphere BVH
// (csrc/rtw_accel.h). Replaces nothing in the reference: Scene::hit
// (hittable.rs:131-143) scans every object; this structure only lets the kernel
// skip spheres it can prove irrelevant, and the kernel still returns the scan's
// (t, first index) result.
//
// Object-median split on the longest centroid axis, one sphere per leaf, so the
// depth is ceil(log2 n) (<= 11 for n <= 2048): the kernel's register stack holds
// 12 entries. Inner nodes are numbered in pre-order (root 0), leaves in walk
// order; a child id >= n_inner names leaf (id - n_inner).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <numeric>
#include <vector>

#include "rtw_accel.h"

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
    uint32_t next_inner = 0, next_leaf = 0, n_inner = 0, max_depth = 0;

    void box_of(uint32_t b, uint32_t e, double lo[3], double hi[3]) const {
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

    // Builds idx[b, e); returns the child id of the subtree's root.
    uint32_t node(uint32_t b, uint32_t e, uint32_t depth) {
        if (e - b == 1) {
            const uint32_t k = next_leaf++, i = idx[b];
            float *L = &out->leaves[8 * static_cast<size_t>(k)];
            L[0] = static_cast<float>(c[3 * i]), L[1] = static_cast<float>(c[3 * i + 1]);
            L[2] = static_cast<float>(c[3 * i + 2]), L[3] = r2p[i];
            const double rr = r[i] * r[i];
            L[4] = up_f32((2. * (static_cast<double>(r2p[i]) - rr)) * (1. + 1e-6));
            L[5] = as_f32(i), L[6] = 0.f, L[7] = 0.f;
            return n_inner + k;
        }
        max_depth = std::max(max_depth, depth);
        const uint32_t id = next_inner++;
        double lo[3], hi[3];
        box_of(b, e, lo, hi);
        // centroid bounds -> split axis
        double clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (uint32_t j = b; j < e; ++j)
            for (int k = 0; k < 3; ++k) {
                clo[k] = std::min(clo[k], c[3 * idx[j] + k]);
                chi[k] = std::max(chi[k], c[3 * idx[j] + k]);
            }
        uint32_t axis = 0;
        for (uint32_t k = 1; k < 3; ++k)
            if (chi[k] - clo[k] > chi[axis] - clo[axis]) axis = k;
        std::sort(idx.begin() + b, idx.begin() + e, [&](uint32_t x, uint32_t y) {
            const double cx = c[3 * x + axis], cy = c[3 * y + axis];
            return cx < cy || (cx == cy && x < y);
        });
        const uint32_t mid = b + (e - b) / 2;
        const uint32_t left = node(b, mid, depth + 1);
        const uint32_t right = node(mid, e, depth + 1);
        // inflate by kPadK * M_b (M_b = max |coordinate|), round outward to f32
        double m = 0.;
        for (int k = 0; k < 3; ++k) m = std::max(m, std::max(std::fabs(lo[k]), std::fabs(hi[k])));
        const double pad = kPadKd * m + 1e-30;
        float *N = &out->nodes[8 * static_cast<size_t>(id)];
        for (int k = 0; k < 3; ++k) {
            N[k] = down_f32(lo[k] - pad);
            N[4 + k] = up_f32(hi[k] + pad);
        }
        N[3] = as_f32(left | (axis << 30));
        N[7] = as_f32(right);
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
    out.n_leaf = m;
    out.n_inner = m ? m - 1 : 0;
    out.nodes.assign(8 * static_cast<size_t>(out.n_inner), 0.f);
    out.leaves.assign(8 * static_cast<size_t>(m), 0.f);
    if (m) {
        Builder b{centers, radii, r2p, rest, &out};
        b.n_inner = out.n_inner;
        b.node(0, m, 1);
        out.depth = b.max_depth;
        if (out.depth > kMaxDepth) return false;
    }
    return true;
}

}  // namespace rtw_accel
