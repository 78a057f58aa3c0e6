// Developer tool: does a wave64 VALU instruction issue faster when most of its
// lanes are masked off? (The drain groups run one pixel's serial chain on all 64
// lanes of a wave; if a 16-lane exec mask cost fewer cycles per instruction, a
// drained segment could run on a quarter wave.) One wave per workgroup, one
// workgroup per CU; each wave times a loop of independent f64 / f32 FMAs (8
// chains) or an integer xorshift chain under an exec mask of L active lanes with
// s_memtime. Prints cycles per instruction per pattern.
// Usage: hipcc --offload-arch=gfx950 -O3 -o ubench_exec tools/ubench_exec.hip && ./ubench_exec
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                           \
    do {                                                                \
        hipError_t e = (x);                                             \
        if (e != hipSuccess) {                                          \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); \
            return 1;                                                   \
        }                                                               \
    } while (0)

constexpr int kIters = 4096;

template <int kKind>
__global__ __launch_bounds__(64) void bench(uint32_t active, uint64_t *cycles, double *sink) {
    const uint32_t lane = threadIdx.x;
    double a0 = lane * 1e-3, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    float f0 = lane * 1e-3f, f1 = f0 + 1, f2 = f0 + 2, f3 = f0 + 3, f4 = f0 + 4, f5 = f0 + 5, f6 = f0 + 6, f7 = f0 + 7;
    uint32_t x0 = lane + 1, x1 = lane + 7, x2 = lane + 11, x3 = lane + 13;
    const double m = 0.999999, c = 1e-9;
    const float mf = 0.999999f, cf = 1e-9f;
    uint64_t t0 = 0, t1 = 0;
    if (lane < active) {
        t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < kIters; ++i) {
            if constexpr (kKind == 0) {  // 8 independent f64 FMA chains
                a0 = __builtin_fma(a0, m, c), a1 = __builtin_fma(a1, m, c), a2 = __builtin_fma(a2, m, c);
                a3 = __builtin_fma(a3, m, c), a4 = __builtin_fma(a4, m, c), a5 = __builtin_fma(a5, m, c);
                a6 = __builtin_fma(a6, m, c), a7 = __builtin_fma(a7, m, c);
            } else if constexpr (kKind == 1) {  // 8 independent f32 FMA chains (not packed: asm barrier)
                f0 = __builtin_fmaf(f0, mf, cf), f1 = __builtin_fmaf(f1, mf, cf), f2 = __builtin_fmaf(f2, mf, cf);
                f3 = __builtin_fmaf(f3, mf, cf), f4 = __builtin_fmaf(f4, mf, cf), f5 = __builtin_fmaf(f5, mf, cf);
                f6 = __builtin_fmaf(f6, mf, cf), f7 = __builtin_fmaf(f7, mf, cf);
                asm volatile("" : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3), "+v"(f4), "+v"(f5), "+v"(f6), "+v"(f7));
            } else if constexpr (kKind == 3) {  // ONE dependent f64 FMA chain (a drain's serial shape)
                a0 = __builtin_fma(a0, m, c);
                asm volatile("" : "+v"(a0));
            } else {  // u128 xorshift(23,17,26) on 4 u32 limbs: an integer chain (8 ops)
                x0 ^= x0 << 23, x1 ^= x1 >> 17, x2 ^= x2 << 26, x3 ^= x3 >> 5;
                asm volatile("" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3));
            }
        }
        t1 = __builtin_amdgcn_s_memtime();
    }
    if (lane == 0) cycles[blockIdx.x] = t1 - t0;
    sink[blockIdx.x * 64 + lane] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + f0 + f1 + f2 + f3 + f4 + f5 + f6 + f7 +
                                   static_cast<double>(x0 ^ x1 ^ x2 ^ x3);
}

// Which SIMD each wave of a 768-thread workgroup lands on (HW_ID.SIMD_ID, bits 5:4),
// with a large dynamic LDS request so one workgroup holds the CU (as the render does).
__global__ __launch_bounds__(768) void simd_map(uint32_t *out) {
    extern __shared__ uint32_t lds[];
    const uint32_t hw = __builtin_amdgcn_s_getreg((1 << 11) | (4 << 6) | 4);  // hwreg(HW_REG_HW_ID, 4, 2)
    if ((threadIdx.x & 63u) == 0) {
        lds[threadIdx.x >> 6] = hw;
        out[blockIdx.x * 12 + (threadIdx.x >> 6)] = hw & 3u;
    }
}

int map_simds(int blocks) {
    uint32_t *d;
    CK(hipMalloc(&d, blocks * 12 * sizeof(uint32_t)));
    hipLaunchKernelGGL(simd_map, dim3(blocks), dim3(768), 140 * 1024, nullptr, d);
    CK(hipDeviceSynchronize());
    std::vector<uint32_t> h(blocks * 12);
    CK(hipMemcpy(h.data(), d, h.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
    std::vector<int> same(12, 0);
    for (int b = 0; b < blocks; ++b)
        for (int w = 0; w < 12; ++w) same[w] += h[b * 12 + w] == h[w];
    std::printf("wave -> SIMD in workgroup 0:");
    for (int w = 0; w < 12; ++w) std::printf(" %u", h[w]);
    std::printf("  (workgroups with the same map per wave:");
    for (int w = 0; w < 12; ++w) std::printf(" %d", same[w]);
    std::printf(" of %d)\n", blocks);
    CK(hipFree(d));
    return 0;
}

template <int kKind>
int run(const char *name, int per_iter, int blocks) {
    uint64_t *cyc;
    double *sink;
    CK(hipMalloc(&cyc, blocks * sizeof(uint64_t)));
    CK(hipMalloc(&sink, blocks * 64 * sizeof(double)));
    for (uint32_t active : {64u, 48u, 32u, 17u, 16u, 8u, 1u}) {
        for (int rep = 0; rep < 2; ++rep) {  // first launch warms up
            hipLaunchKernelGGL(bench<kKind>, dim3(blocks), dim3(64), 0, nullptr, active, cyc, sink);
            CK(hipDeviceSynchronize());
        }
        std::vector<uint64_t> h(blocks);
        CK(hipMemcpy(h.data(), cyc, blocks * sizeof(uint64_t), hipMemcpyDeviceToHost));
        double sum = 0;
        for (uint64_t v : h) sum += static_cast<double>(v);
        std::printf("%-22s active %2u lanes: %.2f cycles per instruction (s_memtime ticks, mean of %d waves)\n", name,
                    active, sum / blocks / (static_cast<double>(kIters) * per_iter), blocks);
    }
    CK(hipFree(cyc));
    CK(hipFree(sink));
    return 0;
}

int main() {
    int n_cu = 0;
    CK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0));
    if (map_simds(n_cu)) return 1;
    if (run<0>("f64 fma (8 chains)", 8, n_cu) || run<1>("f32 fma (8 chains)", 8, n_cu) ||
        run<2>("u32 shift-xor (4x2)", 8, n_cu) || run<3>("f64 fma (1 dep chain)", 1, n_cu))
        return 1;
    return 0;
}
