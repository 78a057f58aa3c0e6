// Developer tool: calibrates rocprofv3 WRITE_SIZE on gfx950 for the access patterns
// of the persistent render kernel (MI355X_MICROARCH.md: "calibrate on a known byte
// count in your own access pattern"). One launch per pattern:
//   coalesced16  16 B per lane, consecutive lanes consecutive (the guide's exact case)
//   pix_scatter  3 x 8 B per "pixel" (an f64 RGB), pixels in a shuffled order (the
//                framebuffer as cost-ordered lanes write it)
//   atomic_one   one device-scope atomicAdd per wave on ONE word (the pixel cursor /
//                completion counters)
//   atomic_many  one atomicAdd per lane on consecutive words
// Usage: rocprofv3 --pmc WRITE_SIZE -d DIR -o run --output-format csv -- ./ubench_write
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x)                                                              \
    do {                                                                   \
        hipError_t e = (x);                                                \
        if (e != hipSuccess) {                                             \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));    \
            return 1;                                                      \
        }                                                                  \
    } while (0)

__global__ void coalesced16(float4 *out, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = make_float4(1.f, 2.f, 3.f, static_cast<float>(i));
}
__global__ void pix_scatter(double *out, const uint32_t *order, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        double *o = out + static_cast<uint64_t>(order[i]) * 3u;
        o[0] = 0.25, o[1] = 0.5, o[2] = static_cast<double>(i);
    }
}
__global__ void atomic_one(uint32_t *c, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && (threadIdx.x & 63u) == 0) atomicAdd(c, 1u);
}
__global__ void atomic_many(uint32_t *c, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) atomicAdd(c + i, 1u);
}

int main() {
    const uint32_t n = 810000;  // the bench image's pixels
    float4 *f4;
    double *fb;
    uint32_t *order, *cnt;
    CK(hipMalloc(&f4, n * sizeof(float4)));
    CK(hipMalloc(&fb, n * 3 * sizeof(double)));
    CK(hipMalloc(&order, n * sizeof(uint32_t)));
    CK(hipMalloc(&cnt, n * sizeof(uint32_t)));
    std::vector<uint32_t> h(n);
    uint64_t x = 88172645463325252ull;
    for (uint32_t i = 0; i < n; ++i) h[i] = i;
    for (uint32_t i = n - 1; i > 0; --i) {  // Fisher-Yates, xorshift64
        x ^= x << 13, x ^= x >> 7, x ^= x << 17;
        std::swap(h[i], h[x % (i + 1)]);
    }
    CK(hipMemcpy(order, h.data(), n * sizeof(uint32_t), hipMemcpyHostToDevice));
    CK(hipMemset(cnt, 0, n * sizeof(uint32_t)));
    const dim3 g((n + 255) / 256), b(256);
    hipLaunchKernelGGL(coalesced16, g, b, 0, nullptr, f4, n);
    hipLaunchKernelGGL(pix_scatter, g, b, 0, nullptr, fb, order, n);
    hipLaunchKernelGGL(atomic_one, g, b, 0, nullptr, cnt, n);
    hipLaunchKernelGGL(atomic_many, g, b, 0, nullptr, cnt, n);
    CK(hipDeviceSynchronize());
    std::printf("n=%u: coalesced16 %u B, pix_scatter %u B, atomic_one %u atomics, atomic_many %u atomics\n", n,
                n * 16, n * 24, n / 64, n);
    return 0;
}
