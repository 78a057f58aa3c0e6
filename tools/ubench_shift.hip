// Developer microbenchmark: issue rate of a 64-bit variable shift (v_lshrrev_b64, as the
// BVH walk extracts 16-bit child refs from a u64) against the 32-bit form (select of a
// word + v_bfe_u32) and a plain 32-bit op, 8 independent chains per lane.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr int kIters = 4096;

__global__ void k_shr64(uint32_t *out, uint32_t salt) {
    uint64_t x[8];
    for (int i = 0; i < 8; ++i) x[i] = (static_cast<uint64_t>(threadIdx.x + i) << 32) | (salt + i);
    uint32_t sh = threadIdx.x & 48u;
    for (int it = 0; it < kIters; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            x[i] = (x[i] >> sh) ^ (x[i] << 16);
            asm volatile("" : "+v"(sh));
        }
    uint64_t s = 0;
    for (int i = 0; i < 8; ++i) s ^= x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = static_cast<uint32_t>(s ^ (s >> 32));
}
__global__ void k_bfe32(uint32_t *out, uint32_t salt) {
    uint32_t lo[8], hi[8];
    for (int i = 0; i < 8; ++i) lo[i] = salt + i, hi[i] = threadIdx.x + i;
    uint32_t j = threadIdx.x & 3u;
    for (int it = 0; it < kIters; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t w = j < 2u ? lo[i] : hi[i];
            lo[i] = __builtin_amdgcn_ubfe(w, (j & 1u) * 16u, 16u) ^ hi[i];
            hi[i] = hi[i] + lo[i];
            asm volatile("" : "+v"(j));
        }
    uint32_t s = 0;
    for (int i = 0; i < 8; ++i) s ^= lo[i] ^ hi[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_add32(uint32_t *out, uint32_t salt) {
    uint32_t x[8];
    for (int i = 0; i < 8; ++i) x[i] = salt + threadIdx.x + i;
    for (int it = 0; it < kIters; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = (x[i] ^ salt) + 0x9e3779b9u;
    uint32_t s = 0;
    for (int i = 0; i < 8; ++i) s ^= x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename F>
double time_ms(F f) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    f();
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) f();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return ms / 5;
}

int main() {
    const int blocks = 2048, threads = 256;
    uint32_t *out;
    hipMalloc(&out, blocks * threads * sizeof(uint32_t));
    const double lane_ops = static_cast<double>(blocks) * threads * kIters * 8;
    const double t64 = time_ms([&] { hipLaunchKernelGGL(k_shr64, dim3(blocks), dim3(threads), 0, 0, out, 7u); });
    const double t32 = time_ms([&] { hipLaunchKernelGGL(k_bfe32, dim3(blocks), dim3(threads), 0, 0, out, 7u); });
    const double ta = time_ms([&] { hipLaunchKernelGGL(k_add32, dim3(blocks), dim3(threads), 0, 0, out, 7u); });
    std::printf("shr64+shl64+xor64 chain step: %.3f ms, %.1f G steps/s\n", t64, lane_ops / t64 / 1e6);
    std::printf("cndmask+bfe+xor+add step:     %.3f ms, %.1f G steps/s\n", t32, lane_ops / t32 / 1e6);
    std::printf("xor+add step (2 VALU):        %.3f ms, %.1f G steps/s\n", ta, lane_ops / ta / 1e6);
    hipFree(out);
    return 0;
}
