// Developer tool: single-wave latencies on gfx950 (s_memtime cycles per op) for
// dependent f32 FMA, f64 FMA, f64 sqrt/div sequences, LDS load->use, and a
// uniform branch loop. Build: hipcc --offload-arch=gfx950 -O3 tools/lat_probe.hip -o /tmp/lat_probe
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ uint64_t now() {
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}

__global__ void probe(float *of, double *od, uint64_t *cyc, int n) {
    __shared__ float4 lds[1024];
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) lds[i] = make_float4(i, 1, 2, 3);
    __syncthreads();
    float x = threadIdx.x * 1e-3f;
    double y = threadIdx.x * 1e-3;
    const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
    uint64_t t0 = now();
#define F4 "v_fma_f32 %0, %0, %0, 1.0\n\tv_fma_f32 %0, %0, %0, 1.0\n\tv_fma_f32 %0, %0, %0, 1.0\n\tv_fma_f32 %0, %0, %0, 1.0\n\t"
    for (int i = 0; i < n / 4; ++i) asm volatile(F4 F4 F4 F4 : "+v"(x));
    uint64_t t1 = now();
    for (int i = 0; i < n; ++i) {
        asm volatile("v_fma_f64 %0, %0, %0, 1.0" : "+v"(y));
        asm volatile("v_fma_f64 %0, %0, %0, 1.0" : "+v"(y));
        asm volatile("v_fma_f64 %0, %0, %0, 1.0" : "+v"(y));
        asm volatile("v_fma_f64 %0, %0, %0, 1.0" : "+v"(y));
    }
    uint64_t t2 = now();
    double z = y;
    for (int i = 0; i < n; ++i) z = __builtin_sqrt(z + 1.0);
    uint64_t t3 = now();
    for (int i = 0; i < n; ++i) z = 3.0 / (z + 1.0);
    uint64_t t4 = now();
    int idx = threadIdx.x & 63;
    float acc = 0.f;
    for (int i = 0; i < n; ++i) {
        const float4 v = lds[idx];
        idx = (static_cast<int>(v.x) + 1) & 1023;
        acc += v.y;
    }
    uint64_t t5 = now();
    float w = x;
    float w2 = acc, w3 = x + 1.f;
#define I4 "v_fma_f32 %0, %0, %0, 1.0\n\tv_fma_f32 %1, %1, %1, 1.0\n\tv_fma_f32 %2, %2, %2, 1.0\n\tv_fma_f32 %3, %3, %3, 1.0\n\t"
    for (int i = 0; i < n / 4; ++i) asm volatile(I4 I4 I4 I4 : "+v"(w), "+v"(x), "+v"(w2), "+v"(w3));
    acc += w2 + w3;
    uint64_t t6 = now();
    // dependent packed f32 FMA chain
    double pk;
    __builtin_memcpy(&pk, &w, 4);
    __builtin_memcpy(reinterpret_cast<char *>(&pk) + 4, &w2, 4);
    const uint64_t t7 = now();
#define P4 "v_pk_fma_f32 %0, %0, %0, %0\n\tv_pk_fma_f32 %0, %0, %0, %0\n\tv_pk_fma_f32 %0, %0, %0, %0\n\tv_pk_fma_f32 %0, %0, %0, %0\n\t"
    for (int i = 0; i < n / 4; ++i) asm volatile(P4 P4 P4 P4 : "+v"(pk));
    const uint64_t t8 = now();
    // VALU compare -> SALU mask op -> VALU cndmask round trips
    float q = w;
    for (int i = 0; i < n / 4; ++i) {
#define X1 "v_cmp_nlt_f32_e64 s[20:21], %0, 1.0\n\ts_or_b64 s[20:21], s[20:21], s[22:23]\n\tv_cndmask_b32_e64 %0, %0, 2.0, s[20:21]\n\t"
        asm volatile("s_mov_b64 s[22:23], 0\n\t" X1 X1 X1 X1 : "+v"(q)::"s20", "s21", "s22", "s23");
    }
    const uint64_t t9 = now();
    acc += q;
    __builtin_memcpy(&w3, &pk, 4);
    acc += w3;
    if (threadIdx.x == 0) {
        cyc[8] = t8 - t7, cyc[9] = t9 - t8;
        cyc[6] = t6 - t0, cyc[7] = __builtin_amdgcn_s_memrealtime() - r0;
        cyc[0] = t1 - t0, cyc[1] = t2 - t1, cyc[2] = t3 - t2, cyc[3] = t4 - t3, cyc[4] = t5 - t4, cyc[5] = t6 - t5;
    }
    of[threadIdx.x + 1] = x + acc + w;
    od[threadIdx.x] = y + z;
}

// the cooperative filter loop of coop_pixel (64 lanes x jn spheres) in isolation
__global__ void filt_probe(const float4 *gfilt, uint32_t n, uint32_t jn_cap, int reps, uint64_t *cyc, uint32_t *out) {
    __shared__ float4 filt[1024];
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) filt[i] = gfilt[i];
    __syncthreads();
    const uint32_t sub = threadIdx.x & 63u;
    float ox = 13.f, oy = 2.f, oz = 3.f, ex = -0.97f, ey = -0.15f, ez = -0.22f, negG = -1e-3f;
    uint32_t acc = 0;
    const uint64_t t0 = now();
    for (int r = 0; r < reps; ++r) {
        uint32_t mask = 0;
        const uint32_t jn = min(jn_cap, (n + 63u) / 64u);
#pragma unroll 8
        for (uint32_t j = 0; j < jn; ++j) {
            const uint32_t i = sub + j * 64u;
            const float4 S = filt[min(i, n - 1u)];
            const float ocx = ox - S.x, ocy = oy - S.y, ocz = oz - S.z;
            const float hb = fmaf(ocx, ex, fmaf(ocy, ey, ocz * ez));
            const float cc = fmaf(ocx, ocx, fmaf(ocy, ocy, fmaf(ocz, ocz, -S.w)));
            const float disc = fmaf(hb, hb, -cc);
            mask |= static_cast<uint32_t>((i < n) & !(disc < negG)) << j;
        }
        acc += mask;
        ox += 1e-7f;  // loop-carried
    }
    const uint64_t t1 = now();
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
    out[threadIdx.x] = acc;
}

int main() {
    float *of;
    double *od;
    uint64_t *cyc;
    hipMalloc(&of, 4096);
    hipMalloc(&od, 8192);
    hipMalloc(&cyc, 160);
    const int n = 1000;
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, nullptr, of, od, cyc, n);
        hipDeviceSynchronize();
    }
    uint64_t h[10];
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    printf("cycles per op (one wave alone): dep f32 fma %.1f, dep f64 fma %.1f, f64 sqrt(+add) %.1f, "
           "f64 div(+add) %.1f, LDS b128 load->use chain %.1f, indep f32 fma %.1f\n",
           h[0] / (4.0 * n), h[1] / (4.0 * n), h[2] / double(n), h[3] / double(n), h[4] / double(n),
           h[5] / (4.0 * n));
    printf("dep v_pk_fma_f32 %.1f, v_cmp->s_or->v_cndmask round trip %.1f\n", h[8] / (4.0 * n), h[9] / (4.0 * n));
    {
        float4 hf[486];
        for (int i = 0; i < 486; ++i) hf[i] = make_float4(i * 0.1f, 0.2f, i * 0.05f, 0.04f);
        float4 *gf;
        uint32_t *o;
        hipMalloc(&gf, sizeof(hf));
        hipMalloc(&o, 4096);
        hipMemcpy(gf, hf, sizeof(hf), hipMemcpyHostToDevice);
        for (uint32_t cap : {1u, 2u, 4u, 8u}) {
            for (int rep = 0; rep < 2; ++rep) {
                hipLaunchKernelGGL(filt_probe, dim3(1), dim3(64), 0, nullptr, gf, 486u, cap, 1000, cyc, o);
                hipDeviceSynchronize();
            }
            uint64_t c;
            hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
            printf("coop filter, %u spheres per lane: %.1f cycles per pass\n", cap, c / 1000.0);
        }
    }
    printf("s_memtime cycles %llu over %llu x 10 ns: %.3f GHz\n", (unsigned long long)h[6], (unsigned long long)h[7],
           h[6] / (h[7] * 10.0));
    return 0;
}
