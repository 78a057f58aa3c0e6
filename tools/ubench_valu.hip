// Developer microbenchmark: sustained VALU rates on gfx950 for the op kinds the
// sampling kernel uses (f32 FMA, packed f32 FMA, f64 add/mul/FMA, f64 sqrt/div
// sequences). 8 independent chains per lane, 2048 x 256 threads. Prints
// G lane-ops/s and the implied FLOP rate (FMA = 2 FLOP).
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int kIters = 4096;

template <typename T>
__global__ void k_fma(T *out, T a, T b) {
    T x[8];
    for (int i = 0; i < 8; ++i) x[i] = static_cast<T>(threadIdx.x + i);
    for (int it = 0; it < kIters; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = __builtin_fma(x[i], a, b);
    T s = 0;
    for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_fma32(float *out, float a, float b) {
    float x[8];
    for (int i = 0; i < 8; ++i) x[i] = static_cast<float>(threadIdx.x + i);
    for (int it = 0; it < kIters; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = __builtin_fmaf(x[i], a, b);
    float s = 0;
    for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_pkfma(float *out, float a, float b) {
    f2 x[8];
    const f2 av = {a, a}, bv = {b, b};
    for (int i = 0; i < 8; ++i) x[i] = f2{static_cast<float>(threadIdx.x + i), 1.f};
    for (int it = 0; it < kIters; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = __builtin_elementwise_fma(x[i], av, bv);
    float s = 0;
    for (int i = 0; i < 8; ++i) s += x[i].x + x[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <int OP>
__global__ void k_f64(double *out, double a, double b) {
    double x[8];
    for (int i = 0; i < 8; ++i) x[i] = static_cast<double>(threadIdx.x + i);
    for (int it = 0; it < kIters; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = OP == 0 ? x[i] + a : OP == 1 ? x[i] * a : __builtin_fma(x[i], a, b);
    double s = 0;
    for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_sqrtdiv(double *out, double a) {
    double x[4];
    for (int i = 0; i < 4; ++i) x[i] = static_cast<double>(threadIdx.x + i + 1);
    for (int it = 0; it < kIters / 16; ++it)
#pragma unroll
        for (int i = 0; i < 4; ++i) x[i] = __builtin_sqrt(x[i]) / a + 1.0;
    out[blockIdx.x * blockDim.x + threadIdx.x] = x[0] + x[1] + x[2] + x[3];
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
    const double lanes = double(blocks) * threads;
    void *buf;
    hipMalloc(&buf, blocks * threads * 8);
    auto report = [&](const char *name, double ms, double ops_per_lane, double flop_per_op) {
        const double gops = lanes * ops_per_lane / (ms * 1e6);
        std::printf("%-22s %8.3f ms  %9.1f G lane-op/s  %7.2f TFLOP/s\n", name, ms, gops,
                    gops * flop_per_op / 1e3);
    };
    const double n8 = 8.0 * kIters;
    report("v_fma_f32", time_ms([&] { k_fma32<<<blocks, threads>>>((float *)buf, 0.999f, 0.5f); }), n8, 2);
    report("v_pk_fma_f32 (x2)", time_ms([&] { k_pkfma<<<blocks, threads>>>((float *)buf, 0.999f, 0.5f); }), 2 * n8, 2);
    report("v_add_f64", time_ms([&] { k_f64<0><<<blocks, threads>>>((double *)buf, 0.5, 0.25); }), n8, 1);
    report("v_mul_f64", time_ms([&] { k_f64<1><<<blocks, threads>>>((double *)buf, 0.999, 0.25); }), n8, 1);
    report("v_fma_f64", time_ms([&] { k_f64<2><<<blocks, threads>>>((double *)buf, 0.999, 0.25); }), n8, 2);
    report("sqrt+div+add f64", time_ms([&] { k_sqrtdiv<<<blocks, threads>>>((double *)buf, 1.7); }), 4.0 * kIters / 16, 1);
    hipFree(buf);
    return 0;
}
