// Micro-benchmark: SIMD cycles per VALU instruction for NCH independent dependent-fma
// chains per wave, f32 and f64, at 1-4 waves per SIMD -- how much instruction-level
// parallelism a wave needs before the SIMD issues at its peak (2 cycles per f32 op,
// 4 per f64 op on gfx950).  Build: hipcc --offload-arch=gfx950 -O3 chain_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITERS = 1 << 13;

template <int NCH>
__global__ __launch_bounds__(64) void k_chaind(double *out, double m, double a)
{
    double acc[NCH];
#pragma unroll
    for (int k = 0; k < NCH; ++k) acc[k] = (double)(threadIdx.x + k);
    for (int it = 0; it < ITERS; ++it)
#pragma unroll
        for (int k = 0; k < NCH; ++k) acc[k] = __builtin_fma(acc[k], m, a);
    double s = 0;
#pragma unroll
    for (int k = 0; k < NCH; ++k) s += acc[k];
    out[blockIdx.x * 64 + threadIdx.x] = s;
}

template <int NCH>
__global__ __launch_bounds__(64) void k_chainf(float *out, float m, float a)
{
    float acc[NCH];
#pragma unroll
    for (int k = 0; k < NCH; ++k) acc[k] = (float)(threadIdx.x + k);
    for (int it = 0; it < ITERS; ++it)
#pragma unroll
        for (int k = 0; k < NCH; ++k) acc[k] = __builtin_fmaf(acc[k], m, a);
    float s = 0;
#pragma unroll
    for (int k = 0; k < NCH; ++k) s += acc[k];
    out[blockIdx.x * 64 + threadIdx.x] = s;
}

int main()
{
    void *out;
    hipMalloc(&out, 256 * 64 * 16 * 8 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](const char *name, int nch, int w, auto launch) {
        const int blocks = 256 * 4 * w;
        launch(blocks);
        hipDeviceSynchronize();
        hipEventRecord(e0);
        launch(blocks);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double cyc = ms * 1e-3 * 2.4e9;
        printf("%s chains %d waves/SIMD %d: %.2f SIMD cycles per instruction, %.2f cycles per dependent step\n", name, nch, w,
               cyc / ((double)ITERS * nch * w), cyc / ITERS);
    };
#define RUNF(N)                                                                                                       \
    for (int w = 1; w <= 4; ++w)                                                                                      \
        run("f32", N, w, [&](int nb) { hipLaunchKernelGGL(k_chainf<N>, dim3(nb), dim3(64), 0, 0, (float *)out, 1.0001f, 0.5f); });
#define RUND(N)                                                                                                       \
    for (int w = 1; w <= 4; ++w)                                                                                      \
        run("f64", N, w, [&](int nb) { hipLaunchKernelGGL(k_chaind<N>, dim3(nb), dim3(64), 0, 0, (double *)out, 1.0001, 0.5); });
    RUNF(1) RUNF(2) RUNF(4) RUNF(8)
    RUND(1) RUND(2) RUND(4) RUND(8)
    return 0;
}
