// Micro-benchmark: dependent-chain cost of v_fma_f32 vs v_pk_fma_f32 at low occupancy
// (1-3 waves per SIMD, like the SVD kernels) -- issue rate is not the whole story
// when every instruction depends on the previous one.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int ITERS = 1 << 14;

template <int NCH>
__global__ __launch_bounds__(64) void k_f32(float *out, float m, float a)
{
    float acc[NCH];
    for (int k = 0; k < NCH; ++k) acc[k] = threadIdx.x + k;
    for (int it = 0; it < ITERS; ++it)
#pragma unroll
        for (int k = 0; k < NCH; ++k) acc[k] = __builtin_fmaf(acc[k], m, a);
    float s = 0;
    for (int k = 0; k < NCH; ++k) s += acc[k];
    out[blockIdx.x * 64 + threadIdx.x] = s;
}

template <int NCH>
__global__ __launch_bounds__(64) void k_pk(float *out, float m, float a)
{
    f2 acc[NCH];
    for (int k = 0; k < NCH; ++k) acc[k] = f2{(float)threadIdx.x + k, (float)k};
    const f2 mm = f2{m, m}, aa = f2{a, a};
    for (int it = 0; it < ITERS; ++it)
#pragma unroll
        for (int k = 0; k < NCH; ++k) acc[k] = __builtin_elementwise_fma(acc[k], mm, aa);
    float s = 0;
    for (int k = 0; k < NCH; ++k) s += acc[k].x + acc[k].y;
    out[blockIdx.x * 64 + threadIdx.x] = s;
}

int main()
{
    float *out;
    hipMalloc(&out, 256 * 64 * 16 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](const char *name, int waves_per_simd, auto launch) {
        const int blocks = 256 * 4 * waves_per_simd;
        launch(blocks);
        hipDeviceSynchronize();
        hipEventRecord(e0);
        launch(blocks);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        printf("%-14s waves/SIMD %d: %.3f ms -> %.2f clk per dependent step per wave (2.4 GHz)\n", name, waves_per_simd, ms,
               ms * 1e-3 * 2.4e9 / ITERS);
    };
    for (int w = 1; w <= 3; ++w) {
        run("f32 chain x1", w, [&](int nb) { hipLaunchKernelGGL(k_f32<1>, dim3(nb), dim3(64), 0, 0, out, 1.0001f, 0.5f); });
        run("pk chain x1", w, [&](int nb) { hipLaunchKernelGGL(k_pk<1>, dim3(nb), dim3(64), 0, 0, out, 1.0001f, 0.5f); });
        run("f32 chain x2", w, [&](int nb) { hipLaunchKernelGGL(k_f32<2>, dim3(nb), dim3(64), 0, 0, out, 1.0001f, 0.5f); });
        run("pk chain x2", w, [&](int nb) { hipLaunchKernelGGL(k_pk<2>, dim3(nb), dim3(64), 0, 0, out, 1.0001f, 0.5f); });
        run("f32 chain x4", w, [&](int nb) { hipLaunchKernelGGL(k_f32<4>, dim3(nb), dim3(64), 0, 0, out, 1.0001f, 0.5f); });
        run("pk chain x4", w, [&](int nb) { hipLaunchKernelGGL(k_pk<4>, dim3(nb), dim3(64), 0, 0, out, 1.0001f, 0.5f); });
    }
    return 0;
}
