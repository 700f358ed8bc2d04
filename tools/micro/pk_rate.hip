// Micro-benchmark: issue rate of v_fma_f32, v_pk_fma_f32 (with a splat operand) and
// v_fma_f64 on one gfx950 chip -- decides whether the f32 Jacobi phase gains from
// packing pairs of rows into float2 registers.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int ITERS = 4096, NACC = 8;

__global__ __launch_bounds__(256) void k_f32(float *out, float m, float a)
{
    float acc[NACC];
    for (int k = 0; k < NACC; ++k) acc[k] = threadIdx.x + k;
    for (int it = 0; it < ITERS; ++it)
#pragma unroll
        for (int k = 0; k < NACC; ++k) acc[k] = __builtin_fmaf(acc[k], m, a);
    float s = 0;
    for (int k = 0; k < NACC; ++k) s += acc[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_pk(float *out, float m, float a)
{
    f2 acc[NACC];
    for (int k = 0; k < NACC; ++k) acc[k] = f2{(float)threadIdx.x + k, (float)k};
    const f2 mm = f2{m, m}, aa = f2{a, a};
    for (int it = 0; it < ITERS; ++it)
#pragma unroll
        for (int k = 0; k < NACC; ++k) acc[k] = __builtin_elementwise_fma(acc[k], mm, aa);
    float s = 0;
    for (int k = 0; k < NACC; ++k) s += acc[k].x + acc[k].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_f64(float *out, double m, double a)
{
    double acc[NACC];
    for (int k = 0; k < NACC; ++k) acc[k] = threadIdx.x + k;
    for (int it = 0; it < ITERS; ++it)
#pragma unroll
        for (int k = 0; k < NACC; ++k) acc[k] = __builtin_fma(acc[k], m, a);
    double s = 0;
    for (int k = 0; k < NACC; ++k) s += acc[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (float)s;
}

// splat of a lane-varying scalar (the broadcast rotation c, s of the Jacobi update)
__global__ __launch_bounds__(256) void k_pk_splat(float *out, const float *cs)
{
    f2 acc[NACC];
    for (int k = 0; k < NACC; ++k) acc[k] = f2{(float)threadIdx.x + k, (float)k};
    float c = cs[threadIdx.x], s = cs[threadIdx.x + 256];
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int k = 0; k < NACC; k += 2) {
            const f2 x = acc[k], y = acc[k + 1];
            acc[k] = __builtin_elementwise_fma((f2)(-s), y, c * x);
            acc[k + 1] = __builtin_elementwise_fma((f2)s, x, c * y);
        }
        c = __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, c), 0xB1, 0xF, 0xF, false) ? c : s;
    }
    float t = 0;
    for (int k = 0; k < NACC; ++k) t += acc[k].x + acc[k].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = t;
}

int main()
{
    float *out, *cs;
    hipMalloc(&out, 256 * 4096 * 4);
    hipMalloc(&cs, 512 * 4);
    hipMemset(cs, 0, 512 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int blocks = 256 * 16;
    auto run = [&](const char *name, auto launch, double ops_per_thread) {
        launch();
        hipDeviceSynchronize();
        hipEventRecord(e0);
        for (int r = 0; r < 5; ++r) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double instr = 5.0 * blocks * 256 / 64 * ops_per_thread;  // wave instructions
        printf("%-10s %8.3f ms  %.3f T wave-instr/s  per CU per clk(2.4GHz): %.3f\n", name, ms, instr / ms / 1e9,
               instr / (ms * 1e-3) / 256 / 2.4e9);
    };
    run("f32 fma", [&] { hipLaunchKernelGGL(k_f32, dim3(blocks), dim3(256), 0, 0, out, 1.0001f, 0.5f); }, ITERS * NACC);
    run("pk fma", [&] { hipLaunchKernelGGL(k_pk, dim3(blocks), dim3(256), 0, 0, out, 1.0001f, 0.5f); }, ITERS * NACC);
    run("f64 fma", [&] { hipLaunchKernelGGL(k_f64, dim3(blocks), dim3(256), 0, 0, out, 1.0001, 0.5); }, ITERS * NACC);
    run("pk rot", [&] { hipLaunchKernelGGL(k_pk_splat, dim3(blocks), dim3(256), 0, 0, out, cs); }, ITERS * NACC);
    printf("(pk rot counts 1 instr per float2 element op pair: 2 pk ops per element -> see ISA)\n");
    return 0;
}
