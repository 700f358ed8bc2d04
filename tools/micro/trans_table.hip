// Truth tables of the gfx950 f32 transcendental approximations v_rsq_f32 / v_rcp_f32
// (not specified to the bit), and a check that their results on every positive normal
// input follow from the table by exact power-of-two scaling:
//   rsq(m * 2^e) = rsq(m * 2^(e mod 2)) * 2^-(e - e mod 2)/2   (table: 2^24 inputs in [1, 4))
//   rcp(m * 2^e) = rcp(m) * 2^-e                               (table: 2^23 inputs in [1, 2))
// Writes rsq.bin / rcp.bin (raw u32 result bits) and prints mismatch counts as JSON.
// Build: hipcc --offload-arch=gfx950 -O3 tools/micro/trans_table.hip -o tools/micro/trans_table
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>

__global__ void tables(uint32_t *rsq, uint32_t *rcp)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < (1u << 24)) {
        const float x = __uint_as_float(((127u + (i >> 23)) << 23) | (i & 0x7FFFFFu));
        rsq[i] = __float_as_uint(__builtin_amdgcn_rsqf(x));
    }
    if (i < (1u << 23)) rcp[i] = __float_as_uint(__builtin_amdgcn_rcpf(__uint_as_float((127u << 23) | i)));
}

// every positive normal input; counts[0]: rsq mismatches, [1]: rcp mismatches with a normal
// predicted result, [2]: rcp inputs whose result would be subnormal (not modelled)
__global__ void check(const uint32_t *rsq, const uint32_t *rcp, unsigned long long *counts, uint32_t *first)
{
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t b = 0x00800000ull + blockIdx.x * blockDim.x + threadIdx.x; b < 0x7F800000ull; b += stride) {
        const float x = __uint_as_float((uint32_t)b);
        const int e = (int)(b >> 23) - 127;
        const int p = e & 1;  // e mod 2 (two's complement: also for e < 0)
        const uint32_t m = (uint32_t)b & 0x7FFFFFu;
        const float pr = __builtin_ldexpf(__uint_as_float(rsq[((uint32_t)p << 23) | m]), -((e - p) / 2));
        if (__float_as_uint(pr) != __float_as_uint(__builtin_amdgcn_rsqf(x))) {
            if (atomicAdd(&counts[0], 1ull) == 0) first[0] = (uint32_t)b;
        }
        const float t = __uint_as_float(rcp[m]);
        // t in (0.5, 1]: t * 2^-e is normal iff its exponent stays >= -126
        const int te = (int)(__float_as_uint(t) >> 23) - 127 - e;
        if (te < -126) {
            atomicAdd(&counts[2], 1ull);
        } else if (__float_as_uint(__builtin_ldexpf(t, -e)) != __float_as_uint(__builtin_amdgcn_rcpf(x))) {
            if (atomicAdd(&counts[1], 1ull) == 0) first[1] = (uint32_t)b;
        }
    }
}

int main(int argc, char **argv)
{
    const char *dir = argc > 1 ? argv[1] : ".";
    uint32_t *rsq, *rcp, *first;
    unsigned long long *counts;
    if (hipMalloc(&rsq, 4u << 24) || hipMalloc(&rcp, 4u << 23) || hipMalloc(&counts, 32) || hipMalloc(&first, 8)) return 1;
    hipMemset(counts, 0, 32);
    hipMemset(first, 0xFF, 8);
    tables<<<(1u << 24) / 256, 256>>>(rsq, rcp);
    check<<<65536, 256>>>(rsq, rcp, counts, first);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    std::vector<uint32_t> h1(1u << 24), h2(1u << 23);
    unsigned long long c[4];
    uint32_t f[2];
    hipMemcpy(h1.data(), rsq, 4u << 24, hipMemcpyDeviceToHost);
    hipMemcpy(h2.data(), rcp, 4u << 23, hipMemcpyDeviceToHost);
    hipMemcpy(c, counts, 32, hipMemcpyDeviceToHost);
    hipMemcpy(f, first, 8, hipMemcpyDeviceToHost);
    char path[4096];
    snprintf(path, sizeof path, "%s/rsq.bin", dir);
    FILE *o = fopen(path, "wb");
    if (!o || fwrite(h1.data(), 4, h1.size(), o) != h1.size()) return 3;
    fclose(o);
    snprintf(path, sizeof path, "%s/rcp.bin", dir);
    o = fopen(path, "wb");
    if (!o || fwrite(h2.data(), 4, h2.size(), o) != h2.size()) return 3;
    fclose(o);
    printf("{\"rsq_scaling_mismatches\": %llu, \"rcp_scaling_mismatches\": %llu, \"rcp_subnormal_results_skipped\": %llu, "
           "\"first_rsq_mismatch\": \"0x%08x\", \"first_rcp_mismatch\": \"0x%08x\"}\n",
           c[0], c[1], c[2], f[0], f[1]);
    return 0;
}
