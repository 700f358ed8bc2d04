// The dgesdd route on the GPU: dispatch of the second passes (tmfwm_fixup.h, one TU per block
// size: tmfwm_fixup<b>.hip) and the stage entry points the parity tests call.
#include "tmfwm_fixup.h"

#include <cstdlib>

namespace tmf {

#define TMF_FIXUP_DECL(B)                                                                                                    \
    hipError_t launch_embed_fixup_##B(const EmbedArgs &, const uint32_t *, const uint32_t *, int64_t, hipStream_t);          \
    hipError_t launch_extract_fixup_##B(const ExtractArgs &, const uint32_t *, const uint32_t *, int64_t, hipStream_t);
TMF_FIXUP_DECL(4)
TMF_FIXUP_DECL(6)
TMF_FIXUP_DECL(8)
TMF_FIXUP_DECL(10)
TMF_FIXUP_DECL(12)
TMF_FIXUP_DECL(14)
TMF_FIXUP_DECL(16)

hipError_t launch_embed_fixup(const EmbedArgs &a, const uint32_t *list, const uint32_t *count, int64_t max_entries, hipStream_t st)
{
    switch (a.block) {
    case 4: return launch_embed_fixup_4(a, list, count, max_entries, st);
    case 6: return launch_embed_fixup_6(a, list, count, max_entries, st);
    case 8: return launch_embed_fixup_8(a, list, count, max_entries, st);
    case 10: return launch_embed_fixup_10(a, list, count, max_entries, st);
    case 12: return launch_embed_fixup_12(a, list, count, max_entries, st);
    case 14: return launch_embed_fixup_14(a, list, count, max_entries, st);
    case 16: return launch_embed_fixup_16(a, list, count, max_entries, st);
    default: return hipErrorInvalidValue;
    }
}

hipError_t launch_extract_fixup(const ExtractArgs &a, const uint32_t *list, const uint32_t *count, int64_t max_entries, hipStream_t st)
{
    switch (a.block) {
    case 4: return launch_extract_fixup_4(a, list, count, max_entries, st);
    case 6: return launch_extract_fixup_6(a, list, count, max_entries, st);
    case 8: return launch_extract_fixup_8(a, list, count, max_entries, st);
    case 10: return launch_extract_fixup_10(a, list, count, max_entries, st);
    case 12: return launch_extract_fixup_12(a, list, count, max_entries, st);
    case 14: return launch_extract_fixup_14(a, list, count, max_entries, st);
    case 16: return launch_extract_fixup_16(a, list, count, max_entries, st);
    default: return hipErrorInvalidValue;
    }
}

// The reference route (TMFWM_ROUTE_REFERENCE): every block of the launch on the dgesdd route.
// The id list is the identity, written on the device (ids 0 .. n-1 and the count n).
__global__ __launch_bounds__(256) void list_all_kernel(uint32_t *__restrict__ list, uint32_t *__restrict__ count, uint32_t n)
{
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i < n) list[i] = i;
    if (i == 0) *count = n;
}

hipError_t launch_list_all(uint32_t *list, uint32_t *count, int64_t n, hipStream_t st)
{
    if (n <= 0 || n > 0xFFFFFFFFll) return hipErrorInvalidValue;
    hipLaunchKernelGGL(list_all_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, list, count, (uint32_t)n);
    return hipGetLastError();
}

// stage entry points (tmfwm_lapack_svd_blocks, tmfwm_lapack_nrm2): the same wave-parallel
// route as the fixup passes, one 64-lane workgroup per block, the workspace in LDS
__global__ __launch_bounds__(64) void lp_svd_blocks_kernel(const float *__restrict__ D, int64_t nb, int b, float *__restrict__ U,
                                                           float *__restrict__ S, float *__restrict__ Vt, int want_v,
                                                           int32_t *__restrict__ info)
{
    __shared__ double ws[lp::ws_doubles(lp::kMaxN)];
    for (int64_t k = blockIdx.x; k < nb; k += gridDim.x) {
        const int64_t o = k * b * b;
        const int rc = want_v ? lp::svd_f32_ws<true, lp::WavePar>(D + o, b, U + o, S + k * b, Vt + o, ws)
                              : lp::svd_f32_ws<false, lp::WavePar>(D + o, b, nullptr, S + k * b, nullptr, ws);
        if (info && threadIdx.x == 0) info[k] = rc;
        __syncthreads();
    }
}

__global__ __launch_bounds__(64) void lp_nrm2_kernel(const double *__restrict__ x, int64_t nvec, int n, int inc, double *__restrict__ out)
{
    const int64_t k = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (k < nvec) out[k] = lp::dnrm2(n, x + k * (int64_t)n * inc, inc);
}

hipError_t launch_lapack_svd_blocks(const float *D, int64_t nb, int block, float *U, float *S, float *Vt, int want_v, int32_t *info,
                                    hipStream_t st)
{
    if (nb == 0) return hipSuccess;
    hipLaunchKernelGGL(lp_svd_blocks_kernel, dim3((unsigned)(nb < 16384 ? nb : 16384)), dim3(64), 0, st, D, nb, block, U, S, Vt, want_v, info);
    return hipGetLastError();
}

hipError_t launch_lapack_nrm2(const double *x, int64_t nvec, int n, int inc, double *out, hipStream_t st)
{
    if (nvec == 0) return hipSuccess;
    hipLaunchKernelGGL(lp_nrm2_kernel, dim3((unsigned)((nvec + 63) / 64)), dim3(64), 0, st, x, nvec, n, inc, out);
    return hipGetLastError();
}

}  // namespace tmf
