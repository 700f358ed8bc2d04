// The dgesdd route on the GPU (tmfwm_lapack.h): the second-pass kernels of embed and
// extract and their launch templates.  Instantiated per block size in tmfwm_fixup<b>.hip
// (compiled in parallel); tmfwm_fallback.hip dispatches and holds the stage entry points.
//
// embed_kernel<b> runs the Jacobi route on every block and appends to a list the blocks
// whose conditioning test fails; embed_fixup_kernel<b> redoes exactly
// those blocks end to end -- luma, DCT, np.linalg.svd as LAPACK computes it, blend,
// reconstruct, IDCT, inverse colour -- and overwrites their pixels.  extract_kernel<b>
// appends the blocks whose sigma_1 enclosure does not decide f32(sigma_1) for either
// image; extract_fixup_kernel<b> computes both sigma_1 on the dgesdd route and writes the
// byte.  One thread per listed block, its working set in LDS; a grid-stride loop over the
// device-side count, so no host round trip sits between the passes.
#pragma once
#include "tmfwm_device.h"
#include "tmfwm_internal.h"
#include "tmfwm_lapack.h"

#include <mutex>

namespace tmf {

template <int B>
TMF_DEVI void load_dct_block(const uint8_t *frame, int W, int bi, int bj, float (&y)[B][B])
{
#pragma unroll
    for (int r = 0; r < B; ++r)
#pragma unroll
        for (int c = 0; c < B; ++c) {
            const uint8_t *p = frame + ((int64_t)(bi * B + r) * W + (int64_t)bj * B + c) * 3;
            y[r][c] = luma(p[0], p[1], p[2]);
        }
    // :192 / :279-282 -- DCT along axis 0, then axis 1
#pragma unroll
    for (int c = 0; c < B; ++c) {
        float col[B];
#pragma unroll
        for (int r = 0; r < B; ++r) col[r] = y[r][c];
        dct::dct2<B>(col);
#pragma unroll
        for (int r = 0; r < B; ++r) y[r][c] = col[r];
    }
#pragma unroll
    for (int r = 0; r < B; ++r) dct::dct2<B>(y[r]);
}

// Each thread's dgesdd works in LDS, not in private (scratch) memory: A, U, VT, d, e, tauq,
// taup and the work vectors (lp::ws_doubles), the block D and the f32 factors.  The route is
// a serial chain of dependent loads and stores per block, so its latency is the memory's:
// kFixT<B> threads per workgroup share <= 48 KB of LDS.
// The block size reaches the dgesdd routines as a run-time value, as it does from the stage
// kernel (lp_svd_blocks_kernel): with every call site in a TU passing the constant B, the
// compiler specialises the noinline routines on it (a TU per block size, tmfwm_fixup<b>.hip),
// and the b = 16 specialisation faulted on the GPU (illegal address) where the shared,
// run-time-n code -- host-sanitiser clean, GPU parity green -- does not.
TMF_DEVI int runtime_n(int n)
{
    asm volatile("" : "+v"(n));
    return n;
}

template <int B>
constexpr int kFixSlot = lp::ws_doubles(B) + (3 * B * B + B + 1) / 2;  // doubles per thread
// Two launches share the list (launch_fixup below).  The route's control flow depends on the
// block (dbdsqr's iteration counts, dlartg / dlasv2 branches), so lanes of one wave running
// different blocks serialise each other's paths: a wave with ONE active lane runs a block
// 1.7-2x sooner than a full one (profiles/r02m_ab_fixt_*), but only ~2k such waves fit the
// chip (the route needs ~250 VGPRs: 2 waves per SIMD).  So the first kLead listed blocks go
// to single-lane waves -- all of them in the common, sparse case -- and the rest, if any, to
// waves of kFixT<B> lanes on a second stream at the same time.
#ifndef TMF_FIX_THREADS
#define TMF_FIX_THREADS 64
#endif
template <int B>
constexpr int kFixT = (48 * 1024) / (8 * kFixSlot<B>) < TMF_FIX_THREADS ? (48 * 1024) / (8 * kFixSlot<B>) : TMF_FIX_THREADS;
constexpr uint32_t kLead = 2048;

struct FixSlot {
    double *ws;
    float *D, *U, *Vt, *S;
};
template <int B>
TMF_DEVI FixSlot fix_slot(double *lds)
{
    FixSlot f;
    f.ws = lds + threadIdx.x * kFixSlot<B>;
    f.D = reinterpret_cast<float *>(f.ws + lp::ws_doubles(B));
    f.U = f.D + B * B;
    f.Vt = f.U + B * B;
    f.S = f.Vt + B * B;
    return f;
}

template <int B, int T>
__global__ __launch_bounds__(64) void embed_fixup_kernel(EmbedArgs a, const uint32_t *__restrict__ list, const uint32_t *__restrict__ count,
                                                         uint32_t lo, uint32_t hi)
{
    extern __shared__ double fix_lds[];
    const FixSlot f = fix_slot<B>(fix_lds);
    const uint32_t n = *count < hi ? *count : hi;
    const uint32_t per_frame = (uint32_t)a.nbh * (uint32_t)a.nbw;
    for (uint32_t t = lo + blockIdx.x * T + threadIdx.x; t < n; t += gridDim.x * T) {
        const uint32_t id = list[t];
        const int64_t fr = id / per_frame;
        const uint32_t rem = id % per_frame;
        const int bi = (int)(rem / (uint32_t)a.nbw), bj = (int)(rem % (uint32_t)a.nbw);
        const uint8_t *src = a.src + fr * a.frame_stride;
        uint8_t *dst = a.dst + fr * a.frame_stride;
        float x[B][B];
        load_dct_block<B>(src, a.W, bi, bj, x);
#pragma unroll
        for (int i = 0; i < B; ++i)
#pragma unroll
            for (int j = 0; j < B; ++j) f.D[i * B + j] = x[i][j];
        lp::svd_f32_ws<true>(f.D, runtime_n(B), f.U, f.S, f.Vt, f.ws);  // :195
        // :198 blend, :201 U @ (diag(S) @ Vt) as OpenBLAS sgemm's fma chain over k
        const double w = (double)a.wm[(int64_t)bi * a.nbw + bj];
        f.S[0] = (float)((double)f.S[0] + a.alpha * (w / 255.0));
#pragma unroll
        for (int i = 0; i < B; ++i)
#pragma unroll
            for (int j = 0; j < B; ++j) {
                float acc = 0.0f;
#pragma unroll
                for (int k = 0; k < B; ++k) acc = __builtin_fmaf(f.U[i * B + k], f.S[k] * f.Vt[k * B + j], acc);
                x[i][j] = acc;
            }
        // :204 IDCT, axis 0 then axis 1
#pragma unroll
        for (int c = 0; c < B; ++c) {
            float col[B];
#pragma unroll
            for (int r = 0; r < B; ++r) col[r] = x[r][c];
            dct::dct3<B>(col);
#pragma unroll
            for (int r = 0; r < B; ++r) x[r][c] = col[r];
        }
#pragma unroll
        for (int r = 0; r < B; ++r) dct::dct3<B>(x[r]);
        // :207-216 write back with the pixel's own chroma, inverse colour
#pragma unroll
        for (int r = 0; r < B; ++r)
#pragma unroll
            for (int c = 0; c < B; ++c) {
                const int64_t off = ((int64_t)(bi * B + r) * a.W + (int64_t)bj * B + c) * 3;
                float cbs, crs;
                chroma(src[off], src[off + 1], src[off + 2], cbs, crs);
                uint32_t R8, G8, B8;
                colour_inv(x[r][c], cbs, crs, R8, G8, B8);
                dst[off] = (uint8_t)R8;
                dst[off + 1] = (uint8_t)G8;
                dst[off + 2] = (uint8_t)B8;
            }
    }
}

template <int B, int T>
__global__ __launch_bounds__(64) void extract_fixup_kernel(ExtractArgs a, const uint32_t *__restrict__ list,
                                                           const uint32_t *__restrict__ count, uint32_t lo, uint32_t hi)
{
    extern __shared__ double fix_lds[];
    const FixSlot f = fix_slot<B>(fix_lds);
    const uint32_t n = *count < hi ? *count : hi;
    const uint32_t per_frame = (uint32_t)a.nbh * (uint32_t)a.nbw;
    for (uint32_t t = lo + blockIdx.x * T + threadIdx.x; t < n; t += gridDim.x * T) {
        const uint32_t id = list[t];
        const int64_t fr = id / per_frame;
        const uint32_t rem = id % per_frame;
        const int bi = (int)(rem / (uint32_t)a.nbw), bj = (int)(rem % (uint32_t)a.nbw);
        float sig[2];
        for (int img = 0; img < 2; ++img) {
            float x[B][B];
            load_dct_block<B>((img == 0 ? a.wsrc : a.osrc) + fr * a.frame_stride, a.W, bi, bj, x);
#pragma unroll
            for (int i = 0; i < B; ++i)
#pragma unroll
                for (int j = 0; j < B; ++j) f.D[i * B + j] = x[i][j];
            lp::svd_f32_ws<false>(f.D, runtime_n(B), nullptr, f.S, nullptr, f.ws);  // :279-282, S only
            sig[img] = f.S[0];
        }
        // :285-289 (numpy-2 NEP 50): f32 difference / f32(alpha); clip and *255 in f64; truncate
        const float e = (sig[0] - sig[1]) / a.alpha32;
        double d = (double)e;
        d = d < 0.0 ? 0.0 : d;
        d = d > 1.0 ? 1.0 : d;
        a.out[fr * a.tile_stride + (int64_t)bi * a.nbw + bj] = (uint8_t)(uint32_t)(d * 255.0);
    }
}

// ---------------------------------------------------------------------------
// launchers: grids are sized for the worst case (every block listed) but capped; threads
// beyond the device-side count exit at once
// ---------------------------------------------------------------------------
inline unsigned fixup_grid(int64_t entries, int threads)
{
    const int64_t g = (entries + threads - 1) / threads;
    return (unsigned)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

// one auxiliary stream per device for the bulk launch (created once, kept)
hipStream_t aux_stream();  // tmfwm_fallback.hip


// lead launch on st for entries [0, kLead); if the list can be longer, the bulk launch for
// [kLead, count) on the auxiliary stream, forked from and joined back into st
bool fixup_lead_disabled();  // TMFWM_DEBUG_NO_LEAD (tmfwm_fallback.hip): every entry to the bulk launch

template <typename Lead, typename Bulk>
inline hipError_t launch_fixup(int64_t max_entries, hipStream_t st, Lead lead, Bulk bulk)
{
    if (fixup_lead_disabled()) {
        bulk(st, 0u);
        return hipGetLastError();
    }
    if (max_entries <= (int64_t)kLead) {
        lead(st);
        return hipGetLastError();
    }
    hipStream_t aux = aux_stream();
    hipEvent_t fork = nullptr, join = nullptr;
    hipError_t e = aux ? hipEventCreateWithFlags(&fork, hipEventDisableTiming) : hipErrorInvalidResourceHandle;
    if (e == hipSuccess) e = hipEventCreateWithFlags(&join, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(fork, st);
    if (e == hipSuccess) e = hipStreamWaitEvent(aux, fork, 0);
    if (e == hipSuccess) {
        bulk(aux, kLead);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipEventRecord(join, aux);
    if (e == hipSuccess) {
        lead(st);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipStreamWaitEvent(st, join, 0);
    if (fork) (void)hipEventDestroy(fork);
    if (join) (void)hipEventDestroy(join);
    return e;
}

template <int B>
inline hipError_t embed_fixup_b(const EmbedArgs &a, const uint32_t *list, const uint32_t *count, int64_t max_entries, hipStream_t st)
{
    constexpr int T = kFixT<B>;
    return launch_fixup(
        max_entries, st,
        [&](hipStream_t s) {
            hipLaunchKernelGGL((embed_fixup_kernel<B, 1>), dim3(fixup_grid(max_entries < kLead ? max_entries : kLead, 1)), dim3(1),
                               kFixSlot<B> * 8, s, a, list, count, 0u, kLead);
        },
        [&](hipStream_t s, uint32_t lo) {
            hipLaunchKernelGGL((embed_fixup_kernel<B, T>), dim3(fixup_grid(max_entries - lo, T)), dim3(T), (size_t)T * kFixSlot<B> * 8, s,
                               a, list, count, lo, 0xFFFFFFFFu);
        });
}

template <int B>
inline hipError_t extract_fixup_b(const ExtractArgs &a, const uint32_t *list, const uint32_t *count, int64_t max_entries, hipStream_t st)
{
    constexpr int T = kFixT<B>;
    return launch_fixup(
        max_entries, st,
        [&](hipStream_t s) {
            hipLaunchKernelGGL((extract_fixup_kernel<B, 1>), dim3(fixup_grid(max_entries < kLead ? max_entries : kLead, 1)), dim3(1),
                               kFixSlot<B> * 8, s, a, list, count, 0u, kLead);
        },
        [&](hipStream_t s, uint32_t lo) {
            hipLaunchKernelGGL((extract_fixup_kernel<B, T>), dim3(fixup_grid(max_entries - lo, T)), dim3(T), (size_t)T * kFixSlot<B> * 8,
                               s, a, list, count, lo, 0xFFFFFFFFu);
        });
}

}  // namespace tmf
