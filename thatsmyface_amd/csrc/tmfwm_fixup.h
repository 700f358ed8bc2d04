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
// byte.
//
// A group of G = 8 (b <= 8) or 16 lanes per listed block, 64 / G blocks per wave, each group's
// working set in LDS: the pixel, colour and transform work is spread over the group's lanes
// (a pixel, a DCT row or column, an element of the reconstruction per lane), and the dgesdd
// route runs under lp::GroupPar<G> (its matrix loops over the group's lanes, its scalar
// recurrences on the group's lanes alike).  A grid-stride loop over the device-side count: no
// host round trip sits between the passes.  (Until round 4 one 64-lane wave took one block,
// lp::WavePar; with every block of the reference route coming here, the scalar recurrences
// left the SIMDs idle -- DESIGN.md 3.5.)
// dbdsqr's non-convergence (np.linalg.svd raises LinAlgError there) is counted in *fb_bad.
#pragma once
#include "tmfwm_device.h"
#include "tmfwm_internal.h"
#include "tmfwm_lapack.h"

namespace tmf {

// The block size reaches the dgesdd routines as a run-time value, so that the compiler keeps
// the LAPACK loops as loops instead of unrolling the whole route per block size.  This is not
// a fault workaround: the workspace indexing stays inside ws_doubles(n) for
// n = 1..16 under AddressSanitizer (tests/native/lp_asan.cpp, exact-size allocations), and a
// build with the constant B passes the GPU's dgesdd-route and b = 16 tests
// (profiles/r03/r03u/constn_tests.log); the round-2 b = 16 fault was in the serial,
// scratch-array form of the route that round 3 replaced.
TMF_DEVI int runtime_n(int n)
{
    asm volatile("" : "+v"(n));
    return n;
}

// Lanes per listed block (lp::GroupPar<G>): 64 / G blocks per wave.  Round 4: the reference
// route (TMFWM_ROUTE_REFERENCE) sends every block here, so the pass is a throughput path, not
// a few stragglers' latency: one block per wave left the SIMDs idle on the route's scalar
// recurrences.
template <int B>
constexpr int kFixLanes = B <= 8 ? 8 : 16;

// a group's lanes see each other's LDS writes in program order (one wave): only the compiler
// must not move LDS accesses across the phase boundaries
TMF_DEVI void group_sync() { asm volatile("" ::: "memory"); }

// this block's luma, then its 2-D DCT (axis 0, then axis 1: watermarking.py:192, :279-282),
// into t[B*B] (row-major) -- the group's lanes take pixels, then columns, then rows
template <int B, int G>
TMF_DEVI void fix_load_dct(const uint8_t *frame, int W, int bi, int bj, float *t, int gl)
{
    for (int k = gl; k < B * B; k += G) {
        const uint8_t *p = frame + ((int64_t)(bi * B + k / B) * W + (int64_t)bj * B + k % B) * 3;
        t[k] = luma(p[0], p[1], p[2]);
    }
    group_sync();
    for (int c = gl; c < B; c += G) {
        float col[B];
#pragma unroll
        for (int r = 0; r < B; ++r) col[r] = t[r * B + c];
        dct::dct2<B>(col);
#pragma unroll
        for (int r = 0; r < B; ++r) t[r * B + c] = col[r];
    }
    group_sync();
    for (int r = gl; r < B; r += G) {
        float row[B];
#pragma unroll
        for (int c = 0; c < B; ++c) row[c] = t[r * B + c];
        dct::dct2<B>(row);
#pragma unroll
        for (int c = 0; c < B; ++c) t[r * B + c] = row[c];
    }
    group_sync();
}

// one group's LDS: the route's workspace (embed: its U and VT, f64 column-major at ws + B^2 and
// ws + 2 B^2, are read in place by the reconstruction; extract: S only, no U and VT -- 1.4 KB
// instead of 2.4 KB per b = 8 group, so LDS no longer caps the extract pass at 2 waves / SIMD),
// the DCT block D -- dead once the route has copied it, so the reconstruction M reuses it -- and S
template <int B, bool WANT_V>
struct FixLdsT {
    double ws[lp::ws_doubles_for<WANT_V>(B)];
    float D[B * B], S[B];
};
template <int B>
using FixLdsS = FixLdsT<B, false>;
// embed above b = 8: the compact workspace (lp::ws_doubles_compact: no work slot) with the DCT
// block D waiting in the U slot (the route copies it into A before anything else writes there),
// the reconstruction M in the A slot (dead after apply_pt) and S in the e slot (e is in
// registers by then): 8.4 -> 6.5 KB per b = 16 group, six waves per CU where four fitted
// (embed<16> -24 %, <12> -6 %, <8> -3 %; b = 6 +-0.5 % keeps the standard layout,
// profiles/r04/r04n/, r04o/)
template <int B>
constexpr bool kFixAlias = B >= 8;
template <int B, bool ALIAS = kFixAlias<B>>
struct FixLds {
    static constexpr bool kCompact = false;
    double ws[lp::ws_doubles(B)];
    float Dm[B * B], Sv[B];
    TMF_DEVI float *D() { return Dm; }
    TMF_DEVI float *M() { return Dm; }
    TMF_DEVI float *S() { return Sv; }
};
template <int B>
struct FixLds<B, true> {
    static constexpr bool kCompact = true;
    double ws[lp::ws_doubles_compact(B)];
    TMF_DEVI float *D() { return reinterpret_cast<float *>(ws + B * B); }
    TMF_DEVI float *M() { return reinterpret_cast<float *>(ws); }
    TMF_DEVI float *S() { return reinterpret_cast<float *>(ws + 3 * B * B + B); }
};

TMF_DEVI void block_of(uint32_t id, uint32_t per_frame, int nbw, int64_t &fr, int &bi, int &bj)
{
    fr = id / per_frame;
    const uint32_t rem = id % per_frame;
    bi = (int)(rem / (uint32_t)nbw);
    bj = (int)(rem % (uint32_t)nbw);
}

// One listed block end to end on the dgesdd route, by G lanes (gl = this lane's index among
// them) under lane policy Par: a group of a GroupPar wave, or a whole wave (WavePar, G = 64).
template <int B, class Par, int G>
TMF_DEVI void embed_fix_block(const EmbedArgs &a, uint32_t id, FixLds<B> &f, int gl)
{
    const uint32_t per_frame = (uint32_t)a.nbh * (uint32_t)a.nbw;
    int64_t fr;
    int bi, bj;
    block_of(id, per_frame, a.nbw, fr, bi, bj);
    const uint8_t *src = a.src + fr * a.frame_stride;
    uint8_t *dst = a.dst + fr * a.frame_stride;
    fix_load_dct<B, G>(src, a.W, bi, bj, f.D(), gl);
    float *S = f.S();
    const int info = lp::svd_f32_ws<true, Par, FixLds<B>::kCompact>(f.D(), runtime_n(B), nullptr, S, nullptr, f.ws);  // :195
    if (info && gl == 0 && a.fb_bad) atomicAdd(a.fb_bad, 1u);
    // :198 blend, :201 U @ (diag(S) @ Vt) as OpenBLAS sgemm's fma chain over k, on U and Vt
    // rounded to f32 (numpy's astype) from the route's f64 U and VT
    const double *U64 = f.ws + B * B, *VT64 = f.ws + 2 * B * B;
    float *M = f.M();
    const double w = (double)a.wm[(int64_t)bi * a.nbw + bj];
    const float s0 = (float)((double)S[0] + a.alpha * (w / 255.0));
    for (int e = gl; e < B * B; e += G) {
        const int i = e / B, j = e % B;
        float acc = 0.0f;
#pragma unroll
        for (int k = 0; k < B; ++k)
            acc = __builtin_fmaf((float)U64[i + k * B], (k == 0 ? s0 : S[k]) * (float)VT64[k + j * B], acc);
        M[e] = acc;
    }
    group_sync();
    // :204 IDCT, axis 0 then axis 1
    for (int c = gl; c < B; c += G) {
        float col[B];
#pragma unroll
        for (int r = 0; r < B; ++r) col[r] = M[r * B + c];
        dct::dct3<B>(col);
#pragma unroll
        for (int r = 0; r < B; ++r) M[r * B + c] = col[r];
    }
    group_sync();
    for (int r = gl; r < B; r += G) {
        float row[B];
#pragma unroll
        for (int c = 0; c < B; ++c) row[c] = M[r * B + c];
        dct::dct3<B>(row);
#pragma unroll
        for (int c = 0; c < B; ++c) M[r * B + c] = row[c];
    }
    group_sync();
    // :207-216 write back with the pixel's own chroma, inverse colour
    for (int k = gl; k < B * B; k += G) {
        const int64_t off = ((int64_t)(bi * B + k / B) * a.W + (int64_t)bj * B + k % B) * 3;
        float cbs, crs;
        chroma(src[off], src[off + 1], src[off + 2], cbs, crs);
        uint32_t R8, G8, B8;
        colour_inv(M[k], cbs, crs, R8, G8, B8);
        dst[off] = (uint8_t)R8;
        dst[off + 1] = (uint8_t)G8;
        dst[off + 2] = (uint8_t)B8;
    }
    group_sync();  // the LDS slots are reused by the next listed block
}

template <int B, class Par, int G>
TMF_DEVI void extract_fix_block(const ExtractArgs &a, uint32_t id, FixLdsS<B> &f, int gl)
{
    const uint32_t per_frame = (uint32_t)a.nbh * (uint32_t)a.nbw;
    int64_t fr;
    int bi, bj;
    block_of(id, per_frame, a.nbw, fr, bi, bj);
    float sig[2];
    for (int img = 0; img < 2; ++img) {
        fix_load_dct<B, G>((img == 0 ? a.wsrc : a.osrc) + fr * a.frame_stride, a.W, bi, bj, f.D, gl);
        const int info = lp::svd_f32_ws<false, Par>(f.D, runtime_n(B), nullptr, f.S, nullptr, f.ws);  // :279-282
        if (info && gl == 0 && a.fb_bad) atomicAdd(a.fb_bad, 1u);
        sig[img] = f.S[0];
        group_sync();
    }
    // :285-289 (numpy-2 NEP 50): f32 difference / f32(alpha); clip and *255 in f64; truncate
    if (gl == 0) {
        const float e = (sig[0] - sig[1]) / a.alpha32;
        double d = (double)e;
        d = d < 0.0 ? 0.0 : d;
        d = d > 1.0 ? 1.0 : d;
        a.out[fr * a.tile_stride + (int64_t)bi * a.nbw + bj] = (uint8_t)(uint32_t)(d * 255.0);
    }
}

// A short list (the hybrid route's few flagged blocks: no more than the grid's workgroups) takes
// a whole wave per block -- the lowest latency per block, and the pass is one block's latency;
// a long one (the reference route: every block) takes 64 / G blocks per wave for throughput.
// The choice is uniform over the grid (the device-side count against the grid size).
template <int B>
__global__ __launch_bounds__(64) void embed_fixup_kernel(EmbedArgs a, const uint32_t *__restrict__ list, const uint32_t *__restrict__ count)
{
    constexpr int G = kFixLanes<B>, NG = 64 / G;
    static_assert(G >= B, "a group holds one element of dbdsqr's vectors per lane");
    __shared__ FixLds<B> fl[NG];
    const uint32_t n = *count;
    if (n <= gridDim.x) {
        if (blockIdx.x < n) embed_fix_block<B, lp::WavePar, 64>(a, list[blockIdx.x], fl[0], (int)threadIdx.x);
        return;
    }
    const int gl = lp::GroupPar<G>::lane(), grp = (int)(threadIdx.x / G);
    for (uint32_t t0 = blockIdx.x * NG; t0 < n; t0 += gridDim.x * NG) {
        const uint32_t t = t0 + (uint32_t)grp;
        if (t < n) embed_fix_block<B, lp::GroupPar<G>, G>(a, list[t], fl[grp], gl);  // else: no block this round
    }
}

template <int B>
__global__ __launch_bounds__(64) void extract_fixup_kernel(ExtractArgs a, const uint32_t *__restrict__ list,
                                                           const uint32_t *__restrict__ count)
{
    constexpr int G = kFixLanes<B>, NG = 64 / G;
    static_assert(G >= B, "a group holds one element of dbdsqr's vectors per lane");
    __shared__ FixLdsS<B> fl[NG];
    const uint32_t n = *count;
    if (n <= gridDim.x) {
        if (blockIdx.x < n) extract_fix_block<B, lp::WavePar, 64>(a, list[blockIdx.x], fl[0], (int)threadIdx.x);
        return;
    }
    const int gl = lp::GroupPar<G>::lane(), grp = (int)(threadIdx.x / G);
    for (uint32_t t0 = blockIdx.x * NG; t0 < n; t0 += gridDim.x * NG) {
        const uint32_t t = t0 + (uint32_t)grp;
        if (t < n) extract_fix_block<B, lp::GroupPar<G>, G>(a, list[t], fl[grp], gl);
    }
}

// ---------------------------------------------------------------------------
// launchers: the grid is sized for the listed blocks the chip holds at once (capped by the
// possible list length); workgroups past the device-side count exit at once, the others
// stride over it
// ---------------------------------------------------------------------------
template <int B>
inline unsigned fixup_grid(int64_t entries)
{
    const int64_t waves = (entries + 64 / kFixLanes<B> - 1) / (64 / kFixLanes<B>);
    return (unsigned)(waves < 1 ? 1 : (waves > 8192 ? 8192 : waves));
}

template <int B>
inline hipError_t embed_fixup_b(const EmbedArgs &a, const uint32_t *list, const uint32_t *count, int64_t max_entries, hipStream_t st)
{
    hipLaunchKernelGGL((embed_fixup_kernel<B>), dim3(fixup_grid<B>(max_entries)), dim3(64), 0, st, a, list, count);
    return hipGetLastError();
}

template <int B>
inline hipError_t extract_fixup_b(const ExtractArgs &a, const uint32_t *list, const uint32_t *count, int64_t max_entries, hipStream_t st)
{
    hipLaunchKernelGGL((extract_fixup_kernel<B>), dim3(fixup_grid<B>(max_entries)), dim3(64), 0, st, a, list, count);
    return hipGetLastError();
}

}  // namespace tmf
