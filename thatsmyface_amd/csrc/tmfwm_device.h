// Device-side arithmetic of the watermark path for gfx950 (MI355X).
//
// Every function here reproduces one step of the reference numerics
// (/root/reference/modules/watermarking.py) at the bit level; the contract is
// SURVEY.md 8(a) N1-N10 and DESIGN.md section 3.  The TU is compiled with
// -ffp-contract=off: every '*', '+', '-' below is one IEEE operation and fused
// multiply-adds appear only where written (__builtin_fma / __builtin_fmaf).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>
#include <utility>

#include "tmfwm_consts.h"

#define TMF_DEVI __device__ __forceinline__

namespace tmf {

// ---------------------------------------------------------------------------
// Colour (N1, N2, N9)
// ---------------------------------------------------------------------------

// f32(v) / 255.0f, correctly rounded (watermarking.py:29), as fma(x, H, x * Lo) with
// 1/255 = H + Lo split into two floats: x*H is exact inside the fma and x*Lo's rounding is
// ~2^-48 relative, far below the distance of any v/255 from an f32 rounding boundary --
// exhaustively equal to the IEEE divide for v = 0..255 (tests/test_host_api.py).  Two
// operations instead of a multiply and a two-fma residual correction.
constexpr float kUnitHi = 0.003921568859368562698f;    // f32(1/255)
constexpr float kUnitLo = -2.3191758e-10f;             // f32(1/255 - kUnitHi)
TMF_DEVI float unit_from_u8(uint32_t v)
{
    const float x = (float)v;
    return __builtin_fmaf(x, kUnitHi, x * kUnitLo);
}

// Y only (watermarking.py:37-45, row 0 of the transform; OpenBLAS dgemv FMA pattern)
TMF_DEVI float luma(uint32_t R, uint32_t G, uint32_t B)
{
    const double r = unit_from_u8(R), g = unit_from_u8(G), b = unit_from_u8(B);
    return (float)__builtin_fma(0.114, b, __builtin_fma(0.299, r, 0.587 * g));
}

// Cb, Cr as stored by rgb_to_ycbcr (f32 of the f64 dot, then "+= 0.5" in f32, :48)
TMF_DEVI void chroma(uint32_t R, uint32_t G, uint32_t B, float &cbs, float &crs)
{
    const double r = unit_from_u8(R), g = unit_from_u8(G), b = unit_from_u8(B);
    cbs = (float)__builtin_fma(0.5, b, __builtin_fma(-0.169, r, -0.331 * g)) + 0.5f;
    crs = (float)__builtin_fma(-0.081, b, __builtin_fma(0.5, r, -0.419 * g)) + 0.5f;
}

// np.clip(.,0,1) in f32, * 255 in f32, astype(uint8) = truncation (watermarking.py:70-73).
// The clip is one v_med3_f32; it differs from np.clip only in the sign of a zero
// result (and on NaN, which no finite pixel produces), and -0 * 255 truncates to 0 too.
TMF_DEVI uint32_t u8_from_unit(float f)
{
    f = __builtin_amdgcn_fmed3f(f, 0.0f, 1.0f);
    return (uint32_t)(f * 255.0f);
}

// ycbcr_to_rgb for one pixel (watermarking.py:55-73): Cb, Cr -= 0.5 in f32, then the
// dgemv pattern fma(Ti[c][2], cr, fma(Ti[c][0], y, Ti[c][1]*cb)) in f64.  Two terms
// of it are exact no-ops and are dropped: with Ti[0][1] = 0, fma(1, y, 0*cb) is y up
// to the sign of a zero, and with Ti[2][2] = 0, fma(0, cr, t) is t up to the sign of
// a zero; a zero of either sign leaves u8_from_unit at 0, so the bytes are the same
// for every input (checked over all 2^24 colours by the GPU colour-table test).
TMF_DEVI void colour_inv(float y, float cbs, float crs, uint32_t &R, uint32_t &G, uint32_t &B)
{
    const double Y = y, CB = cbs - 0.5f, CR = crs - 0.5f;
    R = u8_from_unit((float)__builtin_fma(1.403, CR, Y));
    G = u8_from_unit((float)__builtin_fma(-0.714, CR, Y + -0.344 * CB));
    B = u8_from_unit((float)(Y + 1.773 * CB));
}

// colour_inv that also returns the largest fractional part of the three scaled channel
// values p = f32(clip(v) * 255) whose truncation gives the bytes: the byte certificate's
// test of a Y interval (blocks.h embed_blocks)
TMF_DEVI void colour_inv_frac(float y, float cbs, float crs, uint32_t &R, uint32_t &G, uint32_t &B, float &fr)
{
    const double Y = y, CB = cbs - 0.5f, CR = crs - 0.5f;
    const float pr = __builtin_amdgcn_fmed3f((float)__builtin_fma(1.403, CR, Y), 0.0f, 1.0f) * 255.0f;
    const float pg = __builtin_amdgcn_fmed3f((float)__builtin_fma(-0.714, CR, Y + -0.344 * CB), 0.0f, 1.0f) * 255.0f;
    const float pb = __builtin_amdgcn_fmed3f((float)(Y + 1.773 * CB), 0.0f, 1.0f) * 255.0f;
    R = (uint32_t)pr;
    G = (uint32_t)pg;
    B = (uint32_t)pb;
    fr = __builtin_fmaxf(__builtin_amdgcn_fractf(pr), __builtin_fmaxf(__builtin_amdgcn_fractf(pg), __builtin_amdgcn_fractf(pb)));
}

// ---------------------------------------------------------------------------
// The module-level helpers on non-uint8 inputs (the frame kernels above only ever
// see uint8 pixels).  rgb_to_ycbcr casts any numeric array with np.array(img,
// float32) (:29; the caller's cast) and divides by 255 in f32; ycbcr_to_rgb runs
// in the input's own float type T (:55 img.copy(), :58 "-= 0.5" in T, :64 zeros_like
// -> the f64 dot is stored in T, :70-73 clip, * 255 in T, truncation).
// ---------------------------------------------------------------------------

// :29-48 for f32 pixel values v (0..255 scale): v / 255.0f is the IEEE divide (the
// TU keeps HIP's correctly rounded f32 division: no fast-math), then the dgemv rows.
TMF_DEVI void colour_fwd_f32(float R, float G, float B, float &y, float &cbs, float &crs)
{
    const double r = R / 255.0f, g = G / 255.0f, b = B / 255.0f;
    y = (float)__builtin_fma(0.114, b, __builtin_fma(0.299, r, 0.587 * g));
    cbs = (float)__builtin_fma(0.5, b, __builtin_fma(-0.169, r, -0.331 * g)) + 0.5f;
    crs = (float)__builtin_fma(-0.081, b, __builtin_fma(0.5, r, -0.419 * g)) + 0.5f;
}

// f64 -> f16 with one rounding (numpy's npy_double_to_half): round to odd into f32
// (24 >= 11 + 2 bits, so the following RNE f32 -> f16 conversion rounds as a direct
// f64 -> f16 conversion would), then v_cvt_f16_f32.
TMF_DEVI _Float16 f16_from_f64(double d)
{
    float t = (float)d;
    if ((double)t != d) {
        uint32_t u = __float_as_uint(t);
        if (__builtin_fabs((double)t) > __builtin_fabs(d)) u -= 1; // rounded away from zero: step back
        t = __uint_as_float(u | 1u);
    }
    return (_Float16)t;
}

template <typename T> TMF_DEVI T round_to(double d)
{
    if constexpr (std::is_same_v<T, _Float16>) return f16_from_f64(d);
    else return (T)d;
}

// :70-73 in T: np.clip(., 0, 1), * 255 (one T multiply; f16 products are correctly
// rounded like numpy's half arithmetic), astype(uint8) truncation.  A NaN pixel (only
// reachable from a NaN / inf input) has no defined uint8 in the reference either.
template <typename T> TMF_DEVI uint32_t u8_from_unit_t(T f)
{
    f = f < T(0) ? T(0) : f;
    f = f > T(1) ? T(1) : f;
    const T p = f * T(255);
    if constexpr (std::is_same_v<T, double>) return (uint32_t)p;  // truncate the double itself
    else return (uint32_t)(float)p;                               // a half converts to f32 exactly
}

// :55-73 for one pixel of a T-typed array.  The dropped dgemv terms are the exact
// no-ops of colour_inv (zero products whose sign the clip removes).
template <typename T> TMF_DEVI void colour_inv_t(T y, T cbs, T crs, uint32_t &R, uint32_t &G, uint32_t &B)
{
    if constexpr (std::is_same_v<T, float>) {
        colour_inv(y, cbs, crs, R, G, B);
    } else {
        const double Y = (double)y, CB = (double)(T)(cbs - T(0.5)), CR = (double)(T)(crs - T(0.5));
        R = u8_from_unit_t<T>(round_to<T>(__builtin_fma(1.403, CR, Y)));
        G = u8_from_unit_t<T>(round_to<T>(__builtin_fma(-0.714, CR, Y + -0.344 * CB)));
        B = u8_from_unit_t<T>(round_to<T>(Y + 1.773 * CB));
    }
}

// ---------------------------------------------------------------------------
// pocketfft fp32 DCT-II / DCT-III (N3), every even length 4..16, fully unrolled on
// register arrays.  rfftp radix passes with compile-time (ido, l1).
// ---------------------------------------------------------------------------
// Interval of f32 values [lo, hi] for the hybrid route's byte certificate:
// every operation below is the IEEE round-to-nearest operation on the end points, which is
// monotone in each operand, so the result encloses every value the operation can produce
// from operands inside the intervals (ends swapped by subtraction and negative constants).
struct Ivf {
    float lo, hi;
};
TMF_DEVI Ivf operator+(Ivf a, Ivf b) { return {a.lo + b.lo, a.hi + b.hi}; }
TMF_DEVI Ivf operator-(Ivf a, Ivf b) { return {a.lo - b.hi, a.hi - b.lo}; }
TMF_DEVI Ivf operator-(Ivf a) { return {-a.hi, -a.lo}; }
TMF_DEVI Ivf operator*(float c, Ivf a) { return c >= 0.0f ? Ivf{c * a.lo, c * a.hi} : Ivf{c * a.hi, c * a.lo}; }
TMF_DEVI Ivf operator*(Ivf a, float c) { return c * a; }
TMF_DEVI Ivf &operator*=(Ivf &a, float c) { return a = c * a; }

namespace dct {

constexpr float kSqrt2 = 1.41421356237309504880f;
constexpr float kHsqt2 = 0.70710678118654752440f;

template <int IDO, int L1, int N>
TMF_DEVI void radb2(const float (&cc)[N], float (&ch)[N], const float *wa)
{
#define CC(a, b, c) cc[(a) + IDO * ((b) + 2 * (c))]
#define CH(a, b, c) ch[(a) + IDO * ((b) + L1 * (c))]
#pragma unroll
    for (int k = 0; k < L1; k++) {
        const float x = CC(0, 0, k), y = CC(IDO - 1, 1, k);
        CH(0, k, 0) = x + y;
        CH(0, k, 1) = x - y;
    }
    if constexpr ((IDO & 1) == 0) {
#pragma unroll
        for (int k = 0; k < L1; k++) {
            CH(IDO - 1, k, 0) = 2.0f * CC(IDO - 1, 0, k);
            CH(IDO - 1, k, 1) = -2.0f * CC(0, 1, k);
        }
    }
    if constexpr (IDO > 2) {
#pragma unroll
        for (int k = 0; k < L1; ++k)
#pragma unroll
            for (int i = 2; i < IDO; i += 2) {
                const int ic = IDO - i;
                const float a = CC(i - 1, 0, k), b = CC(ic - 1, 1, k);
                CH(i - 1, k, 0) = a + b;
                const float tr2 = a - b;
                const float c = CC(i, 0, k), d = CC(ic, 1, k);
                const float ti2 = c + d;
                CH(i, k, 0) = c - d;
                const float w0 = wa[i - 2], w1 = wa[i - 1];
                CH(i, k, 1) = w0 * ti2 + w1 * tr2;
                CH(i - 1, k, 1) = w0 * tr2 - w1 * ti2;
            }
    }
#undef CC
#undef CH
}

template <int IDO, int L1, int N>
TMF_DEVI void radb4(const float (&cc)[N], float (&ch)[N], const float *wa)
{
#define CC(a, b, c) cc[(a) + IDO * ((b) + 4 * (c))]
#define CH(a, b, c) ch[(a) + IDO * ((b) + L1 * (c))]
#pragma unroll
    for (int k = 0; k < L1; k++) {
        const float x = CC(0, 0, k), y = CC(IDO - 1, 3, k);
        const float tr2 = x + y, tr1 = x - y;
        const float tr3 = 2.0f * CC(IDO - 1, 1, k);
        const float tr4 = 2.0f * CC(0, 2, k);
        CH(0, k, 0) = tr2 + tr3;
        CH(0, k, 2) = tr2 - tr3;
        CH(0, k, 3) = tr1 + tr4;
        CH(0, k, 1) = tr1 - tr4;
    }
    if constexpr ((IDO & 1) == 0) {
#pragma unroll
        for (int k = 0; k < L1; k++) {
            const float a = CC(0, 3, k), b = CC(0, 1, k);
            const float ti1 = a + b, ti2 = a - b;
            const float c = CC(IDO - 1, 0, k), d = CC(IDO - 1, 2, k);
            const float tr2 = c + d, tr1 = c - d;
            CH(IDO - 1, k, 0) = tr2 + tr2;
            CH(IDO - 1, k, 1) = kSqrt2 * (tr1 - ti1);
            CH(IDO - 1, k, 2) = ti2 + ti2;
            CH(IDO - 1, k, 3) = -kSqrt2 * (tr1 + ti1);
        }
    }
    if constexpr (IDO > 2) {
#pragma unroll
        for (int k = 0; k < L1; ++k)
#pragma unroll
            for (int i = 2; i < IDO; i += 2) {
                const int ic = IDO - i;
                float a, b;
                a = CC(i - 1, 0, k); b = CC(ic - 1, 3, k);
                const float tr2 = a + b, tr1 = a - b;
                a = CC(i, 0, k); b = CC(ic, 3, k);
                const float ti1 = a + b, ti2 = a - b;
                a = CC(i, 2, k); b = CC(ic, 1, k);
                const float tr4 = a + b, ti3 = a - b;
                a = CC(i - 1, 2, k); b = CC(ic - 1, 1, k);
                const float tr3 = a + b, ti4 = a - b;
                CH(i - 1, k, 0) = tr2 + tr3;
                const float cr3 = tr2 - tr3;
                CH(i, k, 0) = ti2 + ti3;
                const float ci3 = ti2 - ti3;
                const float cr4 = tr1 + tr4, cr2 = tr1 - tr4;
                const float ci2 = ti1 + ti4, ci4 = ti1 - ti4;
                float w0 = wa[i - 2], w1 = wa[i - 1];
                CH(i, k, 1) = w0 * ci2 + w1 * cr2;
                CH(i - 1, k, 1) = w0 * cr2 - w1 * ci2;
                w0 = wa[(IDO - 1) + i - 2]; w1 = wa[(IDO - 1) + i - 1];
                CH(i, k, 2) = w0 * ci3 + w1 * cr3;
                CH(i - 1, k, 2) = w0 * cr3 - w1 * ci3;
                w0 = wa[2 * (IDO - 1) + i - 2]; w1 = wa[2 * (IDO - 1) + i - 1];
                CH(i, k, 3) = w0 * ci4 + w1 * cr4;
                CH(i - 1, k, 3) = w0 * cr4 - w1 * ci4;
            }
    }
#undef CC
#undef CH
}

template <int IDO, int L1, int N, typename T>
TMF_DEVI void radf2(const T (&cc)[N], T (&ch)[N], const float *wa)
{
#define CC(a, b, c) cc[(a) + IDO * ((b) + L1 * (c))]
#define CH(a, b, c) ch[(a) + IDO * ((b) + 2 * (c))]
#pragma unroll
    for (int k = 0; k < L1; k++) {
        const T x = CC(0, k, 0), y = CC(0, k, 1);
        CH(0, 0, k) = x + y;
        CH(IDO - 1, 1, k) = x - y;
    }
    if constexpr ((IDO & 1) == 0) {
#pragma unroll
        for (int k = 0; k < L1; k++) {
            CH(0, 1, k) = -CC(IDO - 1, k, 1);
            CH(IDO - 1, 0, k) = CC(IDO - 1, k, 0);
        }
    }
    if constexpr (IDO > 2) {
#pragma unroll
        for (int k = 0; k < L1; k++)
#pragma unroll
            for (int i = 2; i < IDO; i += 2) {
                const int ic = IDO - i;
                const float w0 = wa[i - 2], w1 = wa[i - 1];
                const T e = CC(i - 1, k, 1), f = CC(i, k, 1);
                const T tr2 = w0 * e + w1 * f;
                const T ti2 = w0 * f - w1 * e;
                const T a = CC(i - 1, k, 0);
                CH(i - 1, 0, k) = a + tr2;
                CH(ic - 1, 1, k) = a - tr2;
                const T c = CC(i, k, 0);
                CH(i, 0, k) = ti2 + c;
                CH(ic, 1, k) = ti2 - c;
            }
    }
#undef CC
#undef CH
}

template <int IDO, int L1, int N, typename T>
TMF_DEVI void radf4(const T (&cc)[N], T (&ch)[N], const float *wa)
{
#define CC(a, b, c) cc[(a) + IDO * ((b) + L1 * (c))]
#define CH(a, b, c) ch[(a) + IDO * ((b) + 4 * (c))]
#pragma unroll
    for (int k = 0; k < L1; k++) {
        T a = CC(0, k, 3), b = CC(0, k, 1);
        const T tr1 = a + b;
        CH(0, 2, k) = a - b;
        a = CC(0, k, 0); b = CC(0, k, 2);
        const T tr2 = a + b;
        CH(IDO - 1, 1, k) = a - b;
        CH(0, 0, k) = tr2 + tr1;
        CH(IDO - 1, 3, k) = tr2 - tr1;
    }
    if constexpr ((IDO & 1) == 0) {
#pragma unroll
        for (int k = 0; k < L1; k++) {
            const T ti1 = -kHsqt2 * (CC(IDO - 1, k, 1) + CC(IDO - 1, k, 3));
            const T tr1 = kHsqt2 * (CC(IDO - 1, k, 1) - CC(IDO - 1, k, 3));
            const T a = CC(IDO - 1, k, 0);
            CH(IDO - 1, 0, k) = a + tr1;
            CH(IDO - 1, 2, k) = a - tr1;
            const T c = CC(IDO - 1, k, 2);
            CH(0, 3, k) = ti1 + c;
            CH(0, 1, k) = ti1 - c;
        }
    }
    if constexpr (IDO > 2) {
#pragma unroll
        for (int k = 0; k < L1; k++)
#pragma unroll
            for (int i = 2; i < IDO; i += 2) {
                const int ic = IDO - i;
                float w0 = wa[i - 2], w1 = wa[i - 1];
                T e = CC(i - 1, k, 1), f = CC(i, k, 1);
                const T cr2 = w0 * e + w1 * f, ci2 = w0 * f - w1 * e;
                w0 = wa[(IDO - 1) + i - 2]; w1 = wa[(IDO - 1) + i - 1];
                e = CC(i - 1, k, 2); f = CC(i, k, 2);
                const T cr3 = w0 * e + w1 * f, ci3 = w0 * f - w1 * e;
                w0 = wa[2 * (IDO - 1) + i - 2]; w1 = wa[2 * (IDO - 1) + i - 1];
                e = CC(i - 1, k, 3); f = CC(i, k, 3);
                const T cr4 = w0 * e + w1 * f, ci4 = w0 * f - w1 * e;
                const T tr1 = cr4 + cr2, tr4 = cr4 - cr2;
                const T ti1 = ci2 + ci4, ti4 = ci2 - ci4;
                const T a = CC(i - 1, k, 0), c = CC(i, k, 0);
                const T tr2 = a + cr3, tr3 = a - cr3;
                const T ti2 = c + ci3, ti3 = c - ci3;
                CH(i - 1, 0, k) = tr2 + tr1;
                CH(ic - 1, 3, k) = tr2 - tr1;
                CH(i, 0, k) = ti1 + ti2;
                CH(ic, 3, k) = ti1 - ti2;
                CH(i - 1, 2, k) = tr3 + ti4;
                CH(ic - 1, 1, k) = tr3 - ti4;
                CH(i, 2, k) = tr4 + ti3;
                CH(ic, 1, k) = tr4 - ti3;
            }
    }
#undef CC
#undef CH
}

// Radix 3, 5 and generic odd (7) passes.  For N <= 16 the odd factor is always the
// last backward / first forward factor, so only their ido == 1 parts exist
// (oracle radb3/radb5/radbg, radf3/radf5/radfg).
constexpr float kTaur = -0.5f, kTaui = 0.8660254037844386467637231707529362f;
constexpr float kTr11 = 0.3090169943749474241022934171828191f, kTi11 = 0.9510565162951535721164393333793821f;
constexpr float kTr12 = -0.8090169943749474241022934171828191f, kTi12 = 0.5877852522924731291687059546390728f;

template <int L1, int N>
TMF_DEVI void radb3(const float (&cc)[N], float (&ch)[N])
{
#pragma unroll
    for (int k = 0; k < L1; k++) {
        const float tr2 = 2.0f * cc[1 + 3 * k];
        const float cr2 = cc[3 * k] + kTaur * tr2;
        ch[k] = cc[3 * k] + tr2;
        const float ci3 = (2.0f * kTaui) * cc[2 + 3 * k];
        ch[k + 2 * L1] = cr2 + ci3;
        ch[k + L1] = cr2 - ci3;
    }
}

template <int L1, int N>
TMF_DEVI void radb5(const float (&cc)[N], float (&ch)[N])
{
#pragma unroll
    for (int k = 0; k < L1; k++) {
        const float c0 = cc[5 * k], c1 = cc[5 * k + 1], c2 = cc[5 * k + 2], c3 = cc[5 * k + 3], c4 = cc[5 * k + 4];
        const float ti5 = c2 + c2, ti4 = c4 + c4, tr2 = c1 + c1, tr3 = c3 + c3;
        ch[k] = c0 + tr2 + tr3;
        const float cr2 = c0 + kTr11 * tr2 + kTr12 * tr3;
        const float cr3 = c0 + kTr12 * tr2 + kTr11 * tr3;
        const float ci5 = ti5 * kTi11 + ti4 * kTi12, ci4 = ti5 * kTi12 - ti4 * kTi11;
        ch[k + 4 * L1] = cr2 + ci5;
        ch[k + L1] = cr2 - ci5;
        ch[k + 3 * L1] = cr3 + ci4;
        ch[k + 2 * L1] = cr3 - ci4;
    }
}

// generic odd radix IP <= 7 (single-term tail of pocketfft's accumulation), ido == 1;
// cc is scratch, the result is in ch
template <int IP, int L1, int N>
TMF_DEVI void radbg(float (&cc)[N], float (&ch)[N], const float *cs)
{
    static_assert(IP <= 7, "accumulation tail restated for ip <= 7 only");
    constexpr int IPPH = (IP + 1) / 2;
#pragma unroll
    for (int k = 0; k < L1; ++k) ch[k] = cc[IP * k];
#pragma unroll
    for (int j = 1; j < IPPH; ++j) {
        const int jc = IP - j, j2 = 2 * j - 1;
#pragma unroll
        for (int k = 0; k < L1; ++k) {
            ch[k + L1 * j] = 2.0f * cc[j2 + IP * k];
            ch[k + L1 * jc] = 2.0f * cc[j2 + 1 + IP * k];
        }
    }
#pragma unroll
    for (int l = 1; l < IPPH; ++l) {
        const int lc = IP - l;
#pragma unroll
        for (int ik = 0; ik < L1; ++ik) {
            cc[ik + L1 * l] = ch[ik] + cs[2 * l] * ch[ik + L1] + cs[4 * l] * ch[ik + 2 * L1];
            cc[ik + L1 * lc] = cs[2 * l + 1] * ch[ik + L1 * (IP - 1)] + cs[4 * l + 1] * ch[ik + L1 * (IP - 2)];
        }
        int iang = 2 * l;
#pragma unroll
        for (int j = 3; j < IPPH; ++j) {
            const int jc = IP - j;
            iang += l;
            if (iang > IP) iang -= IP;
#pragma unroll
            for (int ik = 0; ik < L1; ++ik) {
                cc[ik + L1 * l] = cc[ik + L1 * l] + cs[2 * iang] * ch[ik + L1 * j];
                cc[ik + L1 * lc] = cc[ik + L1 * lc] + cs[2 * iang + 1] * ch[ik + L1 * jc];
            }
        }
    }
#pragma unroll
    for (int j = 1; j < IPPH; ++j)
#pragma unroll
        for (int ik = 0; ik < L1; ++ik) ch[ik] = ch[ik] + ch[ik + L1 * j];
#pragma unroll
    for (int j = 1; j < IPPH; ++j) {
        const int jc = IP - j;
#pragma unroll
        for (int k = 0; k < L1; ++k) {
            const float a = cc[k + L1 * j], b = cc[k + L1 * jc];
            ch[k + L1 * jc] = a + b;
            ch[k + L1 * j] = a - b;
        }
    }
}

template <int L1, int N, typename T>
TMF_DEVI void radf3(const T (&cc)[N], T (&ch)[N])
{
#pragma unroll
    for (int k = 0; k < L1; k++) {
        const T cr2 = cc[k + L1] + cc[k + 2 * L1];
        ch[3 * k] = cc[k] + cr2;
        ch[2 + 3 * k] = kTaui * (cc[k + 2 * L1] - cc[k + L1]);
        ch[1 + 3 * k] = cc[k] + kTaur * cr2;
    }
}

template <int L1, int N, typename T>
TMF_DEVI void radf5(const T (&cc)[N], T (&ch)[N])
{
#pragma unroll
    for (int k = 0; k < L1; k++) {
        const T cr2 = cc[k + 4 * L1] + cc[k + L1], ci5 = cc[k + 4 * L1] - cc[k + L1];
        const T cr3 = cc[k + 3 * L1] + cc[k + 2 * L1], ci4 = cc[k + 3 * L1] - cc[k + 2 * L1];
        ch[5 * k] = cc[k] + cr2 + cr3;
        ch[5 * k + 1] = cc[k] + kTr11 * cr2 + kTr12 * cr3;
        ch[5 * k + 2] = kTi11 * ci5 + kTi12 * ci4;
        ch[5 * k + 3] = cc[k] + kTr12 * cr2 + kTr11 * cr3;
        ch[5 * k + 4] = kTi12 * ci5 - kTi11 * ci4;
    }
}

// generic odd radix, ido == 1: the result is left in cc (ch is scratch)
template <int IP, int L1, int N, typename T>
TMF_DEVI void radfg(T (&cc)[N], T (&ch)[N], const float *cs)
{
    static_assert(IP <= 7, "accumulation tail restated for ip <= 7 only");
    constexpr int IPPH = (IP + 1) / 2;
#pragma unroll
    for (int j = 1; j < IPPH; ++j) {
        const int jc = IP - j;
#pragma unroll
        for (int k = 0; k < L1; ++k) {
            const T t1 = cc[k + L1 * j], t2 = cc[k + L1 * jc];
            cc[k + L1 * j] = t2 + t1;
            cc[k + L1 * jc] = t2 - t1;
        }
    }
#pragma unroll
    for (int l = 1; l < IPPH; ++l) {
        const int lc = IP - l;
#pragma unroll
        for (int ik = 0; ik < L1; ++ik) {
            ch[ik + L1 * l] = cc[ik] + cs[2 * l] * cc[ik + L1] + cs[4 * l] * cc[ik + 2 * L1];
            ch[ik + L1 * lc] = cs[2 * l + 1] * cc[ik + L1 * (IP - 1)] + cs[4 * l + 1] * cc[ik + L1 * (IP - 2)];
        }
        int iang = 2 * l;
#pragma unroll
        for (int j = 3; j < IPPH; ++j) {
            const int jc = IP - j;
            iang += l;
            if (iang > IP) iang -= IP;
#pragma unroll
            for (int ik = 0; ik < L1; ++ik) {
                ch[ik + L1 * l] = ch[ik + L1 * l] + cs[2 * iang] * cc[ik + L1 * j];
                ch[ik + L1 * lc] = ch[ik + L1 * lc] + cs[2 * iang + 1] * cc[ik + L1 * jc];
            }
        }
    }
#pragma unroll
    for (int ik = 0; ik < L1; ++ik) ch[ik] = cc[ik];
#pragma unroll
    for (int j = 1; j < IPPH; ++j)
#pragma unroll
        for (int ik = 0; ik < L1; ++ik) ch[ik] = ch[ik] + cc[ik + L1 * j];
#pragma unroll
    for (int k = 0; k < L1; ++k) cc[IP * k] = ch[k];
#pragma unroll
    for (int j = 1; j < IPPH; ++j) {
        const int jc = IP - j, j2 = 2 * j - 1;
#pragma unroll
        for (int k = 0; k < L1; ++k) {
            cc[j2 + IP * k] = ch[k + L1 * j];
            cc[j2 + 1 + IP * k] = ch[k + L1 * jc];
        }
    }
}

// rfftp::exec for the factorisations pocketfft picks (4 -> [4], 6 -> [2,3],
// 8 -> [2,4], 10 -> [2,5], 12 -> [4,3], 14 -> [2,7], 16 -> [4,4]); copy_and_norm
// multiplies by fct at the end.
template <int N>
TMF_DEVI void rfft_backward(float (&c)[N], float fct)
{
    float ch[N];
    if constexpr (N == 4) {
        radb4<1, 1>(c, ch, nullptr);
#pragma unroll
        for (int i = 0; i < N; ++i) c[i] = fct * ch[i];
        return;
    } else if constexpr (N == 6) {
        radb2<3, 1>(c, ch, kRfftTw6);
        radb3<2>(ch, c);
    } else if constexpr (N == 8) {
        radb2<4, 1>(c, ch, kRfftTw8);
        radb4<1, 2>(ch, c, nullptr);
    } else if constexpr (N == 10) {
        radb2<5, 1>(c, ch, kRfftTw10);
        radb5<2>(ch, c);
    } else if constexpr (N == 12) {
        radb4<3, 1>(c, ch, kRfftTw12);
        radb3<4>(ch, c);
    } else if constexpr (N == 14) {
        radb2<7, 1>(c, ch, kRfftTw14);
        radbg<7, 2>(ch, c, kRfftTws14);
    } else {
        radb4<4, 1>(c, ch, kRfftTw16);
        radb4<1, 4>(ch, c, nullptr);
    }
#pragma unroll
    for (int i = 0; i < N; ++i) c[i] *= fct;
}

template <int N, typename T>
TMF_DEVI void rfft_forward(T (&c)[N], float fct)
{
    T ch[N];
    if constexpr (N == 4) {
        radf4<1, 1>(c, ch, nullptr);
#pragma unroll
        for (int i = 0; i < N; ++i) c[i] = fct * ch[i];
        return;
    } else if constexpr (N == 6) {
        radf3<2>(c, ch);
        radf2<3, 1>(ch, c, kRfftTw6);
    } else if constexpr (N == 8) {
        radf4<1, 2>(c, ch, nullptr);
        radf2<4, 1>(ch, c, kRfftTw8);
    } else if constexpr (N == 10) {
        radf5<2>(c, ch);
        radf2<5, 1>(ch, c, kRfftTw10);
    } else if constexpr (N == 12) {
        radf3<4>(c, ch);
        radf4<3, 1>(ch, c, kRfftTw12);
    } else if constexpr (N == 14) {
        radfg<7, 2>(c, ch, kRfftTws14);  // result stays in c
        radf2<7, 1>(c, ch, kRfftTw14);
#pragma unroll
        for (int i = 0; i < N; ++i) c[i] = fct * ch[i];
        return;
    } else {
        radf4<1, 4>(c, ch, nullptr);
        radf4<4, 1>(ch, c, kRfftTw16);
    }
#pragma unroll
    for (int i = 0; i < N; ++i) c[i] *= fct;
}

template <int N> struct Tw;
#define TMF_TW(N) template <> struct Tw<N> { static constexpr const float *d = kDctTw##N; static constexpr float norm = kNorm##N; }
TMF_TW(4);
TMF_TW(6);
TMF_TW(8);
TMF_TW(10);
TMF_TW(12);
TMF_TW(14);
TMF_TW(16);
#undef TMF_TW

// T_dcst23 type 2 (scipy.fftpack.dct, norm="ortho")
template <int N>
TMF_DEVI void dct2(float (&c)[N])
{
    constexpr int NS2 = (N + 1) / 2;
    const float *tw = Tw<N>::d;
    c[0] *= 2.0f;
    c[N - 1] *= 2.0f;
#pragma unroll
    for (int k = 1; k < N - 1; k += 2) {
        const float t = c[k + 1];
        c[k + 1] = t - c[k];
        c[k] = c[k] + t;
    }
    rfft_backward<N>(c, Tw<N>::norm);
#pragma unroll
    for (int k = 1; k < NS2; ++k) {
        const int kc = N - k;
        const float t1 = tw[k - 1] * c[kc] + tw[kc - 1] * c[k];
        const float t2 = tw[k - 1] * c[k] - tw[kc - 1] * c[kc];
        c[k] = 0.5f * (t1 + t2);
        c[kc] = 0.5f * (t1 - t2);
    }
    c[NS2] *= tw[NS2 - 1];
    c[0] *= kSqrt2 * 0.5f;
}

// T_dcst23 type 3 (scipy.fftpack.idct, norm="ortho")
template <int N, typename T>
TMF_DEVI void dct3(T (&c)[N])
{
    constexpr int NS2 = (N + 1) / 2;
    const float *tw = Tw<N>::d;
    c[0] *= kSqrt2;
#pragma unroll
    for (int k = 1; k < NS2; ++k) {
        const int kc = N - k;
        const T t1 = c[k] + c[kc], t2 = c[k] - c[kc];
        c[k] = tw[k - 1] * t2 + tw[kc - 1] * t1;
        c[kc] = tw[k - 1] * t1 - tw[kc - 1] * t2;
    }
    c[NS2] *= 2.0f * tw[NS2 - 1];
    rfft_forward<N>(c, Tw<N>::norm);
#pragma unroll
    for (int k = 1; k < N - 1; k += 2) {
        const T t = c[k];
        c[k] = t - c[k + 1];
        c[k + 1] = t + c[k + 1];
    }
}

}  // namespace dct

// ---------------------------------------------------------------------------
// SVD (N5/N6), DESIGN.md 3.4: phase 1 f32 one-sided Jacobi (<= 4 sweeps) on D,
// phase 2 two Bjorck steps on f64(V32), phase 3 f64 one-sided Jacobi on
// A0 = D V0 to convergence.  B/L rows of A and V per lane, L lanes per block.
// The op sequence is the oracle's: dot products are fma chains over each lane's
// R contiguous rows, combined across the L lanes by an xor butterfly (== the
// oracle's balanced pairwise tree); round-robin pair schedule; the rotation
// tests and the IEEE-only rotation formula of oracle rotation()/rotationf().
// ---------------------------------------------------------------------------
// kBranchy: skip a pair's rotation / update when no block of the wave rotates it
// (pays off in the converging f64 sweeps); branch-free otherwise (the f32 sweeps
// rotate nearly every pair somewhere in the wave, and a join costs register moves).
template <typename T> struct JacP;
template <> struct JacP<double> {
    static constexpr bool kBranchy = true;
    static constexpr int kMaxSweeps = 32;
    static constexpr int max_sweeps(int) { return kMaxSweeps; }
    static constexpr double kTol2 = 7.888609052210118e-31;  // 2^-100
    static constexpr double kC2 = 9.860761315262648e-32;    // 2^-103
};
template <> struct JacP<float> {
    static constexpr bool kBranchy = false;
    // sweeps of phase 1 (oracle JAC32_MAX_SWEEPS).  5 from b = 10 on was measured in round 3:
    // embed<10> / <12> -9 %, <14> -7 %, <16> -3 % on noise covers, but +4..5 % on camera-like
    // covers (profiles/r03/r03y/, r03z/), so every size keeps 4
    static constexpr int max_sweeps(int) { return 4; }
    static constexpr float kTol2 = 9.094947017729282e-13f;  // 2^-40
    static constexpr float kC2 = 2.842170943040401e-14f;    // 2^-45
    static constexpr float kC2A = 3.552713678800501e-15f;   // 2^-48
    static constexpr float kFMin = 9.313225746154785e-10f;  // 2^-30
};

// circle-method schedule: L = [0, 1 + (k-1+s) mod (b-1)], pair p = (L[p], L[b-1-p]) sorted
template <int B>
struct Sched {
    static constexpr int idx(int s, int k) { return k == 0 ? 0 : 1 + ((k - 1 + s) % (B - 1)); }
    static constexpr int lo(int s, int p) { return idx(s, p) < idx(s, B - 1 - p) ? idx(s, p) : idx(s, B - 1 - p); }
    static constexpr int hi(int s, int p) { return idx(s, p) < idx(s, B - 1 - p) ? idx(s, B - 1 - p) : idx(s, p); }
};

// ---- compile-time loops (guaranteed unrolling: register arrays need constant indices)
template <typename F, int... Is>
TMF_DEVI void static_for_impl(F &&f, std::integer_sequence<int, Is...>)
{
    (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, typename F>
TMF_DEVI void static_for(F &&f)
{
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// ---- cross-lane moves inside a block group (DPP / ds_swizzle, no LDS traffic)
// DPP controls: quad_perm [1,0,3,2] = 0xB1 (xor 1), [2,3,0,1] = 0x4E (xor 2),
// row_half_mirror = 0x141 (lane i <-> 7-i within 8 lanes).
// (update_dpp with bound_ctrl: every control used here reads a valid lane, so the same
// value as a plain DPP move, and the compiler can fold the move into the f32 add or
// subtract that consumes it: v_add_f32_dpp)
template <int CTRL>
TMF_DEVI int dpp_i(int v) { return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, true); }
template <int PATTERN>
TMF_DEVI int swz_i(int v) { return __builtin_amdgcn_ds_swizzle(v, PATTERN); }

template <int CTRL>
TMF_DEVI double dpp(double v)
{
    const long long b = __builtin_bit_cast(long long, v);
    const int lo = dpp_i<CTRL>((int)b), hi = dpp_i<CTRL>((int)(b >> 32));
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
template <int CTRL>
TMF_DEVI float dpp(float v) { return __builtin_bit_cast(float, dpp_i<CTRL>(__builtin_bit_cast(int, v))); }
template <int CTRL>
TMF_DEVI int dpp(int v) { return dpp_i<CTRL>(v); }

template <int PATTERN>
TMF_DEVI double swz(double v)
{
    const long long b = __builtin_bit_cast(long long, v);
    const int lo = swz_i<PATTERN>((int)b), hi = swz_i<PATTERN>((int)(b >> 32));
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
template <int PATTERN>
TMF_DEVI float swz(float v) { return __builtin_bit_cast(float, swz_i<PATTERN>(__builtin_bit_cast(int, v))); }
template <int PATTERN>
TMF_DEVI int swz(int v) { return swz_i<PATTERN>(v); }

// Butterfly sum over the L lanes of a group == the oracle's pairwise tree:
// level 3 pairs lane i with 7-i, whose value (p6+p7)+(p4+p5) equals (p4+p5)+(p6+p7) bitwise.
template <int L, typename T>
TMF_DEVI T group_sum(T v)
{
    static_assert(L == 1 || L == 2 || L == 4 || L == 8, "group size");
    if constexpr (L >= 2) v = v + dpp<0xB1>(v);
    if constexpr (L >= 4) v = v + dpp<0x4E>(v);
    if constexpr (L >= 8) v = v + dpp<0x141>(v);
    return v;
}

// value of lane (group base + K) for every lane of the group
template <int L, int K, typename T>
TMF_DEVI T group_bcast(T v)
{
    if constexpr (L == 1) return v;
    else if constexpr (L == 2) return dpp<K == 0 ? 0xA0 : 0xF5>(v);                    // quad_perm [K,K,K+2,K+2]
    else if constexpr (L == 4) return dpp<K | (K << 2) | (K << 4) | (K << 6)>(v);      // quad_perm [K,K,K,K]
    else return swz<(K << 5) | 0x18>(v);                                                // bitmask: (lane & 0x18) | K
}

// OR over the L lanes of a group (same butterfly as group_sum)
template <int L>
TMF_DEVI int group_or(int v)
{
    if constexpr (L >= 2) v = v | dpp<0xB1>(v);
    if constexpr (L >= 4) v = v | dpp<0x4E>(v);
    if constexpr (L >= 8) v = v | dpp<0x141>(v);
    return v;
}

// exec-style mask of the lanes that are member K of their group
template <int L, int K>
constexpr unsigned long long kMemberMask = L == 1 ? ~0ull
                                         : L == 2 ? 0x5555555555555555ull << K
                                         : L == 4 ? 0x1111111111111111ull << K
                                                  : 0x0101010101010101ull << K;

TMF_DEVI double fma_t(double a, double b, double c) { return __builtin_fma(a, b, c); }
TMF_DEVI float fma_t(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
TMF_DEVI double abs_t(double a) { return __builtin_fabs(a); }
TMF_DEVI float abs_t(float a) { return __builtin_fabsf(a); }
TMF_DEVI double sign1_t(double d) { return __builtin_copysign(1.0, d); }
TMF_DEVI float sign1_t(float d) { return __builtin_copysignf(1.0f, d); }

// this lane's part of sum over rows of A[:,i]*A[:,j] (fma chain over its R rows)
template <int R, int B, typename T>
TMF_DEVI T cdot_part(const T (&A)[R][B], int i, int j)
{
    T acc = T(0);
#pragma unroll
    for (int r = 0; r < R; ++r) acc = fma_t(A[r][i], A[r][j], acc);
    return acc;
}

// sum over rows of A[:,i]*A[:,j] in the contract order (oracle cdot / cdotf)
template <int R, int B, int L, typename T>
TMF_DEVI T cdot(const T (&A)[R][B], int i, int j)
{
    return group_sum<L>(cdot_part<R, B>(A, i, j));
}


// Bitwise blend with an opaque lane mask: keeps the selection a v_bfi_b32 on values,
// so the optimiser cannot turn "pick nrm[i] by lane" into a dynamically indexed
// (scratch) array access.
TMF_DEVI double blend(int mask, double x, double y)
{
    const long long m = (long long)mask;  // 0 or -1
    const long long xb = __builtin_bit_cast(long long, x), yb = __builtin_bit_cast(long long, y);
    return __builtin_bit_cast(double, (xb & m) | (yb & ~m));
}
TMF_DEVI float blend(int mask, float x, float y)
{
    const int xb = __builtin_bit_cast(int, x), yb = __builtin_bit_cast(int, y);
    return __builtin_bit_cast(float, (xb & mask) | (yb & ~mask));
}

// 1/sqrt(x) of the contract.  f64 phase: IEEE ops only (oracle rsqrt_n),
// integer seed + 4 Newton steps.  f32 phase (a preconditioner): the hardware v_rsq_f32,
// which the oracle models by its measured truth table (oracle rsq_hw,
// tests/golden/gfx950_trans_delta.npz).
TMF_DEVI double rsqrt_c(double x)
{
    const unsigned long long i = 0x5fe6eb50c7b537a9ull - (__builtin_bit_cast(unsigned long long, x) >> 1);
    double y = __builtin_bit_cast(double, i);
    const double hx = 0.5 * x;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const double t = y * y;
        const double u = __builtin_fma(-hx, t, 1.5);
        y = y * u;
    }
    return y;
}
TMF_DEVI float rsqrt_c(float x) { return __builtin_amdgcn_rsqf(x); }

// Columns i, j of A (and V) <- (c x - s y, s x + c y) as fma(-s, y, c*x), fma(s, x, c*y)
template <int R, int B, bool WANT_V, typename T>
TMF_DEVI void rotate_cols(T (&A)[R][B], T (&V)[R][B], int i, int j, T c, T sn)
{
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const T x = A[r][i], y = A[r][j];
        A[r][i] = fma_t(-sn, y, c * x);
        A[r][j] = fma_t(sn, x, c * y);
    }
    if constexpr (WANT_V) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const T x = V[r][i], y = V[r][j];
            V[r][i] = fma_t(-sn, y, c * x);
            V[r][j] = fma_t(sn, x, c * y);
        }
    }
}

template <typename T>
struct Rot {
    T c, s, tg;
};

// Rotation of a pair (oracle rotation() / rotationf())
template <typename T>
TMF_DEVI Rot<T> rotation(T alpha, T beta, T gamma)
{
    Rot<T> o;
    const T d = beta - alpha;
    const T g = gamma + gamma;
    const T x = fma_t(d, d, g * g);
    const T r = x * rsqrt_c(x);
    const T w = abs_t(d) + r;
    const T q = rsqrt_c((r + r) * w);
    const T sg = sign1_t(d);
    o.c = w * q;
    o.s = (g * sg) * q;
    o.tg = (((g * g) * r) * (q * q)) * sg;
    return o;
}

// One-sided Jacobi on A (and V when WANT_V) in precision T.  Returns this block's
// sweep count exactly as the oracle counts it (sweeps up to and including the
// first one without a rotation, capped at the precision's maximum); the wave runs
// until its slowest block stops -- further sweeps of a converged block are
// no-ops (same A, same tests, no rotation).  Pairs of a round are disjoint, so
// they are applied in any order.  Every lane of a group holds the column norms;
// lane q evaluates the rotations of pairs [q*PP, q*PP+PP) and broadcasts
// (c, s, t*gamma).  Rotation and update branches are wave-uniform (__any): a pair
// no block of the wave rotates costs nothing, and inside the branch lanes whose
// block skips it apply the bitwise-exact identity (no divergent exec masks, so
// the updates stay in place instead of being computed aside and copied back).
// Rows per lane: ceil(B / L); rows past B are zero padding (exact: they add +0 to
// every dot product and stay 0 under every rotation).
template <int B, int L>
constexpr int kRows = (B + L - 1) / L;

// Norms in LDS (8-lane blocks, b = 14 / 16, one pair per lane): instead of every lane
// holding all b column norms, selecting its pair's two by lane-masked blends and applying
// every pair's t*gamma, the block keeps one copy of the norms in LDS (written once per
// sweep by the block's first lane); the owner of a pair reads its two norms there and,
// when it rotates, writes them back updated.  Same operations on the same values as the
// register form, so the same bits; 32 fewer live VGPRs (the norms) in the f64 phase,
// ~40 fewer VALU operations and 16 fewer broadcasts (t*gamma) per round.
template <int L, typename T>
constexpr bool kLdsNorms = L == 8 && std::is_same_v<T, double>;  // the f64 phase (the f32 one: one wave / SIMD at b = 14)

// Rotation parameters through LDS (8-lane blocks): the owner of each pair writes its
// (c, s) next to the norms and every lane of the block reads the pairs it applies
// (ds_write2 + one ds_read2 per pair), instead of two ds_swizzle per 32-bit half of each
// broadcast value.  Pure data movement: the same bits.
template <int L>
constexpr bool kLdsBcast = L == 8;  // 2- and 4-lane groups: DPP moves (LDS measured within noise there)

// Pair dot products through LDS (8-lane blocks, one pair per lane): only the owner of a
// pair needs its gamma, so instead of the 3-level DPP butterfly for every pair on every
// lane, each lane writes its partials and the owner sums its pair's 8 partials in the
// butterfly's tree order ((p0+p1)+(p2+p3))+((p4+p5)+(p6+p7)) -- the same bits.
template <int L, typename T>
constexpr bool kLdsSums = L == 8 && std::is_same_v<T, double>;

// pair p's lower / higher column for every p < b/2 of round s, one 4-bit field per lane
// p; a lane without a pair (p >= b/2: b = 14) gets slot 15, a dummy past the b norms
template <int B, int S, bool HI>
constexpr uint32_t sched_nibbles()
{
    uint32_t v = 0;
    for (int p = 0; p < 8; ++p) v |= (uint32_t)(p < B / 2 ? (HI ? Sched<B>::hi(S, p) : Sched<B>::lo(S, p)) : 15) << (4 * p);
    return v;
}

// keeps the compiler from moving this block's LDS norm accesses across a round boundary
// (the lanes of a wave see each other's LDS writes in program order)
TMF_DEVI void lds_order() { asm volatile("" ::: "memory"); }
// the values leave this point in order: the arithmetic producing them is not moved past it
TMF_DEVI void pin_order(float &a, float &b) { asm volatile("" : "+v"(a), "+v"(b)); }

// One sweep (oracle jacobi_sweep() / the loop body of jacobi()): nrm are recomputed, the
// b-1 rounds of b/2 disjoint pairs rotate every pair that passes the tests.  `enable`
// (same on the L lanes of a block) adds "skip" to every test of this block's pairs: a
// disabled block takes the identity on every pair, bitwise.  Returns 1 on a lane that
// rotated one of its own pairs (group_or over the block = the block rotated).
template <typename T, int B, int L, bool WANT_V>
TMF_DEVI int jacobi_sweep(T (&A)[(B + L - 1) / L][B], T (&V)[(B + L - 1) / L][B], int q, T *nl, T c2, T c2a, bool enable)
{
    using P = JacP<T>;
    // NP pairs per round; lane q evaluates pairs [q*PP, q*PP + PP) that exist
    constexpr int R = kRows<B, L>, NP = B / 2, PP = (NP + L - 1) / L;
    constexpr bool kBranchy = P::kBranchy;
    constexpr bool kLN = kLdsNorms<L, T>;
    constexpr bool kLB = kLdsBcast<L>;
    static_assert(!kLN || NP <= 8, "LDS norms: 4-bit pair table");
    static_assert(!kLB || L * PP <= 8, "LDS broadcast: 8 parameter slots");
    // kLB: (c, s) of pair slot p at prm[2p], prm[2p+1] (after the 16 norms when those are
    // in LDS too), t*gamma at prm[16 + p] when the norms are replicated on the lanes
    T *prm = nl + (kLN ? 16 : 0);
    constexpr bool kLS = kLdsSums<L, T> && PP == 1;
    T *part = nl + 32;  // kLS: partial of pair p from lane k at part[p * 8 + k]
    if constexpr (kLN && B == 16) {
        // q through an opaque move (as in newton_try_lds): the per-round pair columns derived
        // from it are otherwise hoisted out of the sweep loop, held across it and spilled --
        // 4 scratch reloads per round at b = 16 (spilled VGPRs 74 -> 47, none left inside the
        // f64 loop; embed<16> -2.4 % noise / -1.6 % camera-like covers, profiles/r03/r03i/;
        // b = 14 has no spill to remove and measured +1 %)
        asm volatile("" : "+v"(q));
    }
    T nrm[B];
    // batches of dot products: all lane-local chains first, then all cross-lane sums,
    // so that the chains interleave and no DPP read waits on the write just before it
    static_for<B>([&](auto K) { nrm[K] = cdot_part<R, B>(A, K, K); });
    static_for<B>([&](auto K) { nrm[K] = group_sum<L>(nrm[K]); });
    if constexpr (kLN) {
        lds_order();
        if (q == 0) static_for<B>([&](auto K) { nl[K] = nrm[K]; });
        lds_order();
    }
    int rotated = 0;  // this lane rotated one of its own pairs this sweep
    static_for<B - 1>([&](auto S) {
        constexpr int s = S;
        T ga[NP];
        static_for<NP>([&](auto Pi) {
            constexpr int p = Pi, i = Sched<B>::lo(s, p), j = Sched<B>::hi(s, p);
            ga[p] = cdot_part<R, B>(A, i, j);
        });
        T gown = T(0);  // kLS: this lane's pair's gamma
        if constexpr (kLS) {
            lds_order();  // after the previous round's reads
            static_for<NP>([&](auto Pi) { part[Pi * 8 + q] = ga[Pi]; });
            lds_order();
            const T *pp = part + 8 * q;  // lane 7 at b = 14 reads an unused slot: no pair
            gown = ((pp[0] + pp[1]) + (pp[2] + pp[3])) + ((pp[4] + pp[5]) + (pp[6] + pp[7]));
        } else {
            static_for<NP>([&](auto Pi) { ga[Pi] = group_sum<L>(ga[Pi]); });
        }
        // this lane's pairs: select (alpha, beta, gamma), evaluate the rotation test
        // (only here -- the owner's flag travels with its parameters), rotation
        Rot<T> mine[PP];
        unsigned long long own_ball[PP];  // wave mask of the lanes whose U-th pair rotates
        int own_i = 0, own_j = 0;  // kLN: this lane's pair's columns
        static_for<PP>([&](auto U) {
            constexpr int p0 = U, i0 = Sched<B>::lo(s, p0), j0 = Sched<B>::hi(s, p0);
            T a, b, g = kLS ? gown : ga[p0];
            if constexpr (kLN) {
                const int pq = q * PP + p0;  // this lane's U-th pair
                own_i = (int)__builtin_amdgcn_ubfe(sched_nibbles<B, s, false>(), 4 * pq, 4);
                own_j = (int)__builtin_amdgcn_ubfe(sched_nibbles<B, s, true>(), 4 * pq, 4);
                a = nl[own_i];
                b = nl[own_j];
            } else {
                a = nrm[i0];
                b = nrm[j0];
            }
            int slot = -1;  // lane has a U-th pair this round
            static_for<L - 1>([&](auto Q1) {
                constexpr int QQ = Q1 + 1, p = QQ * PP + U;
                int m = -(int)(q == QQ);
                asm volatile("" : "+v"(m));
                if constexpr (p < NP) {
                    constexpr int i = Sched<B>::lo(s, p), j = Sched<B>::hi(s, p);
                    if constexpr (!kLN) {
                        a = blend(m, nrm[i], a);
                        b = blend(m, nrm[j], b);
                    }
                    if constexpr (!kLS) g = blend(m, ga[p], g);
                } else {
                    slot &= ~m;
                }
            });
            const T g2 = g * g;
            // every test evaluated (bitwise |): a short-circuit || becomes exec-mask branches
            bool skip = (g2 <= c2 * (a + b)) | (g2 <= (P::kTol2 * a) * b) | !enable;
            if constexpr (std::is_same_v<T, float>) skip = skip | (g2 <= c2a);
            const bool o = slot != 0 && !skip;
            own_ball[U] = __ballot(o);
            rotated |= (int)o;
            mine[U] = Rot<T>{T(1), T(0), T(0)};
            if (!kBranchy || __any(o)) {  // wave-uniform: every lane computes, non-rotating lanes keep identity
                const Rot<T> r = rotation(a, b, g);
                mine[U].c = o ? r.c : T(1);
                mine[U].s = o ? r.s : T(0);
                mine[U].tg = o ? r.tg : T(0);
            }
            if constexpr (kLN) {  // every lane writes its pair's norms back: old value -+ t*gamma
                nl[own_i] = a - mine[U].tg;  // (t*gamma = 0 when it does not rotate: the same bits)
                nl[own_j] = b + mine[U].tg;
            }
        });
        if constexpr (kLB) {
            lds_order();  // after the previous round's reads
            static_for<PP>([&](auto U) {
                prm[2 * (q * PP + U)] = mine[U].c;
                prm[2 * (q * PP + U) + 1] = mine[U].s;
                if constexpr (!kLN) prm[16 + q * PP + U] = mine[U].tg;
            });
            lds_order();
        }
        static_for<NP>([&](auto Pi) {
            constexpr int p = Pi, i = Sched<B>::lo(s, p), j = Sched<B>::hi(s, p), u = p % PP, src = p / PP;
            T c, sn;
            if constexpr (kLB) {
                c = prm[2 * p];
                sn = prm[2 * p + 1];
            } else {
                c = group_bcast<L, src>(mine[u].c);
                sn = group_bcast<L, src>(mine[u].s);
            }
            // Wave-uniform branch (taken iff the owner lane of this pair rotates it in
            // some block of the wave); lanes whose block skips this pair apply the identity
            // (c, s, t*gamma) = (1, 0, 0): fma(-0, y, 1*x) == x bitwise for every value
            // A (phase 3) and V can hold (their fma chains start from +0 and never make
            // -0), and A32 / phase-1 A only feed cdot(), which ignores signs of zero.
            if (!kBranchy || (own_ball[u] & kMemberMask<L, src>) != 0) {
                if constexpr (!kLN) {
                    T tg;
                    if constexpr (kLB) tg = prm[16 + p];
                    else tg = group_bcast<L, src>(mine[u].tg);
                    nrm[i] = nrm[i] - tg;
                    nrm[j] = nrm[j] + tg;
                }
                rotate_cols<R, B, WANT_V>(A, V, i, j, c, sn);
            }
        });
    });
    return rotated;
}

// F = |A|_F^2 (contract dots) and the Jacobi's noise-floor constants
template <typename T, int B, int L>
TMF_DEVI T frob2(const T (&A)[(B + L - 1) / L][B])
{
    T F = T(0);
    static_for<B>([&](auto K) { F += cdot<kRows<B, L>, B, L>(A, K, K); });
    return F;
}

template <typename T, int B, int L, bool WANT_V>
TMF_DEVI int jacobi(T (&A)[(B + L - 1) / L][B], T (&V)[(B + L - 1) / L][B], int q, T *nl = nullptr)
{
    using P = JacP<T>;
    const T F = frob2<T, B, L>(A);
    const T c2 = P::kC2 * F;
    T c2a = T(0);
    bool live = true;
    if constexpr (std::is_same_v<T, float>) {
        c2a = P::kC2A * (F * F);
        live = F >= P::kFMin;  // oracle jacobi_f32: return 0 (no sweep) below 2^-30
    }
    int count = 0;
    bool active = live;
    for (int sweep = 0; sweep < P::max_sweeps(B); ++sweep) {
        const int rotated = jacobi_sweep<T, B, L, WANT_V>(A, V, q, nl, c2, c2a, live);
        count += active ? 1 : 0;
        active = active && group_or<L>(rotated) != 0;  // block rotated a pair this sweep
        if (!__any(rotated)) break;
    }
    return count;
}

// ---- Phase 3 with a Newton finish (oracle jacobi_newton() / newton_try(),
// DESIGN.md 3.4): after each rotating sweep, F_ij = f32(G_ij) / f32(G_jj - G_ii) over the
// pairs the Jacobi's tests would rotate (G = A^T A); if every |F_ij| <= 2^-27 the block
// takes V <- V (I + F), A <- A (I + F) -- the correction formed in f32 -- and is done,
// otherwise it takes the next sweep.
constexpr float kNwtApply = 7.450580596923828e-09f;  // 2^-27

// upper-triangle index of pair (i, j), i < j
template <int B>
constexpr int tri(int i, int j) { return i * B - i * (i + 1) / 2 + (j - i - 1); }

// The step's scaled acceptance test (round 6; oracle newton_scaled_ok): besides
// every |F_ij| <= 2^-27, with x = 2^27 |F|, r_k = f32(G_kk) * (1 / f32(max G)) and
// q_j = sum_i x_ij^2 r_i (an fmaf chain per column in the sweep's pair order: round s, its pair
// (i, j) adds x^2 r_j to q_i and x^2 r_i to q_j), every pair must have q_j q_k <= 64 (r_j + r_k)
// -- the step's second-order terms then stay on each pair's own scale (the absolute test alone
// left graded blocks' small triplets off by up to 447 units of 2^-53 sigma_1 / g_k).  The pair
// tests run only where the per-column screen (nwt_col_ok) does not already imply them.
constexpr float kNwtScale = 134217728.0f;  // 2^27
TMF_DEVI float nwt_x2(float f)
{
    const float x = __builtin_fabsf(f) * kNwtScale;
    return x * x;
}
TMF_DEVI bool nwt_pair_ok(float qj, float qk, float rj, float rk) { return qj * qk <= 64.0f * (rj + rk); }
// the screen: q_j^2 <= 64 r_j for every column implies every pair's test in f32 (q_j q_k <=
// 64 sqrt(r_j r_k) <= 32 (r_j + r_k), and the factor 2 covers the roundings)
TMF_DEVI bool nwt_col_ok(float qj, float rj) { return qj * qj <= 64.0f * rj; }
// the gate: with x_max the block's largest 2^27 |F|, S = sum r and r_min = min r, every q_j is
// at most x_max^2 S, so (x_max^2 S)^2 <= 32 r_min implies every column's screen (the factor 2
// covers the f32 roundings of the q chains and of the gate); the sums are then not formed
TMF_DEVI bool nwt_gate(float fmax_abs, float S, float rmin)
{
    const float x = fmax_abs * kNwtScale, t = x * x * S;
    return t * t <= 32.0f * rmin;
}
// largest value over the L lanes of a group, for non-negative floats (their bit patterns order alike)
template <int L>
TMF_DEVI float group_max_nonneg(float v)
{
    int b = __builtin_bit_cast(int, v), o;
    if constexpr (L >= 2) b = (o = dpp<0xB1>(b)) > b ? o : b;
    if constexpr (L >= 4) b = (o = dpp<0x4E>(b)) > b ? o : b;
    if constexpr (L >= 8) b = (o = dpp<0x141>(b)) > b ? o : b;
    return __builtin_bit_cast(float, b);
}

template <int B>
TMF_DEVI bool nwt_scaled_ok(const double (&G)[B], const float (&F)[B * (B - 1) / 2], float fmx, bool ok);

// X <- X + f64(f32(X) F) on this lane's rows, F antisymmetric (upper triangle in F[],
// diagonal 0): fma chain over i != j, as the oracle's apply_f().  `take` false: unchanged.
template <int B, int L>
TMF_DEVI void apply_f(double (&X)[(B + L - 1) / L][B], const float (&F)[B * (B - 1) / 2], bool take)
{
    constexpr int R = kRows<B, L>;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        float xr[B];
#pragma unroll
        for (int i = 0; i < B; ++i) xr[i] = (float)X[r][i];
#pragma unroll
        for (int j = 0; j < B; ++j) {
            float acc = 0.0f;
#pragma unroll
            for (int i = 0; i < B; ++i) {
                if (i < j) acc = __builtin_fmaf(xr[i], F[tri<B>(i, j)], acc);
                else if (i > j) acc = __builtin_fmaf(-xr[i], F[tri<B>(j, i)], acc);
            }
            X[r][j] = take ? X[r][j] + (double)acc : X[r][j];
        }
    }
}

// Pair p of the upper triangle (tri<B> order): its columns
template <int B>
struct TriPair {
    static constexpr int i(int p)
    {
        int k = 0;
        for (int a = 0; a < B; ++a)
            for (int b = a + 1; b < B; ++b, ++k)
                if (k == p) return a;
        return -1;
    }
    static constexpr int j(int p)
    {
        int k = 0;
        for (int a = 0; a < B; ++a)
            for (int b = a + 1; b < B; ++b, ++k)
                if (k == p) return b;
        return -1;
    }
};

// fmx: the block's largest |F|; ok: the absolute test passed (the result matters only then)
template <int B>
TMF_DEVI bool nwt_scaled_ok(const double (&G)[B], const float (&F)[B * (B - 1) / 2], float fmx, bool ok)
{
    double gmax = 0.0;
#pragma unroll
    for (int k = 0; k < B; ++k) gmax = G[k] > gmax ? G[k] : gmax;
    const float ginv = 1.0f / (float)gmax;
    float r[B], qw[B], sum = 0.0f, rmin = 1.0f;
#pragma unroll
    for (int k = 0; k < B; ++k) {
        r[k] = (float)G[k] * ginv;
        qw[k] = 0.0f;
        sum += r[k];
        rmin = __builtin_fminf(rmin, r[k]);
    }
    if (!__any(ok && !nwt_gate(fmx, sum, rmin))) return true;
    static_for<B - 1>([&](auto S) {
        static_for<B / 2>([&](auto P) {
            constexpr int i = Sched<B>::lo(S, P), j = Sched<B>::hi(S, P);
            const float x2 = nwt_x2(F[tri<B>(i, j)]);
            qw[i] = __builtin_fmaf(x2, r[j], qw[i]);
            qw[j] = __builtin_fmaf(x2, r[i], qw[j]);
        });
    });
    bool pass = true;
#pragma unroll
    for (int k = 0; k < B; ++k) pass = pass && nwt_col_ok(qw[k], r[k]);
    if (__any(!pass)) {
        pass = true;
#pragma unroll
        for (int j = 0; j < B; ++j)
#pragma unroll
            for (int k = j + 1; k < B; ++k) pass = pass && nwt_pair_ok(qw[j], qw[k], r[j], r[k]);
    }
    return pass;
}

// F_p from the pair's dot product g and the diagonal of G, or 0 if the Jacobi's tests would
// not rotate the pair (oracle newton_try)
TMF_DEVI float newton_f(double g, double gi, double gj, double c2)
{
    const double g2 = g * g;
    const bool rot = !(g2 <= c2 * (gi + gj) || g2 <= (JacP<double>::kTol2 * gi) * gj);
    return rot ? (float)g / (float)(gj - gi) : 0.0f;
}

// Returns true if the step was taken (same on the L lanes of a block; never when !enable).
// 2-lane blocks split the pairs: of each couple (p, p+1) in triangle order, lane 0 forms F_p
// and lane 1 F_(p+1) -- each summing the couple's partial dot products in the butterfly's
// operand order (p0 + p1 and p1 + p0 are the same bits) -- and the two swap F by one DPP
// move, so the tests and the IEEE divides run once per pair instead of on both lanes.
template <int B, int L>
TMF_DEVI bool newton_try(double (&A)[(B + L - 1) / L][B], double (&V)[(B + L - 1) / L][B], double c2, bool enable)
{
    constexpr int R = kRows<B, L>, NP = B * (B - 1) / 2;
    double G[B];
    static_for<B>([&](auto K) { G[K] = cdot_part<R, B>(A, K, K); });
    static_for<B>([&](auto K) { G[K] = group_sum<L>(G[K]); });
    float F[NP], fmx = 0.0f;
    int ok = enable ? 1 : 0;
    if constexpr (L == 2) {
        int q = (int)(__lane_id() & 1);
        asm volatile("" : "+v"(q));  // a lane mask, not a branch
        const int m0 = -(int)(q == 0);
        static_for<NP / 2>([&](auto C) {
            constexpr int p0 = 2 * C, p1 = p0 + 1;
            constexpr int i0 = TriPair<B>::i(p0), j0 = TriPair<B>::j(p0), i1 = TriPair<B>::i(p1), j1 = TriPair<B>::j(p1);
            const double a0 = cdot_part<R, B>(A, i0, j0), a1 = cdot_part<R, B>(A, i1, j1);
            // lane 0 keeps pair p0 and sends its p1 partial, lane 1 the other way round
            const double keep = blend(m0, a0, a1), send = blend(m0, a1, a0);
            const double g = keep + dpp<0xB1>(send);
            const float f = newton_f(g, blend(m0, G[i0], G[i1]), blend(m0, G[j0], G[j1]), c2);
            ok &= (int)(__builtin_fabsf(f) <= kNwtApply);  // NaN / inf fail
            fmx = __builtin_fmaxf(fmx, __builtin_fabsf(f));
            const float other = dpp<0xB1>(f);
            F[p0] = blend(m0, f, other);
            F[p1] = blend(m0, other, f);
        });
        if constexpr (NP % 2 == 1) {  // the last pair on both lanes
            constexpr int p = NP - 1, i = TriPair<B>::i(p), j = TriPair<B>::j(p);
            F[p] = newton_f(cdot<R, B, L>(A, i, j), G[i], G[j], c2);
            ok &= (int)(__builtin_fabsf(F[p]) <= kNwtApply);
            fmx = __builtin_fmaxf(fmx, __builtin_fabsf(F[p]));
        }
        ok &= dpp<0xB1>(ok);
        fmx = group_max_nonneg<2>(fmx);
    } else {
        static_for<NP>([&](auto P) {
            constexpr int p = P, i = TriPair<B>::i(p), j = TriPair<B>::j(p);
            F[p] = newton_f(cdot<R, B, L>(A, i, j), G[i], G[j], c2);
            ok &= (int)(__builtin_fabsf(F[p]) <= kNwtApply);
            fmx = __builtin_fmaxf(fmx, __builtin_fabsf(F[p]));
        });
    }
    if (__any(ok != 0)) ok &= (int)nwt_scaled_ok<B>(G, F, fmx, ok != 0);  // every lane of the block alike
    const bool take = ok != 0;
    if (__any(take)) {
        apply_f<B, L>(V, F, take);
        apply_f<B, L>(A, F, take);
    }
    return take;
}

// The same step for 4- and 8-lane blocks (b = 10..16), whose B(B-1)/2 F values do not fit
// in registers.  The pairs are visited in the sweep's round order; the lane that would
// rotate a pair (its owner) forms F_ij from the pair's dot product (8-lane blocks: summed
// through LDS in the butterfly's order, as kLdsSums) and the diagonal of G (in LDS, as
// kLdsNorms) and writes it to the block's F table in LDS, slot [round][pair].  If the
// block takes the step, every lane applies the table to its rows in newton_try()'s order
// (ascending i; pair (i, j)'s slot is a compile-time function of the schedule).  Same
// operations on the same values as newton_try(), so the same bits.
// newton_try_lds scratch (doubles from the block's nl): G at [0, B) (the norm slots), the
// pair partials at kNwtPart (8-lane blocks: kLdsSums' slots), then (floats) the F table
template <int B, int L>
constexpr int kNwtPart = L == 8 ? 32 : B;
template <int B, int L>
constexpr int kNwtTable = 2 * (kNwtPart<B, L> + (B / 2) * L);  // float offset of the F table
template <int B>
struct PairSlot {  // round and pair index of columns (i, j), i < j, in Sched<B>
    static constexpr int of(int i, int j)
    {
        for (int s = 0; s < B - 1; ++s)
            for (int p = 0; p < B / 2; ++p)
                if (Sched<B>::lo(s, p) == i && Sched<B>::hi(s, p) == j) return s * (B / 2) + p;
        return -1;
    }
};

template <int B, int L>
TMF_DEVI void apply_f_lds(double (&X)[(B + L - 1) / L][B], const float *Ft, bool take)
{
    constexpr int R = kRows<B, L>;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        float xr[B];
#pragma unroll
        for (int i = 0; i < B; ++i) xr[i] = (float)X[r][i];
        static_for<B>([&](auto J) {
            constexpr int j = J;
            // the table is read column by column (held in registers it would take B(B-1)/2 VGPRs)
            lds_order();
            float acc = 0.0f;
            static_for<B>([&](auto I) {
                constexpr int i = I;
                if constexpr (i < j) acc = __builtin_fmaf(xr[i], Ft[PairSlot<B>::of(i, j)], acc);
                else if constexpr (i > j) acc = __builtin_fmaf(-xr[i], Ft[PairSlot<B>::of(j, i)], acc);
            });
            X[r][j] = take ? X[r][j] + (double)acc : X[r][j];
        });
    }
}

template <int B, int L>
TMF_DEVI bool newton_try_lds(double (&A)[(B + L - 1) / L][B], double (&V)[(B + L - 1) / L][B], double c2, bool enable, int q,
                             double *nl)
{
    constexpr int R = kRows<B, L>, NP = B / 2, PP = (NP + L - 1) / L;
    static_assert(L >= 4 && L * PP <= 8, "4- / 8-lane blocks, at most 8 pair slots");
    double *part = nl + kNwtPart<B, L>;  // partial of pair p from lane k at part[p * L + k]
    float *Ft = reinterpret_cast<float *>(nl) + kNwtTable<B, L>;  // F of round s, pair p at Ft[s * NP + p]
    // q through an opaque move: the per-round columns / slots derived from it would
    // otherwise be hoisted out of the sweep loop and held in registers across it
    asm volatile("" : "+v"(q));
    // the scaled test's q_j and r_j (round 6) in the pair partials' slots, free after the rounds
    float *qt = reinterpret_cast<float *>(part), *rt = qt + B;
    static_assert(2 * B <= 2 * (B / 2) * L, "q, r fit the partials' slots");
    float gsum, grmin;  // the gate's S and r_min (nwt_gate), from the diagonal of G
    {
        double G[B];
        static_for<B>([&](auto K) { G[K] = cdot_part<R, B>(A, K, K); });
        static_for<B>([&](auto K) { G[K] = group_sum<L>(G[K]); });
        lds_order();
        if (q == 0) static_for<B>([&](auto K) { nl[K] = G[K]; });
        lds_order();
        double gmax = 0.0;
#pragma unroll
        for (int k = 0; k < B; ++k) gmax = G[k] > gmax ? G[k] : gmax;
        const float ginv = 1.0f / (float)gmax;
        gsum = 0.0f;
        grmin = 1.0f;
#pragma unroll
        for (int k = 0; k < B; ++k) {
            const float r = (float)G[k] * ginv;
            gsum += r;
            grmin = __builtin_fminf(grmin, r);
        }
    }
    int ok = 1;
    float fmx = 0.0f;  // this lane's largest |F|
    static_for<B - 1>([&](auto S) {
        constexpr int s = S;
        // the rounds are independent (A is not modified): without a fence the scheduler
        // interleaves them and runs out of registers
        __builtin_amdgcn_sched_barrier(0);
        double ga[NP];
        static_for<NP>([&](auto Pi) { ga[Pi] = cdot_part<R, B>(A, Sched<B>::lo(s, Pi), Sched<B>::hi(s, Pi)); });
        lds_order();  // after the previous round's reads
        static_for<NP>([&](auto Pi) { part[Pi * L + q] = ga[Pi]; });
        lds_order();
        static_for<PP>([&](auto U) {
            const int pq = q * PP + U;  // this lane's U-th pair of the round (none if >= NP)
            const bool has = pq < NP;
            const int i = (int)__builtin_amdgcn_ubfe(sched_nibbles<B, s, false>(), 4 * pq, 4);
            const int j = (int)__builtin_amdgcn_ubfe(sched_nibbles<B, s, true>(), 4 * pq, 4);
            // the butterfly's order (group_sum): ((p0+p1)+(p2+p3)) [+ ((p4+p5)+(p6+p7))]
            const double *pp = part + (has ? pq : 0) * L;
            double g = (pp[0] + pp[1]) + (pp[2] + pp[3]);
            if constexpr (L == 8) g = g + ((pp[4] + pp[5]) + (pp[6] + pp[7]));
            const double a = nl[i], b = nl[j], g2 = g * g;  // slot 15 (no pair): a dummy read
            const bool rot = has && !((g2 <= c2 * (a + b)) | (g2 <= (JacP<double>::kTol2 * a) * b));
            const float f = rot ? (float)g / (float)(b - a) : 0.0f;
            ok &= (int)(__builtin_fabsf(f) <= kNwtApply);  // NaN / inf fail
            fmx = __builtin_fmaxf(fmx, __builtin_fabsf(f));
            if (has) Ft[s * NP + pq] = f;
        });
    });
    ok = enable && group_or<L>(1 - ok) == 0 ? 1 : 0;
    fmx = group_max_nonneg<L>(fmx);
    const bool gate = nwt_gate(fmx, gsum, grmin);  // decides for the block: no sums
    if (__any(ok != 0 && !gate)) {
        // the scaled test: every lane reads the block's q and r (the owners' updates are done);
        // the pair tests, if the screen does not decide, each lane on the pairs it owns
        lds_order();  // after the owners' table writes and the last round's partial reads
        if (q == 0) {
            double gmax = 0.0;
            static_for<B>([&](auto K) { gmax = nl[K] > gmax ? nl[K] : gmax; });
            const float ginv = 1.0f / (float)gmax;
            static_for<B>([&](auto K) {
                rt[K] = (float)nl[K] * ginv;
                qt[K] = 0.0f;
            });
        }
        lds_order();
        {
            int qq = q;
            asm volatile("" : "+v"(qq));  // the pairs' columns derived here, not hoisted
            // q_j in the round order: each column is in one pair of a round, whose owner updates it
            static_for<B - 1>([&](auto S) {
                constexpr int s = S;
                lds_order();  // after the previous round's updates
                static_for<PP>([&](auto U) {
                    const int pq = qq * PP + U;
                    const int i = (int)__builtin_amdgcn_ubfe(sched_nibbles<B, s, false>(), 4 * pq, 4);
                    const int j = (int)__builtin_amdgcn_ubfe(sched_nibbles<B, s, true>(), 4 * pq, 4);
                    if (pq < NP) {
                        const float x2 = nwt_x2(Ft[s * NP + pq]);
                        qt[i] = __builtin_fmaf(x2, rt[j], qt[i]);
                        qt[j] = __builtin_fmaf(x2, rt[i], qt[j]);
                    }
                });
            });
        }
        lds_order();
        int pass = 1;
#pragma unroll
        for (int jj = 0; jj < (B + L - 1) / L; ++jj) {
            const int j = q + jj * L;
            if (j < B) pass &= (int)nwt_col_ok(qt[j], rt[j]);
        }
        pass = group_or<L>(1 - pass) == 0 ? 1 : 0;
        if (__any(pass == 0)) {
            pass = 1;
            int qq = q;
            asm volatile("" : "+v"(qq));  // the pairs' columns derived here, not hoisted
            static_for<B - 1>([&](auto S) {
                constexpr int s = S;
                lds_order();  // one round's reads at a time
                static_for<PP>([&](auto U) {
                    const int pq = qq * PP + U;
                    const int i = (int)__builtin_amdgcn_ubfe(sched_nibbles<B, s, false>(), 4 * pq, 4);
                    const int j = (int)__builtin_amdgcn_ubfe(sched_nibbles<B, s, true>(), 4 * pq, 4);
                    if (pq < NP) pass &= (int)nwt_pair_ok(qt[i], qt[j], rt[i], rt[j]);
                });
            });
            pass = group_or<L>(1 - pass) == 0 ? 1 : 0;
        }
        ok &= pass;
    }
    const bool take = ok != 0;
    if (__any(take)) {
        lds_order();  // after the owners' table writes
        apply_f_lds<B, L>(V, Ft, take);
        apply_f_lds<B, L>(A, Ft, take);
    }
    lds_order();  // before the tile's next use
    return take;
}

// oracle jacobi_newton(): returns sweeps | (Newton steps << 16).  nl: the block's LDS
// scratch (b >= 10; see newton_try_lds).  defer_max > 0 (the embed kernel's strip pass,
// DESIGN.md 4): once no more than defer_max blocks of the wave are still unfinished after a
// sweep and its Newton try, the wave stops and *unfinished tells each block whether it was
// one of them -- the list pass redoes those from their pixels with the whole loop, so their
// bits are those of the uninterrupted loop (a block's arithmetic never depends on the other
// blocks of its wave).
template <int B, int L>
TMF_DEVI int jacobi_newton(double (&A)[(B + L - 1) / L][B], double (&V)[(B + L - 1) / L][B], int q, double *nl = nullptr,
                           int defer_max = 0, bool *unfinished = nullptr)
{
    const double c2 = JacP<double>::kC2 * frob2<double, B, L>(A);
    bool active = true;
    int sweeps = 0, newton = 0;
    for (int it = 0; it < JacP<double>::kMaxSweeps; ++it) {
        const int rotated = jacobi_sweep<double, B, L, true>(A, V, q, nl, c2, 0.0, active);
        sweeps += active ? 1 : 0;
        active = active && group_or<L>(rotated) != 0;
        if (!__any(active)) break;
        bool took;
        if constexpr (L >= 4) took = newton_try_lds<B, L>(A, V, c2, active, q, nl);
        else took = newton_try<B, L>(A, V, c2, active);
        if (took) {
            newton = 1;
            active = false;
        }
        if (!__any(active)) break;
        if (defer_max > 0 && __builtin_popcountll(__ballot(active && q == 0)) <= defer_max) {
            if (unfinished) *unfinished = active;
            break;
        }
    }
    return sweeps | (newton << 16);
}

// Phase 2 (oracle bjorck()): V <- V N, N = 1.5 I - 0.5 V^T V.  N is symmetric and
// cdot(V, j, k) == cdot(V, k, j) bitwise, so only the upper triangle is computed.
template <int B, int L>
TMF_DEVI void bjorck(double (&V)[(B + L - 1) / L][B])
{
    constexpr int R = kRows<B, L>;
    if constexpr (B > 8) {  // 136 packed doubles would not fit in registers: column by column
        double T[R][B];
        static_for<B>([&](auto K) {
            constexpr int k = K;
            double n[B];
            static_for<B>([&](auto J) {
                constexpr int j = J;
                const double qv = cdot<R, B, L>(V, j, k);
                n[j] = (j == k) ? __builtin_fma(-0.5, qv, 1.5) : -0.5 * qv;
            });
#pragma unroll
            for (int r = 0; r < R; ++r) {
                double acc = 0.0;
#pragma unroll
                for (int j = 0; j < B; ++j) acc = __builtin_fma(V[r][j], n[j], acc);
                T[r][k] = acc;
            }
        });
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int k = 0; k < B; ++k) V[r][k] = T[r][k];
        return;
    }
    double N[B * (B + 1) / 2];  // packed upper triangle, row j: N[j][k], k >= j
    static_for<B>([&](auto J) {     // lane-local chains first, cross-lane sums after (cdot)
        constexpr int j = J;
        static_for<B - j>([&](auto K0) {
            constexpr int k = j + K0, idx = j * B - j * (j - 1) / 2 + K0;
            N[idx] = cdot_part<R, B>(V, j, k);
        });
    });
    static_for<B>([&](auto J) {
        constexpr int j = J;
        static_for<B - j>([&](auto K0) {
            constexpr int k = j + K0, idx = j * B - j * (j - 1) / 2 + K0;
            const double qv = group_sum<L>(N[idx]);
            N[idx] = (j == k) ? __builtin_fma(-0.5, qv, 1.5) : -0.5 * qv;
        });
    });
    double T[R][B];
    static_for<B>([&](auto K) {
        constexpr int k = K;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            double acc = 0.0;
            static_for<B>([&](auto J) {
                constexpr int j = J, lo = j < k ? j : k, hi = j < k ? k : j;
                acc = __builtin_fma(V[r][j], N[lo * B - lo * (lo - 1) / 2 + (hi - lo)], acc);
            });
            T[r][k] = acc;
        }
    });
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int k = 0; k < B; ++k) V[r][k] = T[r][k];
}

// A0 = D V (oracle: fma chain over j = 0..b-1); row j of V comes from lane j / R.
template <int B, int L>
TMF_DEVI void mul_dv(const float (&D)[(B + L - 1) / L][B], const double (&V)[(B + L - 1) / L][B], double (&A)[(B + L - 1) / L][B])
{
    constexpr int R = kRows<B, L>;
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int k = 0; k < B; ++k) A[r][k] = 0.0;
    static_for<B>([&](auto J) {
        constexpr int j = J, src = j / R, jr = j % R;
        double vrow[B];
#pragma unroll
        for (int k = 0; k < B; ++k) vrow[k] = group_bcast<L, src>(V[jr][k]);
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int k = 0; k < B; ++k) A[r][k] = __builtin_fma((double)D[r][j], vrow[k], A[r][k]);
    });
}

// Full SVD of this lane's rows of D (oracle orc_svd_block, phases 1-3): on return A
// holds A V (columns = sigma_k u_k), V the right singular vectors (unsorted).
// Returns f64 sweeps | (f32 sweeps << 8) of this block.
struct NoStamp {
    TMF_DEVI void operator()(int) const {}
};

// nl: this block's LDS scratch for the column norms (kLdsNorms<L>), the broadcast rotation
// parameters (kLdsBcast<L>), the pair partials (kLdsSums<L>) and the Newton table
// (newton_try_lds, b >= 10): kScratchFloats<B, L> floats, 8-byte aligned (unused at L <= 2)
template <int B, int L>
constexpr int kScratchFloats = L <= 2 ? 2 : kNwtTable<B, L> + (B - 1) * (B / 2);
// PARK (4- / 8-lane blocks): D waits for A0 = D V0 in LDS, at park (the lane's rows,
// row-major b x b, from kParkOff<L> floats into the block's scratch: past phase 1's
// parameter slots), instead of in 32-36 registers that the f32 phase needs.
template <int L>
constexpr int kParkOff = L == 8 ? 32 : 0;
template <int B, int L, bool PARK = false, typename Stamp = NoStamp>
TMF_DEVI int svd3(const float (&D)[(B + L - 1) / L][B], double (&A)[(B + L - 1) / L][B], double (&V)[(B + L - 1) / L][B], int q,
                  Stamp stamp = {}, void *nl = nullptr, float *park = nullptr, int defer_max = 0, bool *unfinished = nullptr)
{
    constexpr int R = kRows<B, L>;
    if constexpr (PARK) {
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (q * R + r < B)
#pragma unroll
                for (int c = 0; c < B; ++c) park[(q * R + r) * B + c] = D[r][c];
    }
    int s32;
    {
        float A32[R][B], V32[R][B];
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int c = 0; c < B; ++c) {
                A32[r][c] = D[r][c];
                V32[r][c] = (q * R + r == c) ? 1.0f : 0.0f;
            }
        s32 = jacobi<float, B, L, true>(A32, V32, q, static_cast<float *>(nl));
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int c = 0; c < B; ++c) V[r][c] = (double)V32[r][c];
    }
    stamp(1);
    bjorck<B, L>(V);
    bjorck<B, L>(V);
    if constexpr (PARK) {
        lds_order();  // read back here, not earlier
        float Dp[R][B];
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int c = 0; c < B; ++c) Dp[r][c] = q * R + r < B ? park[(q * R + r) * B + c] : 0.0f;
        mul_dv<B, L>(Dp, V, A);
    } else {
        mul_dv<B, L>(D, V, A);
    }
    stamp(2);
    lds_order();
    int s64;
    s64 = jacobi_newton<B, L>(A, V, q, static_cast<double *>(nl), defer_max, unfinished);
    stamp(3);
    return s64 | (s32 << 8);
}

// ---------------------------------------------------------------------------
// Certified f32(sigma_1) for the extract path.  An f32 power
// iteration on D^T D gives a vector v; in f64 the Rayleigh quotient rho and the
// residual bound the top eigenvalue of D^T D by Kato-Temple:
//     lambda_1 in [rho, rho + |r|^2 / (2 rho - F)]      (needs 2 rho > F = |D|_F^2,
// since lambda_2 <= F - lambda_1 <= F - rho).  Every f64 rounding is covered by
// generous unit-roundoff margins, and the enclosure is widened by a further 2^-45
// (relative) so that it also contains LAPACK's and the oracle's f64 sigma_1.
// If both ends round to the same float, that float IS f32(sigma_1) of the
// reference; otherwise the caller falls back to the exact Jacobi.
// The enclosure holds for any v.  At b = 4 one lane holds the whole block, and v comes from
// SQITERS products with (D^T D / tr)^4, four power steps each, not ITERS single steps: the strip
// pass's 3 steps become 4, the list pass's 8 stay 8, for fewer undecided blocks at about the same
// cost (extract<4> -9 % on noise covers, -1 % on camera-like ones, identical bytes).
// ---------------------------------------------------------------------------
template <int B, int L, int ITERS, int NI, int SQITERS = (ITERS + 3) / 4>
TMF_DEVI void sigma1_certified(const float (&x)[NI][(B + L - 1) / L][B], float (&s1)[NI], bool (&ok)[NI])
{
    // NI images side by side: the same operations per image, interleaved, so that the
    // dependent chains of one image's power iteration overlap the other's
    constexpr int R = kRows<B, L>;
    constexpr double u = 1.1102230246251565e-16;  // 2^-53
    float v[NI][B];
#pragma unroll
    for (int m = 0; m < NI; ++m)
#pragma unroll
        for (int j = 0; j < B; ++j) v[m][j] = j == 0 ? 1.0f : 0.0f;
    if constexpr (B == 4 && L == 1) {
        // one lane holds the block: power steps with (D^T D / tr)^4, four steps per product
#pragma unroll
        for (int m = 0; m < NI; ++m) {
            float M[4][4], M2[4][4], M4[4][4], tr = 0.0f;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = i; j < 4; ++j) {
                    float acc = 0.0f;
#pragma unroll
                    for (int r = 0; r < 4; ++r) acc = __builtin_fmaf(x[m][r][i], x[m][r][j], acc);
                    M[i][j] = M[j][i] = acc;
                }
#pragma unroll
            for (int i = 0; i < 4; ++i) tr += M[i][i];
            const float sc = tr > 1e-30f ? 1.0f / tr : 1.0f;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) M[i][j] *= sc;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = i; j < 4; ++j) {
                    float acc = 0.0f;
#pragma unroll
                    for (int k = 0; k < 4; ++k) acc = __builtin_fmaf(M[i][k], M[k][j], acc);
                    M2[i][j] = M2[j][i] = acc;
                }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = i; j < 4; ++j) {
                    float acc = 0.0f;
#pragma unroll
                    for (int k = 0; k < 4; ++k) acc = __builtin_fmaf(M2[i][k], M2[k][j], acc);
                    M4[i][j] = M4[j][i] = acc;
                }
#pragma unroll
            for (int it = 0; it < SQITERS; ++it) {
                float w[4], nn = 0.0f;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    float acc = 0.0f;
#pragma unroll
                    for (int j = 0; j < 4; ++j) acc = __builtin_fmaf(M4[i][j], v[m][j], acc);
                    w[i] = acc;
                    nn = __builtin_fmaf(acc, acc, nn);
                }
                const bool live = nn > 1e-30f;
                const float inv = __builtin_amdgcn_rsqf(live ? nn : 1.0f);
#pragma unroll
                for (int j = 0; j < 4; ++j) v[m][j] = live ? w[j] * inv : v[m][j];
            }
        }
    } else
#pragma unroll
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int m = 0; m < NI; ++m) {
            float uu[R];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                float acc = 0.0f;
#pragma unroll
                for (int j = 0; j < B; ++j) acc = __builtin_fmaf(x[m][r][j], v[m][j], acc);
                uu[r] = acc;
            }
            float w[B], nn = 0.0f;
#pragma unroll
            for (int j = 0; j < B; ++j) {
                float acc = 0.0f;
#pragma unroll
                for (int r = 0; r < R; ++r) acc = __builtin_fmaf(x[m][r][j], uu[r], acc);
                w[j] = group_sum<L>(acc);
                nn = __builtin_fmaf(w[j], w[j], nn);
            }
            const bool live = nn > 1e-30f;
            const float inv = __builtin_amdgcn_rsqf(live ? nn : 1.0f);
#pragma unroll
            for (int j = 0; j < B; ++j) v[m][j] = live ? w[j] * inv : v[m][j];
        }
    }
#pragma unroll
    for (int m = 0; m < NI; ++m) {
        double Fp = 0.0;
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int j = 0; j < B; ++j) Fp = __builtin_fma((double)x[m][r][j], (double)x[m][r][j], Fp);
        const double F = group_sum<L>(Fp);
        double vd[B], nv = 0.0;
#pragma unroll
        for (int j = 0; j < B; ++j) {
            vd[j] = (double)v[m][j];
            nv = __builtin_fma(vd[j], vd[j], nv);
        }
        double ud[R], ap = 0.0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            double acc = 0.0;
#pragma unroll
            for (int j = 0; j < B; ++j) acc = __builtin_fma((double)x[m][r][j], vd[j], acc);
            ud[r] = acc;
            ap = __builtin_fma(acc, acc, ap);
        }
        const double a = group_sum<L>(ap);
        const double rho = a / nv;
        double rn2 = 0.0;
#pragma unroll
        for (int j = 0; j < B; ++j) {
            double acc = 0.0;
#pragma unroll
            for (int r = 0; r < R; ++r) acc = __builtin_fma((double)x[m][r][j], ud[r], acc);
            const double rj = group_sum<L>(acc) - rho * vd[j];
            rn2 = __builtin_fma(rj, rj, rn2);
        }
        const double rr0 = __builtin_sqrt(rn2 / nv) * (1.0 + 16.0 * u) + 256.0 * u * F;
        const double rr = rr0 * rr0;
        const double rlo = rho * (1.0 - 256.0 * u);
        const double fhi = F * (1.0 + 256.0 * u);
        const double gap = (rlo + rlo) - fhi;
        const double hi = (rho + rr / (gap > 0.0 ? gap : 1.0)) * (1.0 + 256.0 * u);
        const double slo = __builtin_sqrt(rlo) * (1.0 - 512.0 * u);
        const double shi = __builtin_sqrt(hi) * (1.0 + 512.0 * u);
        s1[m] = F == 0.0 ? 0.0f : (float)slo;
        ok[m] = F == 0.0 || (gap > 0.0 && (float)shi == (float)slo && rho == rho);
    }
}

}  // namespace tmf
