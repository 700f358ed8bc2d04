// Study (tools/exp): byte-level rounding certificate for the hybrid route.
//
// Per block, from the Jacobi route's f64 factors (oracle svd_blocks_f64) and a bound
// E_k = K 2^-53 sigma_1 / m_k on how far LAPACK's f64 factors can sit from them
// (sigma: K 2^-53 sigma_1), carry intervals through every rounding of the reference's
// own pipeline after the SVD:
//   f32 factors (RN of the interval ends), S'[0] = f32(f64(S0) + alpha w / 255),
//   B = S' * Vt (f32), M = fmaf chain over k (watermarking.py:201, OpenBLAS sgemm order),
//   the pocketfft fp32 IDCT (every op is an RN add / sub / multiply by a constant, monotone
//   in each operand: swap the ends on subtraction and on negative constants),
//   and the inverse colour (monotone in Y for the pixel's fixed Cb / Cr).
// A block is certified when every channel byte is the same at both ends of its Y interval.
// Build: g++ -O2 -fopenmp -ffp-contract=off -shared -fPIC -I thatsmyface_amd/csrc
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>

#include "tmfwm_consts.h"

namespace {

struct Iv {
    float lo, hi;
};
inline Iv operator+(Iv a, Iv b) { return {a.lo + b.lo, a.hi + b.hi}; }
inline Iv operator-(Iv a, Iv b) { return {a.lo - b.hi, a.hi - b.lo}; }
inline Iv operator-(Iv a) { return {-a.hi, -a.lo}; }
inline Iv operator*(float c, Iv a) { return c >= 0.0f ? Iv{c * a.lo, c * a.hi} : Iv{c * a.hi, c * a.lo}; }
inline Iv operator*(Iv a, float c) { return c * a; }
inline Iv &operator*=(Iv &a, float c) { return a = c * a; }

constexpr float kSqrt2 = 1.41421356237309504880f;
constexpr float kHsqt2 = 0.70710678118654752440f;

template <int IDO, int L1, int N, typename T>
void radf2(const T (&cc)[N], T (&ch)[N], const float *wa)
{
#define CC(a, b, c) cc[(a) + IDO * ((b) + L1 * (c))]
#define CH(a, b, c) ch[(a) + IDO * ((b) + 2 * (c))]
    for (int k = 0; k < L1; k++) {
        const T x = CC(0, k, 0), y = CC(0, k, 1);
        CH(0, 0, k) = x + y;
        CH(IDO - 1, 1, k) = x - y;
    }
    if ((IDO & 1) == 0)
        for (int k = 0; k < L1; k++) {
            CH(0, 1, k) = -CC(IDO - 1, k, 1);
            CH(IDO - 1, 0, k) = CC(IDO - 1, k, 0);
        }
    if (IDO > 2)
        for (int k = 0; k < L1; k++)
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
#undef CC
#undef CH
}

template <int IDO, int L1, int N, typename T>
void radf4(const T (&cc)[N], T (&ch)[N], const float *wa)
{
#define CC(a, b, c) cc[(a) + IDO * ((b) + L1 * (c))]
#define CH(a, b, c) ch[(a) + IDO * ((b) + 4 * (c))]
    for (int k = 0; k < L1; k++) {
        T a = CC(0, k, 3), b = CC(0, k, 1);
        const T tr1 = a + b;
        CH(0, 2, k) = a - b;
        a = CC(0, k, 0);
        b = CC(0, k, 2);
        const T tr2 = a + b;
        CH(IDO - 1, 1, k) = a - b;
        CH(0, 0, k) = tr2 + tr1;
        CH(IDO - 1, 3, k) = tr2 - tr1;
    }
    if ((IDO & 1) == 0)
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
    if (IDO > 2)
        for (int k = 0; k < L1; k++)
            for (int i = 2; i < IDO; i += 2) {
                const int ic = IDO - i;
                float w0 = wa[i - 2], w1 = wa[i - 1];
                T e = CC(i - 1, k, 1), f = CC(i, k, 1);
                const T cr2 = w0 * e + w1 * f, ci2 = w0 * f - w1 * e;
                w0 = wa[(IDO - 1) + i - 2];
                w1 = wa[(IDO - 1) + i - 1];
                e = CC(i - 1, k, 2);
                f = CC(i, k, 2);
                const T cr3 = w0 * e + w1 * f, ci3 = w0 * f - w1 * e;
                w0 = wa[2 * (IDO - 1) + i - 2];
                w1 = wa[2 * (IDO - 1) + i - 1];
                e = CC(i - 1, k, 3);
                f = CC(i, k, 3);
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
#undef CC
#undef CH
}

template <int N> struct Tw;
template <> struct Tw<8> { static constexpr const float *d = kDctTw8; static constexpr float norm = kNorm8; };
template <> struct Tw<16> { static constexpr const float *d = kDctTw16; static constexpr float norm = kNorm16; };

template <int N, typename T>
void rfft_forward(T (&c)[N], float fct)
{
    T ch[N];
    if constexpr (N == 8) {
        radf4<1, 2>(c, ch, nullptr);
        radf2<4, 1>(ch, c, kRfftTw8);
    } else {
        radf4<1, 4>(c, ch, nullptr);
        radf4<4, 1>(ch, c, kRfftTw16);
    }
    for (int i = 0; i < N; ++i) c[i] *= fct;
}

template <int N, typename T>
void dct3(T (&c)[N])
{
    constexpr int NS2 = (N + 1) / 2;
    const float *tw = Tw<N>::d;
    c[0] *= kSqrt2;
    for (int k = 1; k < NS2; ++k) {
        const int kc = N - k;
        const T t1 = c[k] + c[kc], t2 = c[k] - c[kc];
        c[k] = tw[k - 1] * t2 + tw[kc - 1] * t1;
        c[kc] = tw[k - 1] * t1 - tw[kc - 1] * t2;
    }
    c[NS2] *= 2.0f * tw[NS2 - 1];
    rfft_forward<N>(c, Tw<N>::norm);
    for (int k = 1; k < N - 1; k += 2) {
        const T t = c[k];
        c[k] = t - c[k + 1];
        c[k + 1] = t + c[k + 1];
    }
}

inline uint32_t u8_from_unit(float f)
{
    if (f < 0.0f) f = 0.0f;
    if (f > 1.0f) f = 1.0f;
    return (uint32_t)(f * 255.0f);
}

inline void colour_inv(float y, float cbs, float crs, uint32_t out[3])
{
    const float cbp = cbs - 0.5f, crp = crs - 0.5f;
    const double Y = y, CB = cbp, CR = crp;
    out[0] = u8_from_unit((float)fma(1.403, CR, fma(1.0, Y, 0.0 * CB)));
    out[1] = u8_from_unit((float)fma(-0.714, CR, fma(1.0, Y, -0.344 * CB)));
    out[2] = u8_from_unit((float)fma(0.0, CR, fma(1.0, Y, 1.773 * CB)));
}

inline Iv f32_iv(double x, double e)
{
    double lo = x - e, hi = x + e;
    if (lo < -2.0) lo = -2.0;
    if (hi > 2.0) hi = 2.0;
    return {(float)lo, (float)hi};
}

// one block; returns 1 when some byte is uncertain.  stats[0]: uncertain M elements,
// stats[1]: uncertain Y elements.
template <int N>
int cert_block(const double *U, const double *sig, const double *V, uint32_t w, double alpha, const float *cb,
               const float *cr, double K, uint8_t *bytes, int64_t *stats)
{
    double s1 = 0.0;
    for (int k = 0; k < N; ++k) s1 = std::max(s1, sig[k]);
    // m_k = min(sigma_k, gap_k) (oracle orc_svd_flag's quantities)
    double E[N];
    for (int k = 0; k < N; ++k) {
        double g = sig[k];
        for (int j = 0; j < N; ++j)
            if (j != k) g = std::min(g, fabs(sig[k] - sig[j]));
        E[k] = g > 0.0 ? K * 0x1p-53 * s1 / g : 4.0;
    }
    const double Es = K * 0x1p-53 * s1;
    // sorted descending already (svd_blocks_f64); factor intervals
    Iv Ui[N][N], Bi[N][N];
    Iv S[N];
    for (int k = 0; k < N; ++k) {
        double lo = sig[k] - Es, hi = sig[k] + Es;
        if (lo < 0.0) lo = 0.0;
        S[k] = {(float)lo, (float)hi};
    }
    const double c = alpha * ((double)w / 255.0);
    S[0] = {(float)((double)S[0].lo + c), (float)((double)S[0].hi + c)};
    for (int r = 0; r < N; ++r)
        for (int k = 0; k < N; ++k) Ui[r][k] = s1 == 0.0 ? Iv{r == k ? 1.0f : 0.0f, r == k ? 1.0f : 0.0f} : f32_iv(U[r * N + k], E[k]);
    for (int k = 0; k < N; ++k)
        for (int j = 0; j < N; ++j) {
            const Iv v = s1 == 0.0 ? Iv{j == k ? 1.0f : 0.0f, j == k ? 1.0f : 0.0f} : f32_iv(V[j * N + k], E[k]);  // Vt[k][j] = V[j][k]
            const float a = S[k].lo * v.lo, b = S[k].lo * v.hi, d = S[k].hi * v.lo, e = S[k].hi * v.hi;
            Bi[k][j] = {std::min(std::min(a, b), std::min(d, e)), std::max(std::max(a, b), std::max(d, e))};
        }
    int unc = 0;
    for (int k = 0; k < N; ++k) {
        unc |= S[k].lo != S[k].hi;
        for (int j = 0; j < N; ++j) unc |= (Ui[j][k].lo != Ui[j][k].hi) | (Bi[k][j].lo != Bi[k][j].hi);
    }
    stats[2] += unc;
    Iv M[N][N];
    for (int i = 0; i < N; ++i)
        for (int j = 0; j < N; ++j) {
            Iv acc = {0.0f, 0.0f};
            for (int t = 0; t < N; ++t) {
                const Iv u = Ui[i][t], b = Bi[t][j];
                const float l1 = fmaf(u.lo, b.lo, acc.lo), l2 = fmaf(u.lo, b.hi, acc.lo), l3 = fmaf(u.hi, b.lo, acc.lo),
                            l4 = fmaf(u.hi, b.hi, acc.lo);
                const float h1 = fmaf(u.lo, b.lo, acc.hi), h2 = fmaf(u.lo, b.hi, acc.hi), h3 = fmaf(u.hi, b.lo, acc.hi),
                            h4 = fmaf(u.hi, b.hi, acc.hi);
                acc = {std::min(std::min(l1, l2), std::min(l3, l4)), std::max(std::max(h1, h2), std::max(h3, h4))};
            }
            M[i][j] = acc;
            stats[0] += acc.lo != acc.hi;
        }
    // IDCT: columns (axis 0) first, then rows
    for (int j = 0; j < N; ++j) {
        Iv col[N];
        for (int i = 0; i < N; ++i) col[i] = M[i][j];
        dct3<N>(col);
        for (int i = 0; i < N; ++i) M[i][j] = col[i];
    }
    int fail = 0;
    for (int i = 0; i < N; ++i) {
        dct3<N>(M[i]);
        for (int j = 0; j < N; ++j) {
            const Iv y = M[i][j];
            stats[1] += y.lo != y.hi;
            uint32_t lo[3], hi[3];
            colour_inv(y.lo, cb[i * N + j], cr[i * N + j], lo);
            colour_inv(y.hi, cb[i * N + j], cr[i * N + j], hi);
            for (int ch = 0; ch < 3; ++ch) {
                bytes[(i * N + j) * 3 + ch] = (uint8_t)lo[ch];
                fail |= lo[ch] != hi[ch];
            }
        }
    }
    return fail;
}

}  // namespace

extern "C" int cert_blocks(int64_t nb, int b, const double *U, const double *sig, const double *V, const uint8_t *w,
                           double alpha, const float *cb, const float *cr, double K, uint8_t *flag, uint8_t *bytes,
                           int64_t *stats)
{
    if (b != 8 && b != 16) return -1;
    int64_t s0 = 0, s1 = 0, s2 = 0;
#pragma omp parallel for schedule(dynamic, 256) reduction(+ : s0, s1, s2)
    for (int64_t n = 0; n < nb; ++n) {
        const int64_t o = n * b * b;
        int64_t st[3] = {0, 0, 0};
        flag[n] = (uint8_t)(b == 8 ? cert_block<8>(U + o, sig + n * b, V + o, w[n], alpha, cb + o, cr + o, K, bytes + 3 * o, st)
                                   : cert_block<16>(U + o, sig + n * b, V + o, w[n], alpha, cb + o, cr + o, K, bytes + 3 * o, st));
        s0 += st[0];
        s1 += st[1];
        s2 += st[2];
    }
    stats[0] = s0;
    stats[1] = s1;
    stats[2] = s2;
    return 0;
}
