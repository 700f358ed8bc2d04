/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY (see tmfwm_oracle.c).
 *
 * The hybrid route's byte certificate.  The reference's embed bytes
 * come from U, S, Vt = f32(dgesdd(f64(D))) (watermarking.py:195) through
 *   S'[0] = f32(f64(S[0]) + alpha w / 255)                 (:198)
 *   M = U @ (diag(S') @ Vt), sequential fmaf chains (:201, OpenBLAS sgemm order)
 *   Y = pocketfft fp32 IDCT of M                          (:204)
 *   bytes = ycbcr_to_rgb(Y, Cb, Cr)                       (:216)
 * The Jacobi route knows LAPACK's f64 factors only up to a bound: every element of the
 * triplet k within E_k = K 2^-53 sigma_1 / m_k (m_k = min(sigma_k, gap_k)), every sigma
 * within Es = K 2^-53 sigma_1, K = 256 (tools/exp/cert_study.py: LAPACK's own V is off by up
 * to 94 such units from the exact factors, the Jacobi route's by up to 30).  Every later
 * step is an IEEE round-to-nearest operation, monotone in each operand, so carrying
 * [lo, hi] through each of them with the end points computed by the same operation
 * (exact corners for the fmaf chain, swapped ends for subtractions and negative constants)
 * encloses every value the reference can produce.  The inverse colour is monotone in Y
 * for the pixel's fixed Cb / Cr, so a block whose bytes agree at both ends of every Y
 * interval has the reference's bytes; any other block takes the dgesdd route.
 *
 * Contract (the device's embed_kernel computes the same end points bit for bit):
 *   s1 = max sigma_k; s1 == 0: certain (zero block, N6);
 *   D zero but for D[0][0] (a flat block): certain -- dgebd2's reflectors are identities
 *     (tau = 0), dbdsqr only makes d_1 positive: U = I, S = |d|, Vt = diag(sgn d, 1, ..) in
 *     LAPACK, U e_0 = sgn(d) e_0, V = I here, and every other product of the chain is a zero
 *     added to +0, so both routes' M are the same bits;
 *   uncertain (the dgesdd route) when an element interval of a triplet that reaches the output
 *     contains 0 (lo < 0 < hi) and some element interval of the block is not a point: the
 *     device's end-point selection is exact unless a rank has both on the two sides of the
 *     product, and this block-level test covers that (exact zeros of structured blocks);
 *   keep_k = f32(sigma_k) != 0, g_k = min(sigma_k, min_{j != k} |sigma_k - sigma_j|),
 *   E_k = f32(t / g_k) (keep_k; t = 2^-45 s1; in [2^-45, 2^-25] when the conditioning test
 *         passes: held as a float on the device), Es = t;
 *   S_k in [f32(max(sigma_k - Es, 0)), f32(sigma_k + Es)]; S'_0 ends f32(f64(end) + c);
 *   keep_k:  U_rk in [f32(u - E_k), f32(u + E_k)], V_jk likewise, B_kj = S'_k x V_jk
 *            (S' >= 0: lo = S'lo v_lo if v_lo >= 0 else S'hi v_lo; hi = S'lo v_hi if
 *            v_hi <= 0 else S'hi v_hi);
 *   !keep_k: U_rk = [2, 2], B_kj = [-2 S'hi_k, 2 S'hi_k]  (|f32 factor entries| <= 1);
 *   M chain: acc = [0, 0]; acc = [min, max] over the four corners of fmaf(u, b, acc.lo / hi);
 *   IDCT and colour as the reference, on both ends.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>

#include "orc_plan.h"

namespace {

struct Iv {
    float lo, hi;
};
inline Iv operator+(Iv a, Iv b) { return {a.lo + b.lo, a.hi + b.hi}; }
inline Iv operator-(Iv a, Iv b) { return {a.lo - b.hi, a.hi - b.lo}; }
inline Iv operator-(Iv a) { return {-a.hi, -a.lo}; }
inline Iv operator*(float c, Iv a) { return c >= 0.0f ? Iv{c * a.lo, c * a.hi} : Iv{c * a.hi, c * a.lo}; }
inline Iv operator*(Iv a, float c) { return c * a; }
inline Iv &operator+=(Iv &a, Iv b) { return a = a + b; }
inline Iv &operator*=(Iv &a, float c) { return a = c * a; }

const float SQRT2F = 1.41421356237309504880f;
const float HSQT2F = 0.70710678118654752440f;
const float TAUR = -0.5f, TAUI = 0.8660254037844386467637231707529362f;
const float TR11 = 0.3090169943749474241022934171828191f, TI11 = 0.9510565162951535721164393333793821f;
const float TR12 = -0.8090169943749474241022934171828191f, TI12 = 0.5877852522924731291687059546390728f;

/* the forward rfftp passes of tmfwm_oracle.c, over a value type T (same statements) */
template <typename T>
void pm(T &a, T &b, T c, T d)
{
    a = c + d;
    b = c - d;
}
template <typename T>
void mulpm(T &a, T &b, float c, float d, T e, T f)
{
    a = c * e + d * f;
    b = c * f - d * e;
}

template <typename T>
void radf2(int ido, int l1, const T *cc, T *ch, const float *wa)
{
#define CC(a, b, c) cc[(a) + ido * ((b) + l1 * (c))]
#define CH(a, b, c) ch[(a) + ido * ((b) + 2 * (c))]
#define WA(x, i) wa[(i) + (x) * (ido - 1)]
    for (int k = 0; k < l1; k++) pm(CH(0, 0, k), CH(ido - 1, 1, k), CC(0, k, 0), CC(0, k, 1));
    if ((ido & 1) == 0)
        for (int k = 0; k < l1; k++) {
            CH(0, 1, k) = -CC(ido - 1, k, 1);
            CH(ido - 1, 0, k) = CC(ido - 1, k, 0);
        }
    if (ido <= 2) return;
    for (int k = 0; k < l1; k++)
        for (int i = 2; i < ido; i += 2) {
            int ic = ido - i;
            T tr2, ti2;
            mulpm(tr2, ti2, WA(0, i - 2), WA(0, i - 1), CC(i - 1, k, 1), CC(i, k, 1));
            pm(CH(i - 1, 0, k), CH(ic - 1, 1, k), CC(i - 1, k, 0), tr2);
            pm(CH(i, 0, k), CH(ic, 1, k), ti2, CC(i, k, 0));
        }
#undef CC
#undef CH
#undef WA
}

template <typename T>
void radf4(int ido, int l1, const T *cc, T *ch, const float *wa)
{
#define CC(a, b, c) cc[(a) + ido * ((b) + l1 * (c))]
#define CH(a, b, c) ch[(a) + ido * ((b) + 4 * (c))]
#define WA(x, i) wa[(i) + (x) * (ido - 1)]
    for (int k = 0; k < l1; k++) {
        T tr1, tr2;
        pm(tr1, CH(0, 2, k), CC(0, k, 3), CC(0, k, 1));
        pm(tr2, CH(ido - 1, 1, k), CC(0, k, 0), CC(0, k, 2));
        pm(CH(0, 0, k), CH(ido - 1, 3, k), tr2, tr1);
    }
    if ((ido & 1) == 0)
        for (int k = 0; k < l1; k++) {
            T ti1 = -HSQT2F * (CC(ido - 1, k, 1) + CC(ido - 1, k, 3));
            T tr1 = HSQT2F * (CC(ido - 1, k, 1) - CC(ido - 1, k, 3));
            pm(CH(ido - 1, 0, k), CH(ido - 1, 2, k), CC(ido - 1, k, 0), tr1);
            pm(CH(0, 3, k), CH(0, 1, k), ti1, CC(ido - 1, k, 2));
        }
    if (ido <= 2) return;
    for (int k = 0; k < l1; k++)
        for (int i = 2; i < ido; i += 2) {
            int ic = ido - i;
            T ci2, ci3, ci4, cr2, cr3, cr4, ti1, ti2, ti3, ti4, tr1, tr2, tr3, tr4;
            mulpm(cr2, ci2, WA(0, i - 2), WA(0, i - 1), CC(i - 1, k, 1), CC(i, k, 1));
            mulpm(cr3, ci3, WA(1, i - 2), WA(1, i - 1), CC(i - 1, k, 2), CC(i, k, 2));
            mulpm(cr4, ci4, WA(2, i - 2), WA(2, i - 1), CC(i - 1, k, 3), CC(i, k, 3));
            pm(tr1, tr4, cr4, cr2);
            pm(ti1, ti4, ci2, ci4);
            pm(tr2, tr3, CC(i - 1, k, 0), cr3);
            pm(ti2, ti3, CC(i, k, 0), ci3);
            pm(CH(i - 1, 0, k), CH(ic - 1, 3, k), tr2, tr1);
            pm(CH(i, 0, k), CH(ic, 3, k), ti1, ti2);
            pm(CH(i - 1, 2, k), CH(ic - 1, 1, k), tr3, ti4);
            pm(CH(i, 2, k), CH(ic, 1, k), tr4, ti3);
        }
#undef CC
#undef CH
#undef WA
}

template <typename T>
void radf3(int l1, const T *cc, T *ch)
{
    for (int k = 0; k < l1; k++) {
        const T cr2 = cc[k + l1] + cc[k + 2 * l1];
        ch[3 * k] = cc[k] + cr2;
        ch[2 + 3 * k] = TAUI * (cc[k + 2 * l1] - cc[k + l1]);
        ch[1 + 3 * k] = cc[k] + TAUR * cr2;
    }
}

template <typename T>
void radf5(int l1, const T *cc, T *ch)
{
    for (int k = 0; k < l1; k++) {
        T cr2, cr3, ci4, ci5;
        pm(cr2, ci5, cc[k + 4 * l1], cc[k + l1]);
        pm(cr3, ci4, cc[k + 3 * l1], cc[k + 2 * l1]);
        T *c = ch + 5 * k;
        c[0] = cc[k] + cr2 + cr3;
        c[1] = cc[k] + TR11 * cr2 + TR12 * cr3;
        c[2] = TI11 * ci5 + TI12 * ci4;
        c[3] = cc[k] + TR12 * cr2 + TR11 * cr3;
        c[4] = TI12 * ci5 - TI11 * ci4;
    }
}

template <typename T>
void radfg(int ip, int l1, T *cc, T *ch, const float *csarr)
{
    const int ipph = (ip + 1) / 2, idl1 = l1;
#define RF_CC(b, c) cc[(b) + ip * (c)]
#define RF_CH(b, c) ch[(b) + l1 * (c)]
#define RF_C1(b, c) cc[(b) + l1 * (c)]
#define RF_C2(a, b) cc[(a) + idl1 * (b)]
#define RF_CH2(a, b) ch[(a) + idl1 * (b)]
    for (int j = 1, jc = ip - 1; j < ipph; ++j, --jc)
        for (int k = 0; k < l1; ++k) {
            const T t1 = RF_C1(k, j), t2 = RF_C1(k, jc);
            pm(RF_C1(k, j), RF_C1(k, jc), t2, t1);
        }
    for (int l = 1, lc = ip - 1; l < ipph; ++l, --lc) {
        for (int ik = 0; ik < idl1; ++ik) {
            RF_CH2(ik, l) = RF_C2(ik, 0) + csarr[2 * l] * RF_C2(ik, 1) + csarr[4 * l] * RF_C2(ik, 2);
            RF_CH2(ik, lc) = csarr[2 * l + 1] * RF_C2(ik, ip - 1) + csarr[4 * l + 1] * RF_C2(ik, ip - 2);
        }
        int iang = 2 * l;
        for (int j = 3, jc = ip - 3; j < ipph; ++j, --jc) {
            iang += l;
            if (iang > ip) iang -= ip;
            const float ar = csarr[2 * iang], ai = csarr[2 * iang + 1];
            for (int ik = 0; ik < idl1; ++ik) {
                RF_CH2(ik, l) += ar * RF_C2(ik, j);
                RF_CH2(ik, lc) += ai * RF_C2(ik, jc);
            }
        }
    }
    for (int ik = 0; ik < idl1; ++ik) RF_CH2(ik, 0) = RF_C2(ik, 0);
    for (int j = 1; j < ipph; ++j)
        for (int ik = 0; ik < idl1; ++ik) RF_CH2(ik, 0) += RF_C2(ik, j);
    for (int k = 0; k < l1; ++k) RF_CC(0, k) = RF_CH(k, 0);
    for (int j = 1, jc = ip - 1; j < ipph; ++j, --jc) {
        const int j2 = 2 * j - 1;
        for (int k = 0; k < l1; ++k) {
            RF_CC(j2, k) = RF_CH(k, j);
            RF_CC(j2 + 1, k) = RF_CH(k, jc);
        }
    }
#undef RF_CC
#undef RF_CH
#undef RF_C1
#undef RF_C2
#undef RF_CH2
}

/* rfft_exec(r2hc = 1) with copy_and_norm(fct) */
template <typename T>
void rfft_forward(const dct_plan *p, T *c, float fct)
{
    const int n = p->n, nf = p->nf;
    T ch[16];
    T *p1 = c, *p2 = ch;
    for (int k1 = 0, l1 = n; k1 < nf; ++k1) {
        int k = nf - k1 - 1, ip = p->fct[k], ido = n / l1;
        l1 /= ip;
        if (ip == 4) radf4(ido, l1, p1, p2, p->tw[k]);
        else if (ip == 2) radf2(ido, l1, p1, p2, p->tw[k]);
        else if (ip == 3) radf3(l1, p1, p2);
        else if (ip == 5) radf5(l1, p1, p2);
        else { radfg(ip, l1, p1, p2, p->tws[k]); T *t = p1; p1 = p2; p2 = t; }
        T *t = p1; p1 = p2; p2 = t;
    }
    if (p1 != c) {
        for (int i = 0; i < n; ++i) c[i] = fct * p1[i];
    } else {
        for (int i = 0; i < n; ++i) c[i] *= fct;
    }
}

/* T_dcst23 type 3 (tmfwm_oracle.c dct3_1d) */
template <typename T>
void dct3_1d(const dct_plan *p, T *c)
{
    const int N = p->n, NS2 = (N + 1) / 2;
    c[0] *= SQRT2F;
    for (int k = 1, kc = N - 1; k < NS2; ++k, --kc) {
        T t1 = c[k] + c[kc], t2 = c[k] - c[kc];
        c[k] = p->dtw[k - 1] * t2 + p->dtw[kc - 1] * t1;
        c[kc] = p->dtw[k - 1] * t1 - p->dtw[kc - 1] * t2;
    }
    c[NS2] *= 2.0f * p->dtw[NS2 - 1];
    rfft_forward(p, c, p->norm);
    for (int k = 1; k < N - 1; k += 2) {
        T t = c[k];
        c[k] = t - c[k + 1];
        c[k + 1] = t + c[k + 1];
    }
}

/* [min, max] of fmaf(u, b, acc) over the corners: RN is monotone in the exact u*b + acc */
inline Iv fma_iv(Iv u, Iv b, Iv acc)
{
    const float l1 = fmaf(u.lo, b.lo, acc.lo), l2 = fmaf(u.lo, b.hi, acc.lo), l3 = fmaf(u.hi, b.lo, acc.lo),
                l4 = fmaf(u.hi, b.hi, acc.lo);
    const float h1 = fmaf(u.lo, b.lo, acc.hi), h2 = fmaf(u.lo, b.hi, acc.hi), h3 = fmaf(u.hi, b.lo, acc.hi),
                h4 = fmaf(u.hi, b.hi, acc.hi);
    return {std::min(std::min(l1, l2), std::min(l3, l4)), std::max(std::max(h1, h2), std::max(h3, h4))};
}

const double kCertScale = 0x1p-45; /* K 2^-53, K = 256 */

}  // namespace

extern "C" int orc_cert_block(const float *D, const double *U, const double *sig, const double *V, int b, uint8_t w,
                              double alpha, const float *cbs, const float *crs, int64_t *stats)
{
    double s1 = 0.0;
    for (int k = 0; k < b; ++k) s1 = sig[k] > s1 ? sig[k] : s1;
    if (s1 == 0.0) return 0;
    int dc_only = 1;
    for (int i = 1; i < b * b; ++i) dc_only &= D[i] == 0.0f;
    if (dc_only) return 0;
    const double t = kCertScale * s1, Es = t;
    Iv S[16], Ui[16][16], Bi[16][16];
    for (int k = 0; k < b; ++k) {
        const double lo = sig[k] - Es;
        S[k] = {(float)(lo > 0.0 ? lo : 0.0), (float)(sig[k] + Es)};
    }
    const double c = alpha * ((double)w / 255.0);
    S[0] = {(float)((double)S[0].lo + c), (float)((double)S[0].hi + c)};
    if (!(S[0].lo >= 0.0f)) return 1; /* alpha < 0 pushing S'0 below zero: not covered */
    for (int k = 0; k < b; ++k) {
        if ((float)sig[k] == 0.0f) {
            for (int r = 0; r < b; ++r) Ui[r][k] = {2.0f, 2.0f};
            for (int j = 0; j < b; ++j) Bi[k][j] = {-2.0f * S[k].hi, 2.0f * S[k].hi};
            continue;
        }
        double g = sig[k];
        for (int j = 0; j < b; ++j)
            if (j != k) {
                const double d = fabs(sig[k] - sig[j]);
                g = d < g ? d : g;
            }
        const double E = (double)(float)(t / g);
        for (int r = 0; r < b; ++r) {
            const double u = U[r * b + k];
            Ui[r][k] = {(float)(u - E), (float)(u + E)};
        }
        for (int j = 0; j < b; ++j) {
            const double v = V[j * b + k];
            const float vl = (float)(v - E), vh = (float)(v + E);
            Bi[k][j] = {vl >= 0.0f ? S[k].lo * vl : S[k].hi * vl, vh <= 0.0f ? S[k].lo * vh : S[k].hi * vh};
        }
    }
    int str = 0, wid = 0; /* over the triplets that reach the output */
    for (int k = 0; k < b; ++k)
        for (int r = 0; r < b; ++r) {
            wid |= Ui[r][k].lo != Ui[r][k].hi || Bi[k][r].lo != Bi[k][r].hi;
            if ((float)sig[k] != 0.0f)
                str |= (Ui[r][k].lo < 0.0f && Ui[r][k].hi > 0.0f) || (Bi[k][r].lo < 0.0f && Bi[k][r].hi > 0.0f);
        }
    if (str && wid) return 1;
    Iv M[16][16];
    int64_t munc = 0, yunc = 0;
    for (int i = 0; i < b; ++i)
        for (int j = 0; j < b; ++j) {
            Iv acc = {0.0f, 0.0f};
            for (int k = 0; k < b; ++k) acc = fma_iv(Ui[i][k], Bi[k][j], acc);
            M[i][j] = acc;
            munc += acc.lo != acc.hi;
        }
    const dct_plan *p = orc_plan(b);
    for (int j = 0; j < b; ++j) { /* axis 0 first, then rows (watermarking.py:81-83) */
        Iv col[16];
        for (int i = 0; i < b; ++i) col[i] = M[i][j];
        dct3_1d(p, col);
        for (int i = 0; i < b; ++i) M[i][j] = col[i];
    }
    int fail = 0;
    for (int i = 0; i < b; ++i) {
        dct3_1d(p, M[i]);
        for (int j = 0; j < b; ++j) {
            if (M[i][j].lo == M[i][j].hi) continue;
            ++yunc;
            uint8_t lo[3], hi[3];
            orc_colour_inv_px(M[i][j].lo, cbs[i * b + j], crs[i * b + j], lo);
            orc_colour_inv_px(M[i][j].hi, cbs[i * b + j], crs[i * b + j], hi);
            fail |= lo[0] != hi[0] || lo[1] != hi[1] || lo[2] != hi[2];
        }
    }
    if (stats) {
        stats[0] += munc;
        stats[1] += yunc;
    }
    return fail;
}

/* tests: the interval IDCT on degenerate intervals is the oracle's own float IDCT */
extern "C" void orc_cert_idct_point(float *blk, int b)
{
    const dct_plan *p = orc_plan(b);
    Iv M[16][16];
    for (int i = 0; i < b; ++i)
        for (int j = 0; j < b; ++j) M[i][j] = {blk[i * b + j], blk[i * b + j]};
    for (int j = 0; j < b; ++j) {
        Iv col[16];
        for (int i = 0; i < b; ++i) col[i] = M[i][j];
        dct3_1d(p, col);
        for (int i = 0; i < b; ++i) M[i][j] = col[i];
    }
    for (int i = 0; i < b; ++i) {
        dct3_1d(p, M[i]);
        for (int j = 0; j < b; ++j) blk[i * b + j] = M[i][j].lo == M[i][j].hi ? M[i][j].lo : NAN;
    }
}
