/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of the arithmetic of the reference watermark path,
 * /root/reference/modules/watermarking.py (embed_watermark :135-221,
 * extract_watermark :224-294) and of the third-party kernels it calls
 * (scipy 1.15.3 pocketfft DCT-II/III in fp32, numpy 2.2.6 -> LAPACK dgesdd on
 * an f64 upcast, OpenBLAS 0.3.29 dgemv / sgemm FMA patterns).  The numerical
 * contract it follows is SURVEY.md section 8(a) N1-N10 and DESIGN.md section 3.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library, and only as the checker / CPU baseline.  The product path
 * (thatsmyface_amd/, libtmfwm.so) never links or calls it.
 *
 * Parity pinning: tests/golden fixtures were produced by importing the reference
 * itself (tests/golden/gen_golden.py); tests/test_oracle_golden.py checks this
 * file against every fixture and against the survey's known-answer hashes.
 *
 * SVD: the reference's numbers come from f32(dgesdd(f64(D))).  LAPACK itself is
 * not restated; any f64-accurate SVD rounded to f32 reproduces it.
 * The SVD below is a fully specified one-sided (Hestenes) Jacobi in f64 whose
 * every rounding step is fixed so that the HIP kernels
 * reproduce it bit for bit.  Its agreement with LAPACK is pinned by the golden
 * fixtures and measured at scale by tests/test_oracle_vs_lapack.py.
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off, no fast-math).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "orc_plan.h"

#define ORC_MAXB 16

/* SVD routes:
 *   ORC_SVD_JACOBI  every block through the specified 3-phase Jacobi;
 *   ORC_SVD_LAPACK  every block through the restated dgesdd route (tmfwm_lapack.c) --
 *                   the reference's own arithmetic;
 *   ORC_SVD_HYBRID  Jacobi, except blocks the conditioning test orc_svd_flag()
 *                   flags, which take the dgesdd route (the device contract). */
#define ORC_SVD_JACOBI 0
#define ORC_SVD_LAPACK 1
#define ORC_SVD_HYBRID 2
/* the route libtmfwm.so implements (orc_embed_frame / orc_extract_frame) */
#ifndef ORC_SVD_CONTRACT
#define ORC_SVD_CONTRACT ORC_SVD_HYBRID
#endif
int orc_lp_svd_block_f32(const float *D, int n, float *U, float *S, float *Vt);

/* ------------------------------------------------------------------------ */
/* N1 / N2: RGB -> YCbCr (watermarking.py:23-50)                            */
/* ------------------------------------------------------------------------ */

/* watermarking.py:29  np.array(img, float32) / 255.0 -> IEEE fp32 divide */
static inline float unit_from_u8(unsigned v) { return (float)v / 255.0f; }

/* watermarking.py:37-48.  np.dot(f64 3x3, f32 3-vector) runs OpenBLAS dgemv;
 * its SkylakeX tail evaluates row c as fma(T[c][2], b, fma(T[c][0], r, T[c][1]*g))
 * (exhaustively verified over 2^24 colours).  The f64 result is
 * stored into a float32 array; Cb, Cr then get "+= 0.5" in f32 (:48). */
static inline void colour_fwd(unsigned R, unsigned G, unsigned B, float *y, float *cb, float *cr)
{
    const double r = unit_from_u8(R), g = unit_from_u8(G), b = unit_from_u8(B);
    *y = (float)fma(0.114, b, fma(0.299, r, 0.587 * g));
    *cb = (float)fma(0.5, b, fma(-0.169, r, -0.331 * g)) + 0.5f;
    *cr = (float)fma(-0.081, b, fma(0.5, r, -0.419 * g)) + 0.5f;
}

/* ------------------------------------------------------------------------ */
/* N9: YCbCr -> RGB (watermarking.py:53-73)                                 */
/* ------------------------------------------------------------------------ */
static inline uint8_t u8_from_unit(float f)
{
    /* :70 np.clip(rgb, 0, 1) (f32), :73 (rgb * 255).astype(uint8) (f32 multiply, truncation) */
    if (f < 0.0f) f = 0.0f;
    if (f > 1.0f) f = 1.0f;
    return (uint8_t)(f * 255.0f);
}

static inline void colour_inv(float y, float cbs, float crs, uint8_t out[3])
{
    /* :58 Cb, Cr -= 0.5 in f32; :61-67 dgemv with Ti = [[1,0,1.403],[1,-0.344,-0.714],[1,1.773,0]] */
    const float cbp = cbs - 0.5f, crp = crs - 0.5f;
    const double Y = y, CB = cbp, CR = crp;
    out[0] = u8_from_unit((float)fma(1.403, CR, fma(1.0, Y, 0.0 * CB)));
    out[1] = u8_from_unit((float)fma(-0.714, CR, fma(1.0, Y, -0.344 * CB)));
    out[2] = u8_from_unit((float)fma(0.0, CR, fma(1.0, Y, 1.773 * CB)));
}

void orc_colour_inv_px(float y, float cbs, float crs, uint8_t out[3]) { colour_inv(y, cbs, crs, out); }

/* ------------------------------------------------------------------------ */
/* N3: pocketfft fp32 DCT-II / DCT-III (ortho), every even length 4..16     */
/* (the UI block sizes, embed_watermark_page.py:324-331).                    */
/* scipy.fftpack.dct/idct -> pocketfft T_dcst23::exec around rfftp.          */
/* Every statement below is one fp32 operation (no contraction).             */
/* ------------------------------------------------------------------------ */
#define ORC_NPLANS 7 /* n = 4, 6, ..., 16 */
static dct_plan g_plans[ORC_NPLANS];
static int g_plans_ready = 0;

static const long double ORC_PI = 3.141592653589793238462643383279502884197L;

/* twid[m] = (cos, sin)(2 pi m / n) exactly as pocketfft's sincos_2pibyn<float> makes
 * them: octant-reduced cos/sin in double on a two-level (v1[m & mask], v2[m >> shift])
 * table, complex product in double, rounded to float.  Exact-quadrant angles come
 * out as exact signed zeros (cos(2 pi 3/12) = -0.0f), which the N = 12 radix-4 pass
 * uses; a plain cos() would give -2.5e-20f there. */
typedef struct { double r, i; } orc_cd;
static orc_cd sc_calc(size_t x, size_t n, double ang)
{
    orc_cd o;
    x <<= 3;
    if (x < 4 * n) {
        if (x < 2 * n) {
            if (x < n) { o.r = cos((double)x * ang); o.i = sin((double)x * ang); return o; }
            o.r = sin((double)(2 * n - x) * ang); o.i = cos((double)(2 * n - x) * ang); return o;
        }
        x -= 2 * n;
        if (x < n) { o.r = -sin((double)x * ang); o.i = cos((double)x * ang); return o; }
        o.r = -cos((double)(2 * n - x) * ang); o.i = sin((double)(2 * n - x) * ang); return o;
    }
    x = 8 * n - x;
    if (x < 2 * n) {
        if (x < n) { o.r = cos((double)x * ang); o.i = -sin((double)x * ang); return o; }
        o.r = sin((double)(2 * n - x) * ang); o.i = -cos((double)(2 * n - x) * ang); return o;
    }
    x -= 4 * n;
    if (x < n) { o.r = -sin((double)x * ang); o.i = -cos((double)x * ang); return o; }
    o.r = -cos((double)(2 * n - x) * ang); o.i = -sin((double)(2 * n - x) * ang); return o;
}
static void sincos_2pibyn(size_t n, size_t idx, float *re, float *im)
{
    const double ang = (double)(0.25L * ORC_PI / (long double)n);
    size_t nval = (n + 2) / 2, shift = 1;
    while (((size_t)1 << shift) * ((size_t)1 << shift) < nval) ++shift;
    const size_t mask = ((size_t)1 << shift) - 1;
    int conj = 0;
    if (!(2 * idx <= n)) { idx = n - idx; conj = 1; }
    const orc_cd one = {1.0, 0.0};
    const orc_cd x1 = (idx & mask) ? sc_calc(idx & mask, n, ang) : one;
    const orc_cd x2 = (idx >> shift) ? sc_calc((idx >> shift) * (mask + 1), n, ang) : one;
    *re = (float)(x1.r * x2.r - x1.i * x2.i);
    const float i = (float)(x1.r * x2.i + x1.i * x2.r);
    *im = conj ? -i : i;
}
static float tw_cos(long m, long n) { float r, i; sincos_2pibyn((size_t)n, (size_t)m, &r, &i); return r; }
static float tw_sin(long m, long n) { float r, i; sincos_2pibyn((size_t)n, (size_t)m, &r, &i); return i; }

static void plan_init(dct_plan *p, int n)
{
    memset(p, 0, sizeof(*p));
    p->n = n;
    int len = n, nf = 0;
    while (len % 4 == 0) { p->fct[nf++] = 4; len >>= 2; }
    if (len % 2 == 0) {
        len >>= 1;
        p->fct[nf++] = 2;
        int t = p->fct[0]; p->fct[0] = p->fct[nf - 1]; p->fct[nf - 1] = t;
    }
    for (int d = 3; d * d <= len; d += 2)
        while (len % d == 0) { p->fct[nf++] = d; len /= d; }
    if (len > 1) p->fct[nf++] = len;
    p->nf = nf;
    int l1 = 1;
    for (int k = 0; k < nf; ++k) {
        int ip = p->fct[k], ido = n / (l1 * ip);
        if (k < nf - 1) {
            for (int j = 1; j < ip; ++j)
                for (int i = 1; i <= (ido - 1) / 2; ++i) {
                    p->tw[k][(j - 1) * (ido - 1) + 2 * i - 2] = tw_cos(j * l1 * i, n);
                    p->tw[k][(j - 1) * (ido - 1) + 2 * i - 1] = tw_sin(j * l1 * i, n);
                }
        }
        if (ip > 5) {
            p->tws[k][0] = 1.0f;
            p->tws[k][1] = 0.0f;
            for (int i = 2, ic = 2 * ip - 2; i <= ic; i += 2, ic -= 2) {
                p->tws[k][i] = tw_cos(i / 2 * (n / ip), n);
                p->tws[k][i + 1] = tw_sin(i / 2 * (n / ip), n);
                p->tws[k][ic] = tw_cos(i / 2 * (n / ip), n);
                p->tws[k][ic + 1] = -tw_sin(i / 2 * (n / ip), n);
            }
        }
        l1 *= ip;
    }
    for (int i = 0; i < n; ++i) p->dtw[i] = tw_cos(i + 1, 4 * n);
    p->norm = (float)(1.0L / sqrtl((long double)(2 * n)));
}

static void plans_init(void)
{
    if (g_plans_ready) return;
    for (int k = 0; k < ORC_NPLANS; ++k) plan_init(&g_plans[k], 4 + 2 * k);
    g_plans_ready = 1;
}

static const dct_plan *plan_for(int n)
{
    plans_init();
    return &g_plans[(n - 4) / 2];
}

const dct_plan *orc_plan(int n) { return plan_for(n); }

#define PM(a, b, c, d) do { float c_ = (c), d_ = (d); (a) = c_ + d_; (b) = c_ - d_; } while (0)
#define MULPM(a, b, c, d, e, f) do { float c_ = (c), d_ = (d), e_ = (e), f_ = (f); (a) = c_ * e_ + d_ * f_; (b) = c_ * f_ - d_ * e_; } while (0)

static const float SQRT2F = 1.41421356237309504880f;
static const float HSQT2F = 0.70710678118654752440f;

/* backward radix 2 */
static void radb2(int ido, int l1, const float *cc, float *ch, const float *wa)
{
#define CC(a, b, c) cc[(a) + ido * ((b) + 2 * (c))]
#define CH(a, b, c) ch[(a) + ido * ((b) + l1 * (c))]
#define WA(x, i) wa[(i) + (x) * (ido - 1)]
    for (int k = 0; k < l1; k++) PM(CH(0, k, 0), CH(0, k, 1), CC(0, 0, k), CC(ido - 1, 1, k));
    if ((ido & 1) == 0)
        for (int k = 0; k < l1; k++) {
            CH(ido - 1, k, 0) = 2.0f * CC(ido - 1, 0, k);
            CH(ido - 1, k, 1) = -2.0f * CC(0, 1, k);
        }
    if (ido <= 2) return;
    for (int k = 0; k < l1; ++k)
        for (int i = 2; i < ido; i += 2) {
            int ic = ido - i;
            float ti2, tr2;
            PM(CH(i - 1, k, 0), tr2, CC(i - 1, 0, k), CC(ic - 1, 1, k));
            PM(ti2, CH(i, k, 0), CC(i, 0, k), CC(ic, 1, k));
            MULPM(CH(i, k, 1), CH(i - 1, k, 1), WA(0, i - 2), WA(0, i - 1), ti2, tr2);
        }
#undef CC
#undef CH
#undef WA
}

/* backward radix 4 */
static void radb4(int ido, int l1, const float *cc, float *ch, const float *wa)
{
#define CC(a, b, c) cc[(a) + ido * ((b) + 4 * (c))]
#define CH(a, b, c) ch[(a) + ido * ((b) + l1 * (c))]
#define WA(x, i) wa[(i) + (x) * (ido - 1)]
    for (int k = 0; k < l1; k++) {
        float tr1, tr2;
        PM(tr2, tr1, CC(0, 0, k), CC(ido - 1, 3, k));
        float tr3 = 2.0f * CC(ido - 1, 1, k);
        float tr4 = 2.0f * CC(0, 2, k);
        PM(CH(0, k, 0), CH(0, k, 2), tr2, tr3);
        PM(CH(0, k, 3), CH(0, k, 1), tr1, tr4);
    }
    if ((ido & 1) == 0)
        for (int k = 0; k < l1; k++) {
            float tr1, tr2, ti1, ti2;
            PM(ti1, ti2, CC(0, 3, k), CC(0, 1, k));
            PM(tr2, tr1, CC(ido - 1, 0, k), CC(ido - 1, 2, k));
            CH(ido - 1, k, 0) = tr2 + tr2;
            CH(ido - 1, k, 1) = SQRT2F * (tr1 - ti1);
            CH(ido - 1, k, 2) = ti2 + ti2;
            CH(ido - 1, k, 3) = -SQRT2F * (tr1 + ti1);
        }
    if (ido <= 2) return;
    for (int k = 0; k < l1; ++k)
        for (int i = 2; i < ido; i += 2) {
            float ci2, ci3, ci4, cr2, cr3, cr4, ti1, ti2, ti3, ti4, tr1, tr2, tr3, tr4;
            int ic = ido - i;
            PM(tr2, tr1, CC(i - 1, 0, k), CC(ic - 1, 3, k));
            PM(ti1, ti2, CC(i, 0, k), CC(ic, 3, k));
            PM(tr4, ti3, CC(i, 2, k), CC(ic, 1, k));
            PM(tr3, ti4, CC(i - 1, 2, k), CC(ic - 1, 1, k));
            PM(CH(i - 1, k, 0), cr3, tr2, tr3);
            PM(CH(i, k, 0), ci3, ti2, ti3);
            PM(cr4, cr2, tr1, tr4);
            PM(ci2, ci4, ti1, ti4);
            MULPM(CH(i, k, 1), CH(i - 1, k, 1), WA(0, i - 2), WA(0, i - 1), ci2, cr2);
            MULPM(CH(i, k, 2), CH(i - 1, k, 2), WA(1, i - 2), WA(1, i - 1), ci3, cr3);
            MULPM(CH(i, k, 3), CH(i - 1, k, 3), WA(2, i - 2), WA(2, i - 1), ci4, cr4);
        }
#undef CC
#undef CH
#undef WA
}

/* forward radix 2 */
static void radf2(int ido, int l1, const float *cc, float *ch, const float *wa)
{
#define CC(a, b, c) cc[(a) + ido * ((b) + l1 * (c))]
#define CH(a, b, c) ch[(a) + ido * ((b) + 2 * (c))]
#define WA(x, i) wa[(i) + (x) * (ido - 1)]
    for (int k = 0; k < l1; k++) PM(CH(0, 0, k), CH(ido - 1, 1, k), CC(0, k, 0), CC(0, k, 1));
    if ((ido & 1) == 0)
        for (int k = 0; k < l1; k++) {
            CH(0, 1, k) = -CC(ido - 1, k, 1);
            CH(ido - 1, 0, k) = CC(ido - 1, k, 0);
        }
    if (ido <= 2) return;
    for (int k = 0; k < l1; k++)
        for (int i = 2; i < ido; i += 2) {
            int ic = ido - i;
            float tr2, ti2;
            MULPM(tr2, ti2, WA(0, i - 2), WA(0, i - 1), CC(i - 1, k, 1), CC(i, k, 1));
            PM(CH(i - 1, 0, k), CH(ic - 1, 1, k), CC(i - 1, k, 0), tr2);
            PM(CH(i, 0, k), CH(ic, 1, k), ti2, CC(i, k, 0));
        }
#undef CC
#undef CH
#undef WA
}

/* forward radix 4 */
static void radf4(int ido, int l1, const float *cc, float *ch, const float *wa)
{
#define CC(a, b, c) cc[(a) + ido * ((b) + l1 * (c))]
#define CH(a, b, c) ch[(a) + ido * ((b) + 4 * (c))]
#define WA(x, i) wa[(i) + (x) * (ido - 1)]
    for (int k = 0; k < l1; k++) {
        float tr1, tr2;
        PM(tr1, CH(0, 2, k), CC(0, k, 3), CC(0, k, 1));
        PM(tr2, CH(ido - 1, 1, k), CC(0, k, 0), CC(0, k, 2));
        PM(CH(0, 0, k), CH(ido - 1, 3, k), tr2, tr1);
    }
    if ((ido & 1) == 0)
        for (int k = 0; k < l1; k++) {
            float ti1 = -HSQT2F * (CC(ido - 1, k, 1) + CC(ido - 1, k, 3));
            float tr1 = HSQT2F * (CC(ido - 1, k, 1) - CC(ido - 1, k, 3));
            PM(CH(ido - 1, 0, k), CH(ido - 1, 2, k), CC(ido - 1, k, 0), tr1);
            PM(CH(0, 3, k), CH(0, 1, k), ti1, CC(ido - 1, k, 2));
        }
    if (ido <= 2) return;
    for (int k = 0; k < l1; k++)
        for (int i = 2; i < ido; i += 2) {
            int ic = ido - i;
            float ci2, ci3, ci4, cr2, cr3, cr4, ti1, ti2, ti3, ti4, tr1, tr2, tr3, tr4;
            MULPM(cr2, ci2, WA(0, i - 2), WA(0, i - 1), CC(i - 1, k, 1), CC(i, k, 1));
            MULPM(cr3, ci3, WA(1, i - 2), WA(1, i - 1), CC(i - 1, k, 2), CC(i, k, 2));
            MULPM(cr4, ci4, WA(2, i - 2), WA(2, i - 1), CC(i - 1, k, 3), CC(i, k, 3));
            PM(tr1, tr4, cr4, cr2);
            PM(ti1, ti4, ci2, ci4);
            PM(tr2, tr3, CC(i - 1, k, 0), cr3);
            PM(ti2, ti3, CC(i, k, 0), ci3);
            PM(CH(i - 1, 0, k), CH(ic - 1, 3, k), tr2, tr1);
            PM(CH(i, 0, k), CH(ic, 3, k), ti1, ti2);
            PM(CH(i - 1, 2, k), CH(ic - 1, 1, k), tr3, ti4);
            PM(CH(i, 2, k), CH(ic, 1, k), tr4, ti3);
        }
#undef CC
#undef CH
#undef WA
}

/* Radix 3, 5 and generic (7) passes.  For every n <= 16 the odd factor is the last
 * backward / first forward factor, so only their ido == 1 parts ever run; those
 * parts are restated here (pocketfft radb3/radb5/radbg, radf3/radf5/radfg). */
static const float TAUR = -0.5f, TAUI = 0.8660254037844386467637231707529362f;
static const float TR11 = 0.3090169943749474241022934171828191f, TI11 = 0.9510565162951535721164393333793821f;
static const float TR12 = -0.8090169943749474241022934171828191f, TI12 = 0.5877852522924731291687059546390728f;

static void radb3(int l1, const float *cc, float *ch)
{
    for (int k = 0; k < l1; k++) {
        const float tr2 = 2.0f * cc[1 + 3 * k];
        const float cr2 = cc[3 * k] + TAUR * tr2;
        ch[k] = cc[3 * k] + tr2;
        const float ci3 = (2.0f * TAUI) * cc[2 + 3 * k];
        PM(ch[k + 2 * l1], ch[k + l1], cr2, ci3);
    }
}

static void radb5(int l1, const float *cc, float *ch)
{
    for (int k = 0; k < l1; k++) {
        const float *c = cc + 5 * k;
        const float ti5 = c[2] + c[2], ti4 = c[4] + c[4];
        const float tr2 = c[1] + c[1], tr3 = c[3] + c[3];
        ch[k] = c[0] + tr2 + tr3;
        const float cr2 = c[0] + TR11 * tr2 + TR12 * tr3;
        const float cr3 = c[0] + TR12 * tr2 + TR11 * tr3;
        float ci4, ci5;
        MULPM(ci5, ci4, ti5, ti4, TI11, TI12);
        PM(ch[k + 4 * l1], ch[k + l1], cr2, ci5);
        PM(ch[k + 3 * l1], ch[k + 2 * l1], cr3, ci4);
    }
}

/* generic odd radix ip (7 for n = 14), ido == 1; csarr = plan tws.  cc is scratch. */
static void radbg(int ip, int l1, float *cc, float *ch, const float *csarr)
{
    const int ipph = (ip + 1) / 2, idl1 = l1;
#define RB_CC(b, c) cc[(b) + ip * (c)]
#define RB_CH(b, c) ch[(b) + l1 * (c)]
#define RB_C2(a, b) cc[(a) + idl1 * (b)]
#define RB_CH2(a, b) ch[(a) + idl1 * (b)]
    for (int k = 0; k < l1; ++k) RB_CH(k, 0) = RB_CC(0, k);
    for (int j = 1, jc = ip - 1; j < ipph; ++j, --jc) {
        const int j2 = 2 * j - 1;
        for (int k = 0; k < l1; ++k) {
            RB_CH(k, j) = 2.0f * RB_CC(j2, k);
            RB_CH(k, jc) = 2.0f * RB_CC(j2 + 1, k);
        }
    }
    for (int l = 1, lc = ip - 1; l < ipph; ++l, --lc) {
        for (int ik = 0; ik < idl1; ++ik) {
            RB_C2(ik, l) = RB_CH2(ik, 0) + csarr[2 * l] * RB_CH2(ik, 1) + csarr[4 * l] * RB_CH2(ik, 2);
            RB_C2(ik, lc) = csarr[2 * l + 1] * RB_CH2(ik, ip - 1) + csarr[4 * l + 1] * RB_CH2(ik, ip - 2);
        }
        int iang = 2 * l;
        for (int j = 3, jc = ip - 3; j < ipph; ++j, --jc) { /* ip <= 7: single-term tail only */
            iang += l;
            if (iang > ip) iang -= ip;
            const float war = csarr[2 * iang], wai = csarr[2 * iang + 1];
            for (int ik = 0; ik < idl1; ++ik) {
                RB_C2(ik, l) += war * RB_CH2(ik, j);
                RB_C2(ik, lc) += wai * RB_CH2(ik, jc);
            }
        }
    }
    for (int j = 1; j < ipph; ++j)
        for (int ik = 0; ik < idl1; ++ik) RB_CH2(ik, 0) += RB_CH2(ik, j);
    for (int j = 1, jc = ip - 1; j < ipph; ++j, --jc)
        for (int k = 0; k < l1; ++k) PM(RB_CH(k, jc), RB_CH(k, j), RB_C2(k, j), RB_C2(k, jc));
#undef RB_CC
#undef RB_CH
#undef RB_C2
#undef RB_CH2
}

static void radf3(int l1, const float *cc, float *ch)
{
    for (int k = 0; k < l1; k++) {
        const float cr2 = cc[k + l1] + cc[k + 2 * l1];
        ch[3 * k] = cc[k] + cr2;
        ch[2 + 3 * k] = TAUI * (cc[k + 2 * l1] - cc[k + l1]);
        ch[1 + 3 * k] = cc[k] + TAUR * cr2;
    }
}

static void radf5(int l1, const float *cc, float *ch)
{
    for (int k = 0; k < l1; k++) {
        float cr2, cr3, ci4, ci5;
        PM(cr2, ci5, cc[k + 4 * l1], cc[k + l1]);
        PM(cr3, ci4, cc[k + 3 * l1], cc[k + 2 * l1]);
        float *c = ch + 5 * k;
        c[0] = cc[k] + cr2 + cr3;
        c[1] = cc[k] + TR11 * cr2 + TR12 * cr3;
        c[2] = TI11 * ci5 + TI12 * ci4;
        c[3] = cc[k] + TR12 * cr2 + TR11 * cr3;
        c[4] = TI12 * ci5 - TI11 * ci4;
    }
}

/* generic odd radix, ido == 1; the result is left in cc (pocketfft swaps once more) */
static void radfg(int ip, int l1, float *cc, float *ch, const float *csarr)
{
    const int ipph = (ip + 1) / 2, idl1 = l1;
#define RF_CC(b, c) cc[(b) + ip * (c)]
#define RF_CH(b, c) ch[(b) + l1 * (c)]
#define RF_C1(b, c) cc[(b) + l1 * (c)]
#define RF_C2(a, b) cc[(a) + idl1 * (b)]
#define RF_CH2(a, b) ch[(a) + idl1 * (b)]
    for (int j = 1, jc = ip - 1; j < ipph; ++j, --jc)
        for (int k = 0; k < l1; ++k) {
            const float t1 = RF_C1(k, j), t2 = RF_C1(k, jc);
            PM(RF_C1(k, j), RF_C1(k, jc), t2, t1);
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

/* rfftp::exec with copy_and_norm(fct) */
static void rfft_exec(const dct_plan *p, float *c, float fct, int r2hc)
{
    const int n = p->n, nf = p->nf;
    float ch[ORC_MAXB];
    float *p1 = c, *p2 = ch;
    if (r2hc) {
        for (int k1 = 0, l1 = n; k1 < nf; ++k1) {
            int k = nf - k1 - 1, ip = p->fct[k], ido = n / l1;
            l1 /= ip;
            if (ip == 4) radf4(ido, l1, p1, p2, p->tw[k]);
            else if (ip == 2) radf2(ido, l1, p1, p2, p->tw[k]);
            else if (ip == 3) radf3(l1, p1, p2);
            else if (ip == 5) radf5(l1, p1, p2);
            else { radfg(ip, l1, p1, p2, p->tws[k]); float *t = p1; p1 = p2; p2 = t; }
            float *t = p1; p1 = p2; p2 = t;
        }
    } else {
        for (int k = 0, l1 = 1; k < nf; k++) {
            int ip = p->fct[k], ido = n / (ip * l1);
            if (ip == 4) radb4(ido, l1, p1, p2, p->tw[k]);
            else if (ip == 2) radb2(ido, l1, p1, p2, p->tw[k]);
            else if (ip == 3) radb3(l1, p1, p2);
            else if (ip == 5) radb5(l1, p1, p2);
            else radbg(ip, l1, p1, p2, p->tws[k]);
            float *t = p1; p1 = p2; p2 = t;
            l1 *= ip;
        }
    }
    if (p1 != c) {
        if (fct != 1.0f) for (int i = 0; i < n; ++i) c[i] = fct * p1[i];
        else memcpy(c, p1, sizeof(float) * n);
    } else if (fct != 1.0f) {
        for (int i = 0; i < n; ++i) c[i] *= fct;
    }
}

/* T_dcst23::exec, type 2 (forward DCT), cosine=true, ortho=true */
static void dct2_1d(const dct_plan *p, float *c)
{
    const int N = p->n, NS2 = (N + 1) / 2;
    c[0] *= 2.0f;
    if ((N & 1) == 0) c[N - 1] *= 2.0f;
    for (int k = 1; k < N - 1; k += 2) { float t = c[k + 1]; c[k + 1] = t - c[k]; c[k] = c[k] + t; }
    rfft_exec(p, c, p->norm, 0);
    for (int k = 1, kc = N - 1; k < NS2; ++k, --kc) {
        float t1 = p->dtw[k - 1] * c[kc] + p->dtw[kc - 1] * c[k];
        float t2 = p->dtw[k - 1] * c[k] - p->dtw[kc - 1] * c[kc];
        c[k] = 0.5f * (t1 + t2);
        c[kc] = 0.5f * (t1 - t2);
    }
    if ((N & 1) == 0) c[NS2] *= p->dtw[NS2 - 1];
    c[0] *= SQRT2F * 0.5f;
}

/* T_dcst23::exec, type 3 (inverse DCT), cosine=true, ortho=true */
static void dct3_1d(const dct_plan *p, float *c)
{
    const int N = p->n, NS2 = (N + 1) / 2;
    c[0] *= SQRT2F;
    for (int k = 1, kc = N - 1; k < NS2; ++k, --kc) {
        float t1 = c[k] + c[kc], t2 = c[k] - c[kc];
        c[k] = p->dtw[k - 1] * t2 + p->dtw[kc - 1] * t1;
        c[kc] = p->dtw[k - 1] * t1 - p->dtw[kc - 1] * t2;
    }
    if ((N & 1) == 0) c[NS2] *= 2.0f * p->dtw[NS2 - 1];
    rfft_exec(p, c, p->norm, 1);
    for (int k = 1; k < N - 1; k += 2) { float t = c[k]; c[k] = t - c[k + 1]; c[k + 1] = t + c[k + 1]; }
}

/* watermarking.py:76-83: dct(dct(block.T).T) -- axis 0 (columns) first, then rows */
static void dct2d(const dct_plan *p, float *blk, int inverse)
{
    const int n = p->n;
    float col[ORC_MAXB];
    for (int j = 0; j < n; ++j) {
        for (int i = 0; i < n; ++i) col[i] = blk[i * n + j];
        if (inverse) dct3_1d(p, col); else dct2_1d(p, col);
        for (int i = 0; i < n; ++i) blk[i * n + j] = col[i];
    }
    for (int i = 0; i < n; ++i) {
        if (inverse) dct3_1d(p, blk + i * n); else dct2_1d(p, blk + i * n);
    }
}

/* ------------------------------------------------------------------------ */
/* N5 / N6: SVD of one b x b block -- specified one-sided Jacobi in f64     */
/* ------------------------------------------------------------------------ */
#define JAC_MAX_SWEEPS 32
/* Rotate pair (i,j) iff   gamma^2 > TOL2 * alpha * beta          (relative, TOL = 2^-50)
 *                   and   gamma^2 > C * (alpha + beta)           (noise floor, C = 2^-103 * F)
 * with F = ||D||_F^2.  Rotations against large columns leave rounding noise of
 * about eps*sigma_max in every column; the second test stops rotations that only
 * chase that noise (gamma's noise is ~eps*sigma_max*(|a_i|+|a_j|), and
 * (|a_i|+|a_j|)^2 <= 2(alpha+beta)).  Without it rank-deficient blocks never
 * converge; with an F-proportional floor instead, tiny singular triplets stay
 * unresolved and structured covers lose bit-exactness. */
#define JAC_TOL2 7.888609052210118e-31 /* 2^-100 */
#define JAC_C2 9.860761315262648e-32   /* 2^-103 = 2 * (2^-52)^2 */

/* Row chunks of the dot products: P chunks of R = ceil(b/P) contiguous rows (the
 * last ones shorter or empty), their fma-chain partial sums combined by a balanced
 * pairwise tree.  P is the number of GPU lanes per block (a power of two, so the
 * xor butterfly realises the tree); empty chunks contribute +0, which leaves every
 * sum unchanged.  DESIGN.md 3.4. */
static int jac_chunks(int b)
{
    switch (b) {
    case 4: return 1;
    case 6: case 8: return 2;
    case 10: case 12: return 4;
    default: return 8; /* 14, 16 */
    }
}

static double tree_sum(double *v, int n)
{
    while (n > 1) {
        for (int k = 0; k < n / 2; ++k) v[k] = v[2 * k] + v[2 * k + 1];
        n /= 2;
    }
    return v[0];
}

/* sum_r x[r*ldx] * y[r*ldy] in the contract order */
static double cdot(const double *x, const double *y, int ld, int b)
{
    const int P = jac_chunks(b), R = (b + P - 1) / P;
    double part[ORC_MAXB];
    for (int q = 0; q < P; ++q) {
        double acc = 0.0;
        for (int r = q * R; r < (q + 1) * R && r < b; ++r) acc = fma(x[r * ld], y[r * ld], acc);
        part[q] = acc;
    }
    return tree_sum(part, P);
}

/* round-robin (circle method) pair schedule: round s, slot p -> (i, j), i < j */
static void jac_pairs(int b, int s, int p, int *pi, int *pj)
{
    /* L = [0, 1..b-1 rotated by s]; pairs (L[p], L[b-1-p]) */
    int L[ORC_MAXB];
    L[0] = 0;
    for (int k = 1; k < b; ++k) L[k] = 1 + ((k - 1 + s) % (b - 1));
    int a = L[p], c = L[b - 1 - p];
    *pi = a < c ? a : c;
    *pj = a < c ? c : a;
}

/* 1/sqrt(x) for normal x > 0 from IEEE operations only: integer seed
 * (0x5fe6eb50c7b537a9 - bits/2, relative error <= 3.5%) and four Newton steps
 * y <- y * (1.5 - (x/2) y^2), each as t = y*y; u = fma(-x/2, t, 1.5); y = y*u
 * (error 3.5e-2 -> 1.8e-3 -> 4.6e-6 -> 3e-11 -> rounding level).  Unlike the
 * hardware v_rsq_f64 (not correctly rounded, not specified to the bit) every
 * step is reproducible in C and on the GPU.  DESIGN.md 3.4. */
static double rsqrt_n(double x)
{
    uint64_t i;
    double y;
    memcpy(&i, &x, 8);
    i = 0x5fe6eb50c7b537a9ull - (i >> 1);
    memcpy(&y, &i, 8);
    const double hx = 0.5 * x;
    for (int k = 0; k < 4; ++k) {
        const double t = y * y;
        const double u = fma(-hx, t, 1.5);
        y = y * u;
    }
    return y;
}

/* f32 phase: the gfx950 hardware v_rsq_f32 (one instruction on the GPU; not correctly
 * rounded and not specified to the bit), modelled by its measured truth table.  On every
 * positive normal input its result is a power-of-two scaling of the result on the
 * canonical input with the same significand and exponent parity,
 *     rsq(m 2^e) = rsq(m 2^p) 2^-(e-p)/2,  p = e mod 2,  m 2^p in [1, 4)
 * (checked on the GPU for all 2^31 positive normal floats: tools/micro/trans_table.hip),
 * and on the 2^24 canonical inputs it is f32(1 / sqrt(f64(x))) plus a delta of -1, 0 or
 * +1 ulp, stored in tests/golden/gfx950_trans_delta.npz (tools/trans_table.py; oracle.py
 * hands the table over with orc_set_rsq_table).  Phase 1 only: a preconditioner, so the
 * contract can take the cheap instruction; the f64 phase keeps rsqrt_n. */
static const int8_t *g_rsq_delta = NULL;
void orc_set_rsq_table(const int8_t *delta) { g_rsq_delta = delta; }

static float rsq_hw(float x)
{
    uint32_t bx, cb, rb;
    memcpy(&bx, &x, 4);
    const int ex = (int)(bx >> 23);
    if (g_rsq_delta == NULL || ex == 0 || ex == 255 || (bx >> 31)) abort(); /* table missing / outside the model */
    const int e = ex - 127, p = e & 1;
    const uint32_t m = bx & 0x7FFFFFu;
    cb = ((uint32_t)(127 + p) << 23) | m;
    float xc, r;
    memcpy(&xc, &cb, 4);
    r = (float)(1.0 / sqrt((double)xc));
    memcpy(&rb, &r, 4);
    rb = (uint32_t)((int32_t)rb + g_rsq_delta[((uint32_t)p << 23) | m]);
    memcpy(&r, &rb, 4);
    return ldexpf(r, -((e - p) / 2));
}
float orc_rsq_hw(float x) { return rsq_hw(x); } /* tests: the model itself */

/* Rotation of pair (i,j) from alpha = |a_i|^2, beta = |a_j|^2, gamma = a_i.a_j
 * (DESIGN.md 3.4).  With d = beta - alpha, g = 2 gamma, x = d^2 + g^2,
 * r = x rsqrt(x) (= sqrt x), w = |d| + r and q = rsqrt(2 r w):  c = w q,
 * s = sgn(d) g q (t = s/c is the small root of t^2 gamma + t d - gamma = 0), and
 * t*gamma = sgn(d) g^2 r q^2 updates the column norms: alpha' = alpha - t gamma,
 * beta' = beta + t gamma.  c^2 + s^2 = (w^2 + g^2)/(2 r w) = 1 exactly in real
 * arithmetic, whatever the rounding of r. */
static void rotation(double alpha, double beta, double gamma, double *c, double *s, double *tg)
{
    const double d = beta - alpha;
    const double g = gamma + gamma;
    const double x = fma(d, d, g * g);
    const double r = x * rsqrt_n(x);
    const double w = fabs(d) + r;
    const double q = rsqrt_n((r + r) * w);
    const double sg = copysign(1.0, d);
    *c = w * q;
    *s = (g * sg) * q;
    *tg = (((g * g) * r) * (q * q)) * sg;
}

static void rotationf(float alpha, float beta, float gamma, float *c, float *s, float *tg)
{
    const float d = beta - alpha;
    const float g = gamma + gamma;
    const float x = fmaf(d, d, g * g);
    const float r = x * rsq_hw(x);
    const float w = fabsf(d) + r;
    const float q = rsq_hw((r + r) * w);
    const float sg = copysignf(1.0f, d);
    *c = w * q;
    *s = (g * sg) * q;
    *tg = (((g * g) * r) * (q * q)) * sg;
}

static float tree_sumf(float *v, int n)
{
    while (n > 1) {
        for (int k = 0; k < n / 2; ++k) v[k] = v[2 * k] + v[2 * k + 1];
        n /= 2;
    }
    return v[0];
}

/* f32 twin of cdot() (same chunks, fmaf chains, pairwise tree) */
static float cdotf(const float *x, const float *y, int ld, int b)
{
    const int P = jac_chunks(b), R = (b + P - 1) / P;
    float part[ORC_MAXB];
    for (int q = 0; q < P; ++q) {
        float acc = 0.0f;
        for (int r = q * R; r < (q + 1) * R && r < b; ++r) acc = fmaf(x[r * ld], y[r * ld], acc);
        part[q] = acc;
    }
    return tree_sumf(part, P);
}

/* Phase 1 of the SVD: at most jac32_max_sweeps(b) one-sided Jacobi
 * sweeps in f32 on A32 = D, accumulating V32 (a preconditioner: its V only has to
 * be close to the right singular vectors; phase 3 makes them f64-accurate).
 * Rotate iff gamma^2 > 2^-48 F^2 (gamma above the f32 noise of the whole block),
 * gamma^2 > 2^-45 F (alpha+beta) and gamma^2 > 2^-40 alpha beta.  Blocks with
 * F < 2^-30 skip the phase (V32 = I), which keeps every square in the normal range. */
#ifndef JAC32_MAX_SWEEPS
#define JAC32_MAX_SWEEPS 4
#endif
static int jac32_max_sweeps(int b) { (void)b; return JAC32_MAX_SWEEPS; }
#define JAC32_TOL2 9.094947017729282e-13f /* 2^-40 */
#define JAC32_C2 2.842170943040401e-14f   /* 2^-45 */
#define JAC32_C2A 3.552713678800501e-15f  /* 2^-48 */
#define JAC32_FMIN 9.313225746154785e-10f /* 2^-30 */
static int jacobi_f32(float *A, float *V, int b)
{
    int sweep;
    float F = 0.0f, nrm[ORC_MAXB];
    for (int k = 0; k < b; ++k) F += cdotf(A + k, A + k, b, b);
    if (!(F >= JAC32_FMIN)) return 0;
    const float c2 = JAC32_C2 * F, c2a = JAC32_C2A * (F * F);
    for (sweep = 0; sweep < jac32_max_sweeps(b); ++sweep) {
        int rotated = 0;
        for (int k = 0; k < b; ++k) nrm[k] = cdotf(A + k, A + k, b, b);
        for (int st = 0; st < b - 1; ++st)
            for (int p = 0; p < b / 2; ++p) {
                int i, j;
                jac_pairs(b, st, p, &i, &j);
                const float alpha = nrm[i], beta = nrm[j];
                const float gamma = cdotf(A + i, A + j, b, b);
                const float g2 = gamma * gamma;
                if (g2 <= c2a || g2 <= c2 * (alpha + beta) || g2 <= (JAC32_TOL2 * alpha) * beta) continue;
                rotated = 1;
                float c, sn, tg;
                rotationf(alpha, beta, gamma, &c, &sn, &tg);
                nrm[i] = alpha - tg;
                nrm[j] = beta + tg;
                for (int r = 0; r < b; ++r) {
                    const float x = A[r * b + i], y = A[r * b + j];
                    A[r * b + i] = fmaf(-sn, y, c * x);
                    A[r * b + j] = fmaf(sn, x, c * y);
                }
                for (int r = 0; r < b; ++r) {
                    const float x = V[r * b + i], y = V[r * b + j];
                    V[r * b + i] = fmaf(-sn, y, c * x);
                    V[r * b + j] = fmaf(sn, x, c * y);
                }
            }
        if (!rotated) { ++sweep; break; }
    }
    return sweep;
}

/* Phase 2: one Bjorck / Newton-Schulz step toward the orthogonal
 * polar factor, V <- V N with N = 1.5 I - 0.5 V^T V.  (V^T V)_jk is cdot() over
 * rows; N_kk = fma(-0.5, Q_kk, 1.5), N_jk = -0.5 Q_jk; (V N)_rk is an fma chain
 * over j = 0..b-1.  Two steps take the f32 phase's ~1e-6 to rounding level. */
#define JAC_BJORCK_STEPS 2
static void bjorck(double *V, int b)
{
    double N[ORC_MAXB * ORC_MAXB], T[ORC_MAXB * ORC_MAXB];
    for (int j = 0; j < b; ++j)
        for (int k = j; k < b; ++k) {
            const double q = cdot(V + j, V + k, b, b);
            N[j * b + k] = N[k * b + j] = (j == k) ? fma(-0.5, q, 1.5) : -0.5 * q;
        }
    for (int r = 0; r < b; ++r)
        for (int k = 0; k < b; ++k) {
            double acc = 0.0;
            for (int j = 0; j < b; ++j) acc = fma(V[r * b + j], N[j * b + k], acc);
            T[r * b + k] = acc;
        }
    memcpy(V, T, sizeof(double) * b * b);
}

/* A (b x b, row-major, f64) is overwritten with A*V; V (row-major) accumulates.
 * Column norms are recomputed (contract dot) at the start of every sweep and
 * updated with t*gamma inside it.  Returns sweeps done. */
static int jacobi(double *A, double *V, int b, int want_v)
{
    int sweep;
    double F = 0.0, nrm[ORC_MAXB];
    for (int k = 0; k < b; ++k) F += cdot(A + k, A + k, b, b);
    const double c2 = JAC_C2 * F;
    for (sweep = 0; sweep < JAC_MAX_SWEEPS; ++sweep) {
        int rotated = 0;
        for (int k = 0; k < b; ++k) nrm[k] = cdot(A + k, A + k, b, b);
        for (int st = 0; st < b - 1; ++st) {
            for (int p = 0; p < b / 2; ++p) {
                int i, j;
                jac_pairs(b, st, p, &i, &j);
                const double alpha = nrm[i], beta = nrm[j];
                const double gamma = cdot(A + i, A + j, b, b);
                const double g2 = gamma * gamma;
                if (g2 <= c2 * (alpha + beta) || g2 <= (JAC_TOL2 * alpha) * beta) continue;
                rotated = 1;
                double c, sn, tg;
                rotation(alpha, beta, gamma, &c, &sn, &tg);
                nrm[i] = alpha - tg;
                nrm[j] = beta + tg;
                for (int r = 0; r < b; ++r) {
                    const double x = A[r * b + i], y = A[r * b + j];
                    A[r * b + i] = fma(-sn, y, c * x);
                    A[r * b + j] = fma(sn, x, c * y);
                }
                if (want_v)
                    for (int r = 0; r < b; ++r) {
                        const double x = V[r * b + i], y = V[r * b + j];
                        V[r * b + i] = fma(-sn, y, c * x);
                        V[r * b + j] = fma(sn, x, c * y);
                    }
            }
        }
        if (!rotated) { ++sweep; break; }
    }
    return sweep;
}

static void mul_dv(const float *D, const double *V, double *A, int b)
{
    for (int r = 0; r < b; ++r)
        for (int k = 0; k < b; ++k) {
            double acc = 0.0;
            for (int j = 0; j < b; ++j) acc = fma((double)D[r * b + j], V[j * b + k], acc);
            A[r * b + k] = acc;
        }
}

/* One sweep of the f64 Jacobi of jacobi() (same schedule, tests and rotation); returns 1
 * if it rotated a pair. */
static int jacobi_sweep(double *A, double *V, int b, double c2)
{
    int rotated = 0;
    double nrm[ORC_MAXB];
    for (int k = 0; k < b; ++k) nrm[k] = cdot(A + k, A + k, b, b);
    for (int st = 0; st < b - 1; ++st)
        for (int p = 0; p < b / 2; ++p) {
            int i, j;
            jac_pairs(b, st, p, &i, &j);
            const double alpha = nrm[i], beta = nrm[j];
            const double gamma = cdot(A + i, A + j, b, b);
            const double g2 = gamma * gamma;
            if (g2 <= c2 * (alpha + beta) || g2 <= (JAC_TOL2 * alpha) * beta) continue;
            rotated = 1;
            double c, sn, tg;
            rotation(alpha, beta, gamma, &c, &sn, &tg);
            nrm[i] = alpha - tg;
            nrm[j] = beta + tg;
            for (int r = 0; r < b; ++r) {
                const double x = A[r * b + i], y = A[r * b + j];
                A[r * b + i] = fma(-sn, y, c * x);
                A[r * b + j] = fma(sn, x, c * y);
            }
            for (int r = 0; r < b; ++r) {
                const double x = V[r * b + i], y = V[r * b + j];
                V[r * b + i] = fma(-sn, y, c * x);
                V[r * b + j] = fma(sn, x, c * y);
            }
        }
    return rotated;
}

/* ---- Phase 3 with a Newton finish ---------------------------------------
 * Once a sweep has left only tiny couplings, one first-order Newton step replaces the
 * sweeps that would follow (typically a rotating sweep of tiny angles plus the sweep that
 * finds nothing to rotate).  With V orthogonal to rounding level and A = D V, the step
 * V' = V (I + F), A' = A (I + F) with
 *     F_ij = f32(G_ij) / f32(G_jj - G_ii),  F_ji = -F_ij  (i < j),  F_kk = 0,  G = A^T A
 * (contract dots; IEEE f32 divide; a coupling the Jacobi's own tests would not rotate --
 * relative 2^-50, noise floor 2^-103 F (alpha+beta) -- gives F_ij = 0) makes A'^T A'
 * diagonal to second order.  It is taken, and ends the block, only when every
 * |F_ij| <= 2^-27: the neglected terms (second order in F, and (I+F)^T (I+F) - I = -F^2)
 * are then below f64 rounding (times the gap amplification every f64 method carries).
 * The correction X F is formed in f32 from f32(X) (fma chain over i != j; its error,
 * <= ~2^-24 |X| |F|, is below f64 rounding at that size) and added in f64.  Otherwise
 * the block takes the next sweep.  Per block: sweep; if it rotated nothing, done (the
 * Jacobi's own test); Newton try; repeat (at most JAC_MAX_SWEEPS sweeps). */
#define NWT_APPLY 7.450580596923828e-09f /* 2^-27 */
static int g_newton_max_b = ORC_MAXB; /* the Newton finish for b <= this (0: phase 3 = jacobi() for every b) */
void orc_set_newton_finish(int on) { g_newton_max_b = on ? ORC_MAXB : 0; } /* studies only: tools/exp */
void orc_set_newton_max_b(int b) { g_newton_max_b = b; }

/* X <- X + f64(f32(X) F) row by row (fma chain over i != j in f32) */
static void apply_f(double *X, const float *F, int b)
{
    for (int r = 0; r < b; ++r) {
        float xr[ORC_MAXB], cr[ORC_MAXB];
        for (int i = 0; i < b; ++i) xr[i] = (float)X[r * b + i];
        for (int j = 0; j < b; ++j) {
            float acc = 0.0f;
            for (int i = 0; i < b; ++i)
                if (i != j) acc = fmaf(xr[i], F[i * b + j], acc);
            cr[j] = acc;
        }
        for (int j = 0; j < b; ++j) X[r * b + j] = X[r * b + j] + (double)cr[j];
    }
}

/* The step's acceptance test (round 6; tests/k_corpus.py).  Besides every
 * |F_ij| <= 2^-27, the step's neglected second-order terms must stay small on every pair's
 * own scale: they put a coupling of about sum_i F_ij F_ik G_ii on the pair (j, k), with G_ii up
 * to sigma_1^2, and the absolute test alone left the small triplets of graded blocks
 * (sigma_k ~ 1e-5 sigma_1) off by up to 447 units of 2^-53 sigma_1 / g_k.  With x = 2^27 |F|,
 * r_k = f32(G_kk) * (1 / f32(max G)) and q_j = sum_i x_ij^2 r_i -- an fmaf chain per column in
 * the sweep's pair order (round s = 0..b-2, each round's pair (i, j) adding x^2 r_j to q_i and
 * x^2 r_i to q_j) -- the step is taken only if every pair has q_j q_k <= 64 (r_j + r_k): by
 * Cauchy-Schwarz sum_i |F_ij F_ik| G_ii <= 2^-51 (sigma_j + sigma_k) sigma_1, so the pair's
 * rotation error stays within ~12 units of 2^-53 sigma_1 / g.  On the pixel-derived covers of
 * the sweep study it rejects no step the absolute test took.  All f32 IEEE operations in a
 * fixed order: the device evaluates it bit for bit alike (and may skip the pair tests when
 * (max q)^2 <= 128 min r, which implies every one of them in f32). */
static int g_newton_scaled = 1;
void orc_set_newton_scaled(int on) { g_newton_scaled = on; } /* studies only: 0 = the round-5 test */

static int newton_scaled_ok(const double *G, const float *F, int b)
{
    double gmax = 0.0;
    for (int k = 0; k < b; ++k) gmax = G[k] > gmax ? G[k] : gmax;
    const float ginv = 1.0f / (float)gmax;
    float r[ORC_MAXB], qw[ORC_MAXB];
    for (int k = 0; k < b; ++k) {
        r[k] = (float)G[k] * ginv;
        qw[k] = 0.0f;
    }
    for (int s = 0; s < b - 1; ++s)
        for (int p = 0; p < b / 2; ++p) {
            int i, j;
            jac_pairs(b, s, p, &i, &j);
            const float x = fabsf(F[i * b + j]) * 134217728.0f, x2 = x * x; /* 2^27 |F| <= 1 */
            qw[i] = fmaf(x2, r[j], qw[i]);
            qw[j] = fmaf(x2, r[i], qw[j]);
        }
    int ok = 1;
    for (int j = 0; j < b; ++j)
        for (int k = j + 1; k < b; ++k) ok &= qw[j] * qw[k] <= 64.0f * (r[j] + r[k]);
    return ok;
}

/* Returns 1 if the step was taken (the block is done). */
static int newton_try(double *A, double *V, int b, double c2)
{
    double G[ORC_MAXB];
    float F[ORC_MAXB * ORC_MAXB];
    int ok = 1;
    for (int k = 0; k < b; ++k) G[k] = cdot(A + k, A + k, b, b);
    for (int i = 0; i < b; ++i) {
        F[i * b + i] = 0.0f;
        for (int j = i + 1; j < b; ++j) {
            const double g = cdot(A + i, A + j, b, b), g2 = g * g;
            float f = 0.0f;
            if (!(g2 <= c2 * (G[i] + G[j]) || g2 <= (JAC_TOL2 * G[i]) * G[j])) f = (float)g / (float)(G[j] - G[i]);
            F[i * b + j] = f;
            F[j * b + i] = -f;
            ok &= fabsf(f) <= NWT_APPLY; /* NaN / inf fail */
        }
    }
    if (ok && g_newton_scaled) ok = newton_scaled_ok(G, F, b);
    if (!ok) return 0;
    apply_f(V, F, b);
    apply_f(A, F, b);
    return 1;
}

/* returns sweeps | (Newton steps << 16) */
static int jacobi_newton(double *A, double *V, int b)
{
    double F = 0.0;
    for (int k = 0; k < b; ++k) F += cdot(A + k, A + k, b, b);
    const double c2 = JAC_C2 * F;
    int sweeps;
    for (sweeps = 1; sweeps <= JAC_MAX_SWEEPS; ++sweeps) {
        if (!jacobi_sweep(A, V, b, c2)) break;
        if (newton_try(A, V, b, c2)) return sweeps | (1 << 16);
    }
    return sweeps > JAC_MAX_SWEEPS ? JAC_MAX_SWEEPS : sweeps;
}

/* Full SVD of one block in f64, before rounding: D (b x b f32 row-major) -> U (b x b,
 * u[r][k]), sig (b), V (b x b, v[r][k]), sorted by descending sig.  Zero block: U = V = I.
 * Returns the sweeps done: f64 sweeps | (f32 sweeps << 8). */
int orc_svd_block_f64(const float *D, int b, double *U, double *sig, double *V)
{
    double A[ORC_MAXB * ORC_MAXB];
    int allzero = 1;
    for (int k = 0; k < b * b; ++k) { A[k] = D[k]; if (D[k] != 0.0f) allzero = 0; }
    for (int r = 0; r < b; ++r) for (int k = 0; k < b; ++k) V[r * b + k] = (r == k) ? 1.0 : 0.0;
    if (allzero) {
        /* N6: LAPACK returns U = I, Vt = I for the zero matrix */
        for (int r = 0; r < b; ++r) for (int k = 0; k < b; ++k) U[r * b + k] = (r == k);
        for (int k = 0; k < b; ++k) sig[k] = 0.0;
        return 0;
    }
    /* phase 1: f32 Jacobi on D; phase 2: V0 = Bjorck^2(f64(V32)); phase 3: f64
     * Jacobi on A0 = D V0 (fma chain over j), accumulating onto V0 (with the
     * Newton finish) */
    float A32[ORC_MAXB * ORC_MAXB], V32[ORC_MAXB * ORC_MAXB];
    for (int k = 0; k < b * b; ++k) { A32[k] = D[k]; V32[k] = (k / b == k % b) ? 1.0f : 0.0f; }
    const int s32 = jacobi_f32(A32, V32, b);
    for (int k = 0; k < b * b; ++k) V[k] = V32[k];
    int sweeps;
    for (int it = 0; it < JAC_BJORCK_STEPS; ++it) bjorck(V, b);
    mul_dv(D, V, A, b);
    if (b <= g_newton_max_b) sweeps = jacobi_newton(A, V, b) | (s32 << 8);
    else sweeps = jacobi(A, V, b, 1) | (s32 << 8);
    for (int k = 0; k < b; ++k) {
        sig[k] = sqrt(cdot(A + k, A + k, b, b));
        if (sig[k] == 0.0) {
            for (int r = 0; r < b; ++r) U[r * b + k] = 0.0;
        } else {
            const double inv = 1.0 / sig[k];
            for (int r = 0; r < b; ++r) U[r * b + k] = A[r * b + k] * inv;
        }
    }
    /* odd-even transposition sort, descending on the f64 singular values */
    for (int round = 0; round < b; ++round)
        for (int k = round & 1; k + 1 < b; k += 2)
            if (sig[k] < sig[k + 1]) {
                double ts = sig[k]; sig[k] = sig[k + 1]; sig[k + 1] = ts;
                for (int r = 0; r < b; ++r) {
                    double tu = U[r * b + k]; U[r * b + k] = U[r * b + k + 1]; U[r * b + k + 1] = tu;
                    double tv = V[r * b + k]; V[r * b + k] = V[r * b + k + 1]; V[r * b + k + 1] = tv;
                }
            }
    return sweeps;
}

/* Full SVD of one block: D (b x b f32 row-major) -> U (b x b), S (b), Vt (b x b), f32, sorted descending.
 * Returns the sweeps done: f64 sweeps | (f32 sweeps << 8). */
int orc_svd_block(const float *D, int b, float *U, float *S, float *Vt)
{
    double U64[ORC_MAXB * ORC_MAXB], V64[ORC_MAXB * ORC_MAXB], sig[ORC_MAXB];
    const int sweeps = orc_svd_block_f64(D, b, U64, sig, V64);
    for (int k = 0; k < b; ++k) {
        S[k] = (float)sig[k];
        for (int r = 0; r < b; ++r) { U[r * b + k] = (float)U64[r * b + k]; Vt[k * b + r] = (float)V64[r * b + k]; }
    }
    return sweeps;
}

void orc_svd_blocks_f64(const float *D, int64_t nb, int b, double *U, double *S, double *V, int nthreads)
{
    if (nthreads < 1) nthreads = 1;
#pragma omp parallel for num_threads(nthreads) schedule(static)
    for (int64_t k = 0; k < nb; ++k) orc_svd_block_f64(D + k * b * b, b, U + k * b * b, S + k * b, V + k * b * b);
}

/* sigma_1 only (extract path), Jacobi route: f32(max_k ||(A V)_k||) */
float orc_sigma1_block(const float *D, int b)
{
    double A[ORC_MAXB * ORC_MAXB];
    for (int k = 0; k < b * b; ++k) A[k] = D[k];
    jacobi(A, NULL, b, 0);
    double m = 0.0;
    for (int k = 0; k < b; ++k) {
        double s = sqrt(cdot(A + k, A + k, b, b));
        if (s > m) m = s;
    }
    return (float)m;
}

/* Conditioning test of the hybrid route.  Where the f64 Jacobi and LAPACK part ways in
 * the last bits, the f32-rounded factors can differ, and with them the reconstructed
 * block: both methods' factor errors grow like eps * sigma_1 / min(gap_k, sigma_k)
 * (gap_k = distance of sigma_k to the nearest other singular value).  A block is
 * flagged when that amplification exceeds 2^20 for any singular triplet that reaches
 * the output (f32(sigma_k) != 0).  Measured (tests/test_oracle_lapack.py): every
 * block whose reconstruction differs between the two routes has amplification
 * >= 6e7; flagged fractions 0.01 % (noise covers) to 0.5 % (camera-like covers).
 * sig: the f64 singular values of the Jacobi route (any order). */
#define ORC_FLAG_T 1048576.0 /* 2^20 */
int orc_svd_flag(const double *sig, int b)
{
    double s1 = 0.0;
    for (int k = 0; k < b; ++k) if (sig[k] > s1) s1 = sig[k];
    if (s1 == 0.0) return 0; /* zero block: U = V = I exactly on both routes (N6) */
    double m = s1;
    for (int k = 0; k < b; ++k) {
        if ((float)sig[k] == 0.0f) continue;
        double g = sig[k];
        for (int j = 0; j < b; ++j) {
            if (j == k) continue;
            const double d = fabs(sig[k] - sig[j]);
            if (d < g) g = d;
        }
        if (g < m) m = g;
    }
    return m * ORC_FLAG_T < s1;
}

/* One block's factors by route; returns 1 when the dgesdd route produced them.  The hybrid
 * route also needs the block's watermark byte, alpha and chroma for its byte certificate
 * (tmfwm_cert.cpp); cbs == NULL skips the certificate (the conditioning test alone). */
static int svd_block_route(const float *D, int b, int mode, float *U, float *S, float *Vt, uint8_t w, double alpha,
                           const float *cbs, const float *crs)
{
    if (mode == ORC_SVD_LAPACK) {
        orc_lp_svd_block_f32(D, b, U, S, Vt);
        return 1;
    }
    double U64[ORC_MAXB * ORC_MAXB], V64[ORC_MAXB * ORC_MAXB], sig[ORC_MAXB];
    orc_svd_block_f64(D, b, U64, sig, V64);
    if (mode == ORC_SVD_HYBRID &&
        (orc_svd_flag(sig, b) || (cbs && orc_cert_block(D, U64, sig, V64, b, w, alpha, cbs, crs, NULL)))) {
        orc_lp_svd_block_f32(D, b, U, S, Vt);
        return 1;
    }
    for (int k = 0; k < b; ++k) {
        S[k] = (float)sig[k];
        for (int r = 0; r < b; ++r) { U[r * b + k] = (float)U64[r * b + k]; Vt[k * b + r] = (float)V64[r * b + k]; }
    }
    return 0;
}

int orc_svd_block_mode(const float *D, int b, int mode, float *U, float *S, float *Vt)
{
    return svd_block_route(D, b, mode, U, S, Vt, 0, 0.0, NULL, NULL);
}

/* sigma_1 by route: the Jacobi value, or LAPACK's S[0] (the reference's value; the
 * device extract certifies it or computes it on the dgesdd route). */
static float sigma1_mode(const float *D, int b, int mode)
{
    if (mode == ORC_SVD_JACOBI) return orc_sigma1_block(D, b);
    float U[ORC_MAXB * ORC_MAXB], S[ORC_MAXB], Vt[ORC_MAXB * ORC_MAXB];
    orc_lp_svd_block_f32(D, b, U, S, Vt);
    return S[0];
}

/* N7 blend + N8 reconstruct: S'[0] = f32(f64(S0) + alpha*(w/255.0)); M = U @ (diag(S') @ Vt) */
void orc_blend_reconstruct(const float *U, const float *S, const float *Vt, int b, uint8_t w, double alpha, float *M)
{
    float Sp[ORC_MAXB], B[ORC_MAXB * ORC_MAXB];
    for (int k = 0; k < b; ++k) Sp[k] = S[k];
    Sp[0] = (float)((double)S[0] + alpha * ((double)w / 255.0));
    for (int k = 0; k < b; ++k) for (int j = 0; j < b; ++j) B[k * b + j] = Sp[k] * Vt[k * b + j];
    for (int i = 0; i < b; ++i)
        for (int j = 0; j < b; ++j) {
            float acc = 0.0f;
            for (int k = 0; k < b; ++k) acc = fmaf(U[i * b + k], B[k * b + j], acc);
            M[i * b + j] = acc;
        }
}

void orc_blend_reconstruct_blocks(const float *U, const float *S, const float *Vt, int64_t nb, int b, const uint8_t *w, double alpha, float *M)
{
    for (int64_t k = 0; k < nb; ++k)
        orc_blend_reconstruct(U + k * b * b, S + k * b, Vt + k * b * b, b, w[k], alpha, M + k * b * b);
}

/* ------------------------------------------------------------------------ */
/* Exported stage functions                                                 */
/* ------------------------------------------------------------------------ */
int orc_supported_block(int b) { return b >= 4 && b <= 16 && (b & 1) == 0; }

void orc_rgb_to_ycbcr(const uint8_t *rgb, int64_t npix, float *ycc)
{
    for (int64_t p = 0; p < npix; ++p) colour_fwd(rgb[3 * p], rgb[3 * p + 1], rgb[3 * p + 2], ycc + 3 * p, ycc + 3 * p + 1, ycc + 3 * p + 2);
}

void orc_ycbcr_to_rgb(const float *ycc, int64_t npix, uint8_t *rgb)
{
    for (int64_t p = 0; p < npix; ++p) colour_inv(ycc[3 * p], ycc[3 * p + 1], ycc[3 * p + 2], rgb + 3 * p);
}

/* rgb_to_ycbcr of a non-uint8 input (watermarking.py:29): rgb = np.array(img, float32)
 * (the caller's cast), then "/ 255.0" as an f32 divide and the :37-48 rows. */
void orc_rgb_to_ycbcr_f32(const float *rgb, int64_t npix, float *ycc)
{
    for (int64_t p = 0; p < npix; ++p) {
        const double r = rgb[3 * p] / 255.0f, g = rgb[3 * p + 1] / 255.0f, b = rgb[3 * p + 2] / 255.0f;
        ycc[3 * p] = (float)fma(0.114, b, fma(0.299, r, 0.587 * g));
        ycc[3 * p + 1] = (float)fma(0.5, b, fma(-0.169, r, -0.331 * g)) + 0.5f;
        ycc[3 * p + 2] = (float)fma(-0.081, b, fma(0.5, r, -0.419 * g)) + 0.5f;
    }
}

/* ycbcr_to_rgb of a float64 input: img.copy() keeps float64 (:55), so ":58 -= 0.5", the
 * stored dot (:64-67), np.clip (:70) and "* 255" (:73) are all f64; astype(uint8) truncates. */
static uint8_t u8_from_unit_f64(double f)
{
    if (f < 0.0) f = 0.0;
    if (f > 1.0) f = 1.0;
    return (uint8_t)(f * 255.0);
}

void orc_ycbcr_to_rgb_f64(const double *ycc, int64_t npix, uint8_t *rgb)
{
    for (int64_t p = 0; p < npix; ++p) {
        const double Y = ycc[3 * p], CB = ycc[3 * p + 1] - 0.5, CR = ycc[3 * p + 2] - 0.5;
        rgb[3 * p] = u8_from_unit_f64(fma(1.403, CR, fma(1.0, Y, 0.0 * CB)));
        rgb[3 * p + 1] = u8_from_unit_f64(fma(-0.714, CR, fma(1.0, Y, -0.344 * CB)));
        rgb[3 * p + 2] = u8_from_unit_f64(fma(0.0, CR, fma(1.0, Y, 1.773 * CB)));
    }
}

/* IEEE binary16 (numpy float16) held in doubles.  half_round(x) is the binary16 value
 * nearest x (ties to even, gradual underflow, overflow to inf) -- numpy's
 * npy_double_to_half, and the result of every half operation below, since numpy
 * evaluates a half '+', '-', '*' in float32 and rounds once more to half, which for
 * these operations equals the correctly rounded half result (24 >= 2 * 11 + 2 bits). */
static double half_round(double x)
{
    if (x == 0.0 || !isfinite(x)) return x;
    int e;
    frexp(x, &e); /* |x| in [2^(e-1), 2^e) */
    const int q = e - 1 < -14 ? -24 : e - 11; /* ulp exponent: 10 fraction bits; subnormals 2^-24 */
    const double r = ldexp(nearbyint(ldexp(x, -q)), q);
    return fabs(r) >= 65520.0 ? copysign(INFINITY, x) : r;
}

static double half_bits_to_double(uint16_t h)
{
    const int s = h >> 15, e = (h >> 10) & 0x1f, m = h & 0x3ff;
    double v;
    if (e == 0) v = ldexp((double)m, -24);
    else if (e == 31) v = m ? NAN : INFINITY;
    else v = ldexp((double)(m | 0x400), e - 25);
    return s ? -v : v;
}

static uint8_t u8_from_unit_f16(double f) /* f is a half value */
{
    if (f < 0.0) f = 0.0;
    if (f > 1.0) f = 1.0;
    return (uint8_t)half_round(f * 255.0); /* the product is exact in f64, then one half rounding */
}

/* ycbcr_to_rgb of a float16 input (ycc = the raw binary16 bits): every step of the f64
 * path above rounded back to half where numpy stores a half (:58, :64 zeros_like, :73). */
void orc_ycbcr_to_rgb_f16(const uint16_t *ycc, int64_t npix, uint8_t *rgb)
{
    for (int64_t p = 0; p < npix; ++p) {
        const double Y = half_bits_to_double(ycc[3 * p]);
        const double CB = half_round(half_bits_to_double(ycc[3 * p + 1]) - 0.5);
        const double CR = half_round(half_bits_to_double(ycc[3 * p + 2]) - 0.5);
        rgb[3 * p] = u8_from_unit_f16(half_round(fma(1.403, CR, fma(1.0, Y, 0.0 * CB))));
        rgb[3 * p + 1] = u8_from_unit_f16(half_round(fma(-0.714, CR, fma(1.0, Y, -0.344 * CB))));
        rgb[3 * p + 2] = u8_from_unit_f16(half_round(fma(0.0, CR, fma(1.0, Y, 1.773 * CB))));
    }
}

/* nb blocks of b x b, row-major each, in place */
void orc_dct2d_blocks(float *blocks, int64_t nb, int b, int inverse)
{
    const dct_plan *p = plan_for(b);
    for (int64_t k = 0; k < nb; ++k) dct2d(p, blocks + k * b * b, inverse);
}

/* 1-D transforms along contiguous rows (for pinning against scipy row-wise) */
void orc_dct_rows(float *x, int64_t nrows, int n, int inverse)
{
    const dct_plan *p = plan_for(n);
    for (int64_t k = 0; k < nrows; ++k) { if (inverse) dct3_1d(p, x + k * n); else dct2_1d(p, x + k * n); }
}

int orc_svd_blocks(const float *D, int64_t nb, int b, float *U, float *S, float *Vt, int32_t *sweeps)
{
    int maxs = 0;
    for (int64_t k = 0; k < nb; ++k) {
        int s = orc_svd_block(D + k * b * b, b, U + k * b * b, S + k * b, Vt + k * b * b);
        if (sweeps) sweeps[k] = s;
        if (s > maxs) maxs = s;
    }
    return maxs;
}

/* Y plane (H x W f32) -> DCT blocks (nbh*nbw, b, b) */
void orc_gather_blocks(const float *Y, int H, int W, int b, float *blocks)
{
    const int nbh = H / b, nbw = W / b;
    for (int bi = 0; bi < nbh; ++bi)
        for (int bj = 0; bj < nbw; ++bj) {
            float *blk = blocks + ((int64_t)bi * nbw + bj) * b * b;
            for (int r = 0; r < b; ++r)
                for (int c = 0; c < b; ++c) blk[r * b + c] = Y[(int64_t)(bi * b + r) * W + bj * b + c];
        }
}

void orc_scatter_blocks(const float *blocks, int H, int W, int b, float *Y)
{
    const int nbh = H / b, nbw = W / b;
    for (int bi = 0; bi < nbh; ++bi)
        for (int bj = 0; bj < nbw; ++bj) {
            const float *blk = blocks + ((int64_t)bi * nbw + bj) * b * b;
            for (int r = 0; r < b; ++r)
                for (int c = 0; c < b; ++c) Y[(int64_t)(bi * b + r) * W + bj * b + c] = blk[r * b + c];
        }
}

/* One block row (bi) of the embed: Y plane updated in place (ycc: the frame's Cb, Cr). */
static int64_t embed_block_row(float *Y, const float *ycc, int W, int b, int bi, int nbw, const uint8_t *wm, double alpha,
                               int mode)
{
    int64_t fallback = 0;
    const dct_plan *p = plan_for(b);
    float D[ORC_MAXB * ORC_MAXB], U[ORC_MAXB * ORC_MAXB], Vt[ORC_MAXB * ORC_MAXB], S[ORC_MAXB], M[ORC_MAXB * ORC_MAXB];
    float cbs[ORC_MAXB * ORC_MAXB], crs[ORC_MAXB * ORC_MAXB];
    for (int bj = 0; bj < nbw; ++bj) {
        for (int r = 0; r < b; ++r)
            for (int c = 0; c < b; ++c) {
                const int64_t q = (int64_t)(bi * b + r) * W + bj * b + c;
                D[r * b + c] = Y[q];
                cbs[r * b + c] = ycc[3 * q + 1];
                crs[r * b + c] = ycc[3 * q + 2];
            }
        const uint8_t w = wm[(int64_t)bi * nbw + bj];
        dct2d(p, D, 0);                                                     /* :192 */
        fallback += svd_block_route(D, b, mode, U, S, Vt, w, alpha, cbs, crs); /* :195 */
        orc_blend_reconstruct(U, S, Vt, b, w, alpha, M);                   /* :198-201 */
        dct2d(p, M, 1);                                                     /* :204 */
        for (int r = 0; r < b; ++r)
            for (int c = 0; c < b; ++c) Y[(int64_t)(bi * b + r) * W + bj * b + c] = M[r * b + c]; /* :207-210 */
    }
    return fallback;
}

static int clamp_threads(int nthreads) { return nthreads < 1 ? 1 : nthreads; }

/* embed_watermark arithmetic for one frame (watermarking.py:163-216).
 * rgb: H x W x 3 u8; wm: (H/b) x (W/b) u8 tile (already resized); out: H x W x 3 u8.
 * mode: ORC_SVD_*; n_fallback (optional) receives the blocks that took the dgesdd route. */
int orc_embed_frame_mode(const uint8_t *rgb, int H, int W, const uint8_t *wm, int b, double alpha, uint8_t *out,
                         int nthreads, int mode, int64_t *n_fallback)
{
    if (!orc_supported_block(b) || H < 0 || W < 0) return -1;
    plans_init();
    const int64_t npix = (int64_t)H * W;
    float *ycc = (float *)malloc(sizeof(float) * 3 * (npix ? npix : 1));
    float *Y = (float *)malloc(sizeof(float) * (npix ? npix : 1));
    if (!ycc || !Y) { free(ycc); free(Y); return -2; }
    nthreads = clamp_threads(nthreads);
#pragma omp parallel for num_threads(nthreads) schedule(static)
    for (int64_t q = 0; q < npix; ++q) {
        colour_fwd(rgb[3 * q], rgb[3 * q + 1], rgb[3 * q + 2], ycc + 3 * q, ycc + 3 * q + 1, ycc + 3 * q + 2);
        Y[q] = ycc[3 * q];
    }
    const int nbh = H / b, nbw = W / b;
    int64_t fallback = 0;
#pragma omp parallel for num_threads(nthreads) schedule(dynamic, 1) reduction(+ : fallback)
    for (int bi = 0; bi < nbh; ++bi) fallback += embed_block_row(Y, ycc, W, b, bi, nbw, wm, alpha, mode);
#pragma omp parallel for num_threads(nthreads) schedule(static)
    for (int64_t q = 0; q < npix; ++q) colour_inv(Y[q], ycc[3 * q + 1], ycc[3 * q + 2], out + 3 * q);
    free(ycc);
    free(Y);
    if (n_fallback) *n_fallback = fallback;
    return 0;
}

int orc_embed_frame(const uint8_t *rgb, int H, int W, const uint8_t *wm, int b, double alpha, uint8_t *out, int nthreads)
{
    return orc_embed_frame_mode(rgb, H, W, wm, b, alpha, out, nthreads, ORC_SVD_CONTRACT, NULL);
}

/* extract_watermark arithmetic for one frame pair (watermarking.py:241-289).
 * Both images H x W x 3 (the original already cropped to the watermarked size). out: (H/b) x (W/b). */
int orc_extract_frame_mode(const uint8_t *wrgb, const uint8_t *orgb, int H, int W, int b, double alpha, uint8_t *out,
                           int nthreads, int mode)
{
    if (!orc_supported_block(b) || H < 0 || W < 0) return -1;
    plans_init();
    const int nbh = H / b, nbw = W / b;
    const float alpha32 = (float)alpha;
    const dct_plan *p = plan_for(b);
    nthreads = clamp_threads(nthreads);
#pragma omp parallel for num_threads(nthreads) schedule(dynamic, 1)
    for (int bi = 0; bi < nbh; ++bi) {
        float Dw[ORC_MAXB * ORC_MAXB], Do[ORC_MAXB * ORC_MAXB];
        for (int bj = 0; bj < nbw; ++bj) {
            for (int r = 0; r < b; ++r)
                for (int c = 0; c < b; ++c) {
                    const int64_t q = (int64_t)(bi * b + r) * W + bj * b + c;
                    float y, cb, cr;
                    colour_fwd(wrgb[3 * q], wrgb[3 * q + 1], wrgb[3 * q + 2], &y, &cb, &cr);
                    Dw[r * b + c] = y;
                    colour_fwd(orgb[3 * q], orgb[3 * q + 1], orgb[3 * q + 2], &y, &cb, &cr);
                    Do[r * b + c] = y;
                }
            dct2d(p, Dw, 0);
            dct2d(p, Do, 0);
            const float sw = sigma1_mode(Dw, b, mode), so = sigma1_mode(Do, b, mode);
            /* :285 numpy-2 NEP 50: float32 - float32, then / python float in float32 */
            const float e = (sw - so) / alpha32;
            /* :288-289 stored in f64, clip [0,1], *255 (f64), astype(uint8) */
            double d = (double)e;
            if (d < 0.0) d = 0.0;
            if (d > 1.0) d = 1.0;
            out[(int64_t)bi * nbw + bj] = (uint8_t)(d * 255.0);
        }
    }
    return 0;
}

int orc_extract_frame(const uint8_t *wrgb, const uint8_t *orgb, int H, int W, int b, double alpha, uint8_t *out, int nthreads)
{
    return orc_extract_frame_mode(wrgb, orgb, H, W, b, alpha, out, nthreads, ORC_SVD_CONTRACT);
}

/* Batched helpers for the CPU baseline (frames laid out back to back). */
int orc_embed_batch(const uint8_t *rgb, int64_t n, int H, int W, const uint8_t *wm, int b, double alpha, uint8_t *out, int nthreads)
{
    const int64_t fs = (int64_t)H * W * 3;
    for (int64_t f = 0; f < n; ++f) {
        int rc = orc_embed_frame(rgb + f * fs, H, W, wm, b, alpha, out + f * fs, nthreads);
        if (rc) return rc;
    }
    return 0;
}

int orc_extract_batch(const uint8_t *wrgb, const uint8_t *orgb, int64_t n, int H, int W, int b, double alpha, uint8_t *out, int nthreads)
{
    const int64_t fs = (int64_t)H * W * 3, ts = (int64_t)(H / b) * (W / b);
    for (int64_t f = 0; f < n; ++f) {
        int rc = orc_extract_frame(wrgb + f * fs, orgb + f * fs, H, W, b, alpha, out + f * ts, nthreads);
        if (rc) return rc;
    }
    return 0;
}

/* ------------------------------------------------------------------------ */
/* Watermark preparation (watermarking.py:102-132 after convert("L")):      */
/* Pillow 12.2.0 Image.resize(LANCZOS) on an 8-bit L image -- Resample.c    */
/* precompute_coeffs (double), normalize_coeffs_8bpc (22-bit fixed point),  */
/* horizontal pass over the used rows, then vertical pass -- and the        */
/* ratio-preserving paste on a white canvas.  Pillow is the reference's     */
/* third-party dependency; parity is pinned against PIL itself and the      */
/* golden tiles (tests/test_oracle_golden.py).                              */
/* ------------------------------------------------------------------------ */
#define RS_PRECISION_BITS (32 - 8 - 2)

static double rs_sinc(double x)
{
    if (x == 0.0) return 1.0;
    x = x * 3.14159265358979323846; /* M_PI */
    return sin(x) / x;
}

static double rs_lanczos(double x) { return (-3.0 <= x && x < 3.0) ? rs_sinc(x) * rs_sinc(x / 3) : 0.0; }

/* returns ksize; bounds[2*out], kk[out*ksize] (fixed point) are malloc'ed */
static int rs_coeffs(int inSize, int outSize, int **boundsp, int32_t **kkp)
{
    const float in0 = 0.0f, in1 = (float)inSize; /* box = (0, 0, w, h) as floats */
    double filterscale, scale;
    filterscale = scale = (double)(in1 - in0) / outSize;
    if (filterscale < 1.0) filterscale = 1.0;
    const double support = 3.0 * filterscale;
    const int ksize = (int)ceil(support) * 2 + 1;
    double *kd = (double *)malloc(sizeof(double) * (size_t)outSize * ksize);
    int *bounds = (int *)malloc(sizeof(int) * (size_t)outSize * 2);
    int32_t *kk = (int32_t *)malloc(sizeof(int32_t) * (size_t)outSize * ksize);
    for (int xx = 0; xx < outSize; xx++) {
        const double center = in0 + (xx + 0.5) * scale, ss = 1.0 / filterscale;
        double ww = 0.0;
        int xmin = (int)(center - support + 0.5);
        if (xmin < 0) xmin = 0;
        int xmax = (int)(center + support + 0.5);
        if (xmax > inSize) xmax = inSize;
        xmax -= xmin;
        double *k = kd + (size_t)xx * ksize;
        int x;
        for (x = 0; x < xmax; x++) {
            const double w = rs_lanczos((x + xmin - center + 0.5) * ss);
            k[x] = w;
            ww += w;
        }
        for (x = 0; x < xmax; x++)
            if (ww != 0.0) k[x] /= ww;
        for (; x < ksize; x++) k[x] = 0;
        bounds[xx * 2] = xmin;
        bounds[xx * 2 + 1] = xmax;
    }
    for (size_t i = 0; i < (size_t)outSize * ksize; i++)
        kk[i] = kd[i] < 0 ? (int)(-0.5 + kd[i] * (1 << RS_PRECISION_BITS)) : (int)(0.5 + kd[i] * (1 << RS_PRECISION_BITS));
    free(kd);
    *boundsp = bounds;
    *kkp = kk;
    return ksize;
}

static uint8_t rs_clip8(int v)
{
    v >>= RS_PRECISION_BITS;
    return v < 0 ? 0 : v > 255 ? 255 : (uint8_t)v;
}

/* Image.resize((ow, oh), Image.LANCZOS) of an ih x iw L image into out (oh x ow,
 * row stride ldo).  Returns -1 for an empty size (PIL raises). */
int orc_resize_lanczos(const uint8_t *in, int ih, int iw, int oh, int ow, uint8_t *out, int ldo)
{
    if (ih <= 0 || iw <= 0 || oh <= 0 || ow <= 0) return -1;
    if (oh == ih && ow == iw) { /* Image.resize returns a copy */
        for (int y = 0; y < oh; y++) memcpy(out + (size_t)y * ldo, in + (size_t)y * iw, (size_t)iw);
        return 0;
    }
    int *bh, *bv;
    int32_t *kh, *kv;
    const int need_h = ow != iw, need_v = oh != ih;
    const int ksh = rs_coeffs(iw, ow, &bh, &kh), ksv = rs_coeffs(ih, oh, &bv, &kv);
    const int yfirst = bv[0], ylast = bv[oh * 2 - 2] + bv[oh * 2 - 1];
    const uint8_t *src = in;
    int sw = iw;
    uint8_t *tmp = NULL;
    if (need_h) {
        for (int i = 0; i < oh; i++) bv[i * 2] -= yfirst;
        const int sh = ylast - yfirst;
        tmp = (uint8_t *)malloc((size_t)sh * ow + 1);
        for (int yy = 0; yy < sh; yy++)
            for (int xx = 0; xx < ow; xx++) {
                const int xmin = bh[xx * 2], xmax = bh[xx * 2 + 1];
                const int32_t *k = kh + (size_t)xx * ksh;
                int ss0 = 1 << (RS_PRECISION_BITS - 1);
                for (int x = 0; x < xmax; x++) ss0 += (int)in[(size_t)(yy + yfirst) * iw + x + xmin] * k[x];
                tmp[(size_t)yy * ow + xx] = rs_clip8(ss0);
            }
        src = tmp;
        sw = ow;
    }
    if (need_v) {
        for (int yy = 0; yy < oh; yy++) {
            const int32_t *k = kv + (size_t)yy * ksv;
            const int ymin = bv[yy * 2], ymax = bv[yy * 2 + 1];
            for (int xx = 0; xx < sw; xx++) {
                int ss0 = 1 << (RS_PRECISION_BITS - 1);
                for (int y = 0; y < ymax; y++) ss0 += (int)src[(size_t)(y + ymin) * sw + xx] * k[y];
                out[(size_t)yy * ldo + xx] = rs_clip8(ss0);
            }
        }
    } else {
        for (int y = 0; y < oh; y++) memcpy(out + (size_t)y * ldo, src + (size_t)y * sw, (size_t)sw);
    }
    free(tmp);
    free(bh);
    free(bv);
    free(kh);
    free(kv);
    return 0;
}

/* resize_watermark (watermarking.py:105-132) on an already-"L" watermark:
 * preserve_ratio -> LANCZOS to (int(w*ratio), int(h*ratio)), centred on a white
 * th x tw canvas; otherwise LANCZOS straight to th x tw. */
int orc_prepare_tile(const uint8_t *wm, int wh, int ww, int th, int tw, int preserve_ratio, uint8_t *tile)
{
    if (wh <= 0 || ww <= 0 || th <= 0 || tw <= 0) return -1;
    if (!preserve_ratio) return orc_resize_lanczos(wm, wh, ww, th, tw, tile, tw);
    const double rw = (double)tw / (double)ww, rh = (double)th / (double)wh;
    const double ratio = rw < rh ? rw : rh; /* Python min() keeps the first of equals */
    const int nw = (int)((double)ww * ratio), nh = (int)((double)wh * ratio);
    if (nw <= 0 || nh <= 0) return -1;
    memset(tile, 255, (size_t)th * tw);
    const int px = (tw - nw) / 2, py = (th - nh) / 2;
    return orc_resize_lanczos(wm, wh, ww, nh, nw, tile + (size_t)py * tw + px, tw);
}

/* Synthetic input generator shared with the GPU generator:
 * byte = splitmix64(seed ^ (frame << 40) ^ idx) & 0xFF over the linear HWC index. */
static inline uint64_t splitmix64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

void orc_synth_bytes(uint64_t seed, int64_t frame0, int64_t nframes, int64_t frame_bytes, uint8_t *out)
{
    for (int64_t f = 0; f < nframes; ++f)
        for (int64_t i = 0; i < frame_bytes; ++i)
            out[f * frame_bytes + i] = (uint8_t)(splitmix64(seed ^ ((uint64_t)(frame0 + f) << 40) ^ (uint64_t)i) & 0xFF);
}
