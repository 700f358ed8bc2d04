/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of the f64 SVD the reference calls at
 * /root/reference/modules/watermarking.py:195 (embed) and :279-282 (extract):
 * np.linalg.svd(block) on a float32 b x b block.  numpy 2.2.6 upcasts to f64 and
 * runs LAPACK dgesdd (JOBZ='A') from scipy-openblas64 0.3.29 (LAPACK 3.12.0 Fortran
 * compiled for baseline x86-64, i.e. SSE2 without FMA; BLAS level-1/2 kernels of the
 * OpenBLAS "SkylakeX" DYNAMIC_ARCH core selected on this container's CPU).  The
 * reference's bytes inherit every rounding of that route, so this file restates it
 * operation by operation:
 *
 *   dgesdd path 5 (M >= N, M < MNTHR), JOBZ='A':
 *     dgebrd -> dgebd2 (n < crossover 128): dlarfg + dlarf per column / row
 *     dbdsdc('U','I') -> n <= SMLSIZ (25): dlaset U = VT = I, dlasdq -> dbdsqr
 *     dormbr('Q','L','N') -> dormqr -> dorm2r (k < NB 32): dlarf backwards
 *     dormbr('P','R','T') -> dormlq -> dorml2 on A(1,2), VT(1,2): dlarf backwards
 *   dlarf (3.12.0, with iladlc / iladlr trimming) -> OpenBLAS dgemv_t / dgemv_n / dger
 *   dlarfg -> OpenBLAS dnrm2 (x87 80-bit, 4 accumulators), dlapy2, dscal
 *   dbdsqr -> dlartg (3.10+ la_xlartg), dlas2, dlasv2, dlasr, drot (SkylakeX: fma)
 *
 * The OpenBLAS kernels' operation order was read from the disassembly of
 * libscipy_openblas64_ (dgemv_n_SKYLAKEX, dgemv_t_SKYLAKEX and their 4x4 / 4x2 /
 * 4x1 helpers, dnrm2_k_SKYLAKEX = the x87 nrm2.S, drot) and every stage is pinned
 * bit for bit against that library's own entry points and against np.linalg.svd in
 * tests/test_oracle_lapack.py (this container's CPU selects the SkylakeX core).
 *
 * Storage is LAPACK's: column-major, leading dimension ld, 0-based indices here.
 * Sizes: n <= LP_MAXN (16, the largest block of the app's slider).
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off; long double is x87 extended
 * on x86-64, which is what OpenBLAS's nrm2.S computes in).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#define LP_MAXN 16
#define AT(a, i, j, ld) (a)[(i) + (size_t)(j) * (ld)]

static const double LP_EPS = 0x1p-53;         /* dlamch('E') (rounding: eps = 2^-53) */
static const double LP_PREC = 0x1p-52;        /* dlamch('P') = eps * radix */
static const double LP_SAFMIN = 0x1p-1022;    /* dlamch('S') */
static const double LP_HUGE = 0x1.fffffffffffffp+1023; /* dlamch('O') */

/* ------------------------------------------------------------------------ */
/* OpenBLAS 0.3.29 SkylakeX BLAS kernels (only the call shapes LAPACK uses)  */
/* ------------------------------------------------------------------------ */

/* dnrm2: kernel/x86_64/nrm2.S -- x87 extended precision, four accumulators for
 * the 8-unrolled body (element k of each group of four goes to accumulator k),
 * remainder into accumulator 0, combined as d + ((c + a) + b), fsqrt in extended
 * precision, then stored to double (a second rounding). */
double orc_lp_dnrm2(int n, const double *x, int inc)
{
    if (n <= 0) return 0.0;
    long double a = 0, b = 0, c = 0, d = 0;
    int i = 0;
    for (int g = 0; g < n / 8; ++g)
        for (int h = 0; h < 2; ++h, i += 4) {
            const long double q0 = (long double)x[(size_t)i * inc] * x[(size_t)i * inc];
            const long double q1 = (long double)x[(size_t)(i + 1) * inc] * x[(size_t)(i + 1) * inc];
            const long double q2 = (long double)x[(size_t)(i + 2) * inc] * x[(size_t)(i + 2) * inc];
            const long double q3 = (long double)x[(size_t)(i + 3) * inc] * x[(size_t)(i + 3) * inc];
            d += q3; c += q2; b += q1; a += q0;
        }
    for (; i < n; ++i) a += (long double)x[(size_t)i * inc] * x[(size_t)i * inc];
    long double t = (c + a) + b;
    t = d + t;
    return (double)sqrtl(t);
}

/* y := A^T x, alpha = 1, beta = 0 (interface: y scaled to 0 first).  dgemv_t_4.c:
 * rows in multiples of 4 go through a column kernel -- 4x4 (ymm, fma, lane = row
 * mod 4, reduced (l0+l2)+(l1+l3)) for column groups of four, 4x2 (xmm, mul+add,
 * lane = row mod 2) for a remaining pair, 4x1 (two xmm, mul+add, lane = row mod 4)
 * for a last column -- then the last m mod 4 rows as one contracted expression. */
static void gemv_t(int m, int n, const double *A, int lda, const double *x, int incx, double *y)
{
    const int m3 = m & 3, m1 = m - m3, n4 = n & ~3, n2 = n & 3;
    for (int j = 0; j < n; ++j) {
        const double *a = A + (size_t)j * lda;
        double yy = 0.0;
        if (m1) {
            double t;
            if (j < n4) {
                double l[4] = {0, 0, 0, 0};
                for (int r = 0; r < m1; ++r) l[r & 3] = fma(a[r], x[(size_t)r * incx], l[r & 3]);
                t = (l[0] + l[2]) + (l[1] + l[3]);
            } else if ((n2 & 2) && j < n4 + 2) {
                double l[2] = {0, 0};
                for (int r = 0; r < m1; ++r) l[r & 1] = l[r & 1] + a[r] * x[(size_t)r * incx];
                t = l[0] + l[1];
            } else {
                double l[4] = {0, 0, 0, 0};
                for (int r = 0; r < m1; ++r) l[r & 3] = l[r & 3] + a[r] * x[(size_t)r * incx];
                t = (l[0] + l[2]) + (l[1] + l[3]);
            }
            yy = fma(t, 1.0, yy);
        }
        const double *xt = x + (size_t)m1 * incx;
        if (m3 == 3)
            yy = yy + fma(a[m1 + 2], xt[2 * (size_t)incx], fma(a[m1], xt[0], a[m1 + 1] * xt[incx]));
        else if (m3 == 2)
            yy = yy + fma(a[m1], xt[0], a[m1 + 1] * xt[incx]);
        else if (m3 == 1)
            yy = fma(a[m1], xt[0], yy);
        y[j] = yy;
    }
}

/* y := A x, alpha = 1, beta = 0.  dgemv_n_4.c (SkylakeX): rows in multiples of 4:
 * per group of four columns s = a1 x1; s = fma(a0,x0,s); fma(a2..); fma(a3..);
 * y = fma(1, s, y); then (unit-stride x) a pair: s = a1 x1; s = fma(a0,x0,s);
 * y = fma(1,s,y); then single columns y = y + a*(x*1) (mul + add).  Non-unit x:
 * every column after the groups of four is a single column.  Last m mod 4 rows:
 * t = fma chain over the columns, y = fma(1, t, y). */
static void gemv_n(int m, int n, const double *A, int lda, const double *x, int incx, double *y)
{
    const int m3 = m & 3, m1 = m - m3, n4 = n & ~3;
    for (int r = 0; r < m; ++r) y[r] = 0.0;
    for (int r = 0; r < m1; ++r) {
        int j = 0;
        for (; j < n4; j += 4) {
            double s = AT(A, r, j + 1, lda) * x[(size_t)(j + 1) * incx];
            s = fma(AT(A, r, j, lda), x[(size_t)j * incx], s);
            s = fma(AT(A, r, j + 2, lda), x[(size_t)(j + 2) * incx], s);
            s = fma(AT(A, r, j + 3, lda), x[(size_t)(j + 3) * incx], s);
            y[r] = fma(1.0, s, y[r]);
        }
        if (incx == 1 && (n & 2)) {
            double s = AT(A, r, j + 1, lda) * x[j + 1];
            s = fma(AT(A, r, j, lda), x[j], s);
            y[r] = fma(1.0, s, y[r]);
            j += 2;
        }
        for (; j < n; ++j) y[r] = y[r] + AT(A, r, j, lda) * (x[(size_t)j * incx] * 1.0);
    }
    for (int r = m1; r < m; ++r) {
        double t = 0.0;
        for (int j = 0; j < n; ++j) t = fma(AT(A, r, j, lda), x[(size_t)j * incx], t);
        y[r] = fma(1.0, t, y[r]);
    }
}

/* A += alpha x y^T: dger_k -> daxpy per column with da = alpha*y[j]: a = fma(da, x, a) */
static void ger(int m, int n, double alpha, const double *x, int incx, const double *y, int incy, double *A, int lda)
{
    if (m <= 0 || n <= 0 || alpha == 0.0) return;
    for (int j = 0; j < n; ++j) {
        const double t = alpha * y[(size_t)j * incy];
        for (int i = 0; i < m; ++i) AT(A, i, j, lda) = fma(t, x[(size_t)i * incx], AT(A, i, j, lda));
    }
}

/* drot (SkylakeX): x' = fma(c, x, s*y), y' = fma(c, y, -(s*x)) */
static void drot(int n, double *x, int incx, double *y, int incy, double c, double s)
{
    for (int i = 0; i < n; ++i) {
        const double xi = x[(size_t)i * incx], yi = y[(size_t)i * incy];
        x[(size_t)i * incx] = fma(c, xi, s * yi);
        y[(size_t)i * incy] = fma(c, yi, -(s * xi));
    }
}

static void dswap(int n, double *x, int incx, double *y, int incy)
{
    for (int i = 0; i < n; ++i) {
        const double t = x[(size_t)i * incx];
        x[(size_t)i * incx] = y[(size_t)i * incy];
        y[(size_t)i * incy] = t;
    }
}

/* ------------------------------------------------------------------------ */
/* LAPACK 3.12.0 (plain IEEE double, no FMA)                                 */
/* ------------------------------------------------------------------------ */

static double fsign(double a, double b) { return signbit(b) ? -fabs(a) : fabs(a); } /* Fortran SIGN */

/* dlapy2: sqrt(x^2 + y^2) avoiding overflow */
static double dlapy2(double x, double y)
{
    const double xa = fabs(x), ya = fabs(y);
    const double w = xa > ya ? xa : ya, z = xa < ya ? xa : ya;
    if (z == 0.0 || w > LP_HUGE) return w;
    const double q = z / w;
    return w * sqrt(1.0 + q * q);
}

/* dlarfg(n, alpha, x, incx, tau) */
static void dlarfg(int n, double *alpha, double *x, int incx, double *tau)
{
    if (n <= 1) { *tau = 0.0; return; }
    double xnorm = orc_lp_dnrm2(n - 1, x, incx);
    if (xnorm == 0.0) { *tau = 0.0; return; }
    double beta = -fsign(dlapy2(*alpha, xnorm), *alpha);
    const double safmin = LP_SAFMIN / LP_EPS, rsafmn = 1.0 / safmin;
    int knt = 0;
    if (fabs(beta) < safmin) {
        do {
            ++knt;
            for (int i = 0; i < n - 1; ++i) x[(size_t)i * incx] *= rsafmn;
            beta *= rsafmn;
            *alpha *= rsafmn;
        } while (fabs(beta) < safmin && knt < 20);
        xnorm = orc_lp_dnrm2(n - 1, x, incx);
        beta = -fsign(dlapy2(*alpha, xnorm), *alpha);
    }
    *tau = (beta - *alpha) / beta;
    const double sc = 1.0 / (*alpha - beta);
    for (int i = 0; i < n - 1; ++i) x[(size_t)i * incx] *= sc; /* dscal */
    for (int j = 0; j < knt; ++j) beta *= safmin;
    *alpha = beta;
}

static int iladlc(int m, int n, const double *A, int lda)
{
    if (n == 0) return 0;
    if (AT(A, 0, n - 1, lda) != 0.0 || AT(A, m - 1, n - 1, lda) != 0.0) return n;
    for (int j = n; j >= 1; --j)
        for (int i = 0; i < m; ++i)
            if (AT(A, i, j - 1, lda) != 0.0) return j;
    return 0;
}

static int iladlr(int m, int n, const double *A, int lda)
{
    if (m == 0) return 0;
    if (AT(A, m - 1, 0, lda) != 0.0 || AT(A, m - 1, n - 1, lda) != 0.0) return m;
    int r = 0;
    for (int j = 0; j < n; ++j) {
        int i = m;
        while (i >= 1 && AT(A, (i > 1 ? i : 1) - 1, j, lda) == 0.0) --i;
        if (i > r) r = i;
    }
    return r;
}

/* dlarf(side, m, n, v, incv, tau, C, ldc): H = I - tau v v^T applied from the left
 * (left != 0) or the right, with the 3.12.0 trailing-zero trimming of v and C. */
static void dlarf(int left, int m, int n, const double *v, int incv, double tau, double *C, int ldc)
{
    double work[LP_MAXN];
    int lastv = 0, lastc = 0;
    if (tau != 0.0) {
        lastv = left ? m : n;
        int i = incv > 0 ? (lastv - 1) * incv : 0;
        while (lastv > 0 && v[i] == 0.0) { --lastv; i -= incv; }
        lastc = left ? iladlc(lastv, n, C, ldc) : iladlr(m, lastv, C, ldc);
    }
    if (lastv <= 0 || lastc <= 0) return; /* dgemv / dger return at once on a zero size */
    if (left) {
        gemv_t(lastv, lastc, C, ldc, v, incv, work);
        ger(lastv, lastc, -tau, v, incv, work, 1, C, ldc);
    } else {
        gemv_n(lastc, lastv, C, ldc, v, incv, work);
        ger(lastc, lastv, -tau, work, 1, v, incv, C, ldc);
    }
}

/* dgebd2 (m >= n): A = Q B P^T, B upper bidiagonal (d, e) */
static void dgebd2(int m, int n, double *A, int lda, double *d, double *e, double *tauq, double *taup)
{
    for (int i = 0; i < n; ++i) {
        dlarfg(m - i, &AT(A, i, i, lda), &AT(A, (i + 1 < m ? i + 1 : m - 1), i, lda), 1, &tauq[i]);
        d[i] = AT(A, i, i, lda);
        AT(A, i, i, lda) = 1.0;
        if (i < n - 1) dlarf(1, m - i, n - i - 1, &AT(A, i, i, lda), 1, tauq[i], &AT(A, i, i + 1, lda), lda);
        AT(A, i, i, lda) = d[i];
        if (i < n - 1) {
            dlarfg(n - i - 1, &AT(A, i, i + 1, lda), &AT(A, i, (i + 2 < n ? i + 2 : n - 1), lda), lda, &taup[i]);
            e[i] = AT(A, i, i + 1, lda);
            AT(A, i, i + 1, lda) = 1.0;
            dlarf(0, m - i - 1, n - i - 1, &AT(A, i, i + 1, lda), lda, taup[i], &AT(A, i + 1, i + 1, lda), lda);
            AT(A, i, i + 1, lda) = e[i];
        } else {
            taup[i] = 0.0;
        }
    }
}

/* dlartg (LAPACK 3.10+, la_xlartg.f90) */
static void dlartg(double f, double g, double *c, double *s, double *r)
{
    const double safmin = LP_SAFMIN, safmax = 1.0 / LP_SAFMIN;
    const double rtmin = sqrt(safmin), rtmax = sqrt(safmax / 2);
    const double f1 = fabs(f), g1 = fabs(g);
    if (g == 0.0) {
        *c = 1.0; *s = 0.0; *r = f;
    } else if (f == 0.0) {
        *c = 0.0; *s = fsign(1.0, g); *r = g1;
    } else if (f1 > rtmin && f1 < rtmax && g1 > rtmin && g1 < rtmax) {
        const double d = sqrt(f * f + g * g);
        *c = f1 / d;
        *r = fsign(d, f);
        *s = g / *r;
    } else {
        double u = f1 > g1 ? f1 : g1;
        if (safmin > u) u = safmin;
        if (u > safmax) u = safmax;
        const double fs = f / u, gs = g / u;
        const double d = sqrt(fs * fs + gs * gs);
        *c = fabs(fs) / d;
        *r = fsign(d, f);
        *s = gs / *r;
        *r = *r * u;
    }
}

/* dlas2: singular values of [[f, g], [0, h]] */
static void dlas2(double f, double g, double h, double *ssmin, double *ssmax)
{
    const double fa = fabs(f), ga = fabs(g), ha = fabs(h);
    const double fhmn = fa < ha ? fa : ha, fhmx = fa > ha ? fa : ha;
    if (fhmn == 0.0) {
        *ssmin = 0.0;
        if (fhmx == 0.0) {
            *ssmax = ga;
        } else {
            const double mx = fhmx > ga ? fhmx : ga, mn = fhmx < ga ? fhmx : ga;
            const double q = mn / mx;
            *ssmax = mx * sqrt(1.0 + q * q);
        }
    } else if (ga < fhmx) {
        const double as = 1.0 + fhmn / fhmx, at = (fhmx - fhmn) / fhmx;
        const double au0 = ga / fhmx, au = au0 * au0;
        const double c = 2.0 / (sqrt(as * as + au) + sqrt(at * at + au));
        *ssmin = fhmn * c;
        *ssmax = fhmx / c;
    } else {
        const double au = fhmx / ga;
        if (au == 0.0) {
            *ssmin = (fhmn * fhmx) / ga;
            *ssmax = ga;
        } else {
            const double as = 1.0 + fhmn / fhmx, at = (fhmx - fhmn) / fhmx;
            const double p = as * au, q = at * au;
            const double c = 1.0 / (sqrt(1.0 + p * p) + sqrt(1.0 + q * q));
            double mn = (fhmn * c) * au;
            *ssmin = mn + mn;
            *ssmax = ga / (c + c);
        }
    }
}

/* dlasv2: SVD of [[f, g], [0, h]] with rotations */
static void dlasv2(double f, double g, double h, double *ssmin, double *ssmax, double *snr, double *csr, double *snl,
                   double *csl)
{
    double ft = f, fa = fabs(ft), ht = h, ha = fabs(h);
    int pmax = 1;
    const int swap = ha > fa;
    if (swap) {
        pmax = 3;
        double t = ft; ft = ht; ht = t;
        t = fa; fa = ha; ha = t;
    }
    const double gt = g, ga = fabs(gt);
    double clt, crt, slt, srt;
    if (ga == 0.0) {
        *ssmin = ha; *ssmax = fa;
        clt = 1.0; crt = 1.0; slt = 0.0; srt = 0.0;
    } else {
        int gasmal = 1;
        if (ga > fa) {
            pmax = 2;
            if (fa / ga < LP_EPS) {
                gasmal = 0;
                *ssmax = ga;
                if (ha > 1.0) *ssmin = fa / (ga / ha);
                else *ssmin = (fa / ga) * ha;
                clt = 1.0;
                slt = ht / gt;
                srt = 1.0;
                crt = ft / gt;
            }
        }
        if (gasmal) {
            const double dd = fa - ha;
            double l = (dd == fa) ? 1.0 : dd / fa;
            const double mm0 = gt / ft;
            double t = 2.0 - l;
            const double mm = mm0 * mm0, tt = t * t;
            const double s = sqrt(tt + mm);
            const double r = (l == 0.0) ? fabs(mm0) : sqrt(l * l + mm);
            const double a = 0.5 * (s + r);
            *ssmin = ha / a;
            *ssmax = fa * a;
            if (mm == 0.0) {
                if (l == 0.0) t = fsign(2.0, ft) * fsign(1.0, gt);
                else t = gt / fsign(dd, ft) + mm0 / t;
            } else {
                t = (mm0 / (s + t) + mm0 / (r + l)) * (1.0 + a);
            }
            l = sqrt(t * t + 4.0);
            crt = 2.0 / l;
            srt = t / l;
            clt = (crt + srt * mm0) / a;
            slt = ((ht / ft) * srt) / a;
        }
    }
    if (swap) { *csl = srt; *snl = crt; *csr = slt; *snr = clt; }
    else { *csl = clt; *snl = slt; *csr = crt; *snr = srt; }
    double tsign = 1.0;
    if (pmax == 1) tsign = fsign(1.0, *csr) * fsign(1.0, *csl) * fsign(1.0, f);
    if (pmax == 2) tsign = fsign(1.0, *snr) * fsign(1.0, *csl) * fsign(1.0, g);
    if (pmax == 3) tsign = fsign(1.0, *snr) * fsign(1.0, *snl) * fsign(1.0, h);
    *ssmax = fsign(*ssmax, tsign);
    *ssmin = fsign(*ssmin, tsign * fsign(1.0, f) * fsign(1.0, h));
}

/* dlasr with PIVOT = 'V'.  left: A := P A (rows j, j+1 rotated), else A := A P^T
 * (columns).  fwd: j = 0..k-2, else backwards.  A is m x n. */
static void dlasr(int left, int fwd, int m, int n, const double *c, const double *s, double *A, int lda)
{
    const int k = left ? m : n;
    for (int q = 0; q < k - 1; ++q) {
        const int j = fwd ? q : k - 2 - q;
        const double ct = c[j], st = s[j];
        if (ct == 1.0 && st == 0.0) continue;
        if (left) {
            for (int i = 0; i < n; ++i) {
                const double t = AT(A, j + 1, i, lda);
                AT(A, j + 1, i, lda) = ct * t - st * AT(A, j, i, lda);
                AT(A, j, i, lda) = st * t + ct * AT(A, j, i, lda);
            }
        } else {
            for (int i = 0; i < m; ++i) {
                const double t = AT(A, i, j + 1, lda);
                AT(A, i, j + 1, lda) = ct * t - st * AT(A, i, j, lda);
                AT(A, i, j, lda) = st * t + ct * AT(A, i, j, lda);
            }
        }
    }
}

static double lp_tolmul(void)
{
    /* TOLMUL = MAX(10, MIN(100, EPS**MEIGTH)), MEIGTH = -0.125 (gfortran: pow) */
    double t = pow(LP_EPS, -0.125);
    if (t > 100.0) t = 100.0;
    if (t < 10.0) t = 10.0;
    return t;
}

/* dbdsqr('U', n, ncvt = n, nru = n, ncc = 0): implicit zero-shift / shifted QR on the
 * upper bidiagonal (d, e), rotations applied to VT (n x n, rows) and U (n x n, cols).
 * Returns info (0 = converged). */
static int dbdsqr(int n, double *d, double *e, double *VT, int ldvt, double *U, int ldu)
{
    const int maxitr = 6;
    if (n == 0) return 0;
    if (n > 1) {
        const int nm1 = n - 1, nm12 = nm1 + nm1, nm13 = nm12 + nm1;
        double work[4 * LP_MAXN];
        const double eps = LP_EPS, unfl = LP_SAFMIN;
        const double tol = lp_tolmul() * eps;
        double smax = 0.0;
        for (int i = 0; i < n; ++i) smax = fmax(smax, fabs(d[i]));
        for (int i = 0; i < n - 1; ++i) smax = fmax(smax, fabs(e[i]));
        double sminoa = 0.0, thresh;
        /* relative accuracy (tol >= 0) */
        sminoa = fabs(d[0]);
        if (sminoa != 0.0) {
            double mu = sminoa;
            for (int i = 1; i < n; ++i) {
                mu = fabs(d[i]) * (mu / (mu + fabs(e[i - 1])));
                sminoa = fmin(sminoa, mu);
                if (sminoa == 0.0) break;
            }
        }
        sminoa = sminoa / sqrt((double)n);
        {
            const double a = tol * sminoa, b = (double)maxitr * ((double)n * ((double)n * unfl));
            thresh = a > b ? a : b;
        }
        const int maxitdivn = maxitr * n;
        int iterdivn = 0, iter = -1, oldll = -1, oldm = -1, idir = 0;
        int m = n; /* 1-based index of the last element of the unconverged part */
        /* 1-based accessors */
#define D_(i) d[(i) - 1]
#define E_(i) e[(i) - 1]
#define W_(i) work[(i) - 1]
        for (;;) {
            if (m <= 1) break;
            if (iter >= n) {
                iter -= n;
                ++iterdivn;
                if (iterdivn >= maxitdivn) return 1; /* not converged */
            }
            /* find diagonal block of matrix to work on */
            double smin = 0.0;
            smax = fabs(D_(m));
            int ll = 0, split = 0;
            for (int lll = 1; lll <= m - 1; ++lll) {
                ll = m - lll;
                const double abss = fabs(D_(ll)), abse = fabs(E_(ll));
                if (abse <= thresh) { split = 1; break; }
                smax = fmax(smax, fmax(abss, abse));
            }
            if (split) {
                E_(ll) = 0.0;
                if (ll == m - 1) { m = m - 1; continue; }
            } else {
                ll = 0;
            }
            ll = ll + 1;
            if (ll == m - 1) {
                /* 2 by 2 block */
                double sigmn, sigmx, sinr, cosr, sinl, cosl;
                dlasv2(D_(m - 1), E_(m - 1), D_(m), &sigmn, &sigmx, &sinr, &cosr, &sinl, &cosl);
                D_(m - 1) = sigmx;
                E_(m - 1) = 0.0;
                D_(m) = sigmn;
                drot(n, &AT(VT, m - 2, 0, ldvt), ldvt, &AT(VT, m - 1, 0, ldvt), ldvt, cosr, sinr);
                drot(n, &AT(U, 0, m - 2, ldu), 1, &AT(U, 0, m - 1, ldu), 1, cosl, sinl);
                m = m - 2;
                continue;
            }
            /* new submatrix: choose shift direction */
            if (ll > oldm || m < oldll) {
                if (fabs(D_(ll)) >= fabs(D_(m))) idir = 1;
                else idir = 2;
            }
            /* convergence tests */
            int conv = 0;
            if (idir == 1) {
                if (fabs(E_(m - 1)) <= fabs(tol) * fabs(D_(m))) { E_(m - 1) = 0.0; continue; }
                double mu = fabs(D_(ll));
                smin = mu;
                for (int lll = ll; lll <= m - 1; ++lll) {
                    if (fabs(E_(lll)) <= tol * mu) { E_(lll) = 0.0; conv = 1; break; }
                    mu = fabs(D_(lll + 1)) * (mu / (mu + fabs(E_(lll))));
                    smin = fmin(smin, mu);
                }
            } else {
                if (fabs(E_(ll)) <= fabs(tol) * fabs(D_(ll))) { E_(ll) = 0.0; continue; }
                double mu = fabs(D_(m));
                smin = mu;
                for (int lll = m - 1; lll >= ll; --lll) {
                    if (fabs(E_(lll)) <= tol * mu) { E_(lll) = 0.0; conv = 1; break; }
                    mu = fabs(D_(lll)) * (mu / (mu + fabs(E_(lll))));
                    smin = fmin(smin, mu);
                }
            }
            if (conv) continue;
            oldll = ll;
            oldm = m;
            /* shift */
            double shift, r;
            {
                const double lhs = (double)n * tol * (smin / smax);
                const double rhs = eps > 0.01 * tol ? eps : 0.01 * tol;
                if (lhs <= rhs) {
                    shift = 0.0;
                } else {
                    double sll;
                    if (idir == 1) { sll = fabs(D_(ll)); dlas2(D_(m - 1), E_(m - 1), D_(m), &shift, &r); }
                    else { sll = fabs(D_(m)); dlas2(D_(ll), E_(ll), D_(ll + 1), &shift, &r); }
                    if (sll > 0.0) {
                        const double q = shift / sll;
                        if (q * q < eps) shift = 0.0;
                    }
                }
            }
            iter = iter + m - ll;
            if (shift == 0.0) {
                if (idir == 1) {
                    double cs = 1.0, oldcs = 1.0, sn = 0.0, oldsn = 0.0;
                    for (int i = ll; i <= m - 1; ++i) {
                        dlartg(D_(i) * cs, E_(i), &cs, &sn, &r);
                        if (i > ll) E_(i - 1) = oldsn * r;
                        dlartg(oldcs * r, D_(i + 1) * sn, &oldcs, &oldsn, &D_(i));
                        W_(i - ll + 1) = cs;
                        W_(i - ll + 1 + nm1) = sn;
                        W_(i - ll + 1 + nm12) = oldcs;
                        W_(i - ll + 1 + nm13) = oldsn;
                    }
                    const double h = D_(m) * cs;
                    D_(m) = h * oldcs;
                    E_(m - 1) = h * oldsn;
                    dlasr(1, 1, m - ll + 1, n, &W_(1), &W_(n), &AT(VT, ll - 1, 0, ldvt), ldvt);
                    dlasr(0, 1, n, m - ll + 1, &W_(nm12 + 1), &W_(nm13 + 1), &AT(U, 0, ll - 1, ldu), ldu);
                    if (fabs(E_(m - 1)) <= thresh) E_(m - 1) = 0.0;
                } else {
                    double cs = 1.0, oldcs = 1.0, sn = 0.0, oldsn = 0.0;
                    for (int i = m; i >= ll + 1; --i) {
                        dlartg(D_(i) * cs, E_(i - 1), &cs, &sn, &r);
                        if (i < m) E_(i) = oldsn * r;
                        dlartg(oldcs * r, D_(i - 1) * sn, &oldcs, &oldsn, &D_(i));
                        W_(i - ll) = cs;
                        W_(i - ll + nm1) = -sn;
                        W_(i - ll + nm12) = oldcs;
                        W_(i - ll + nm13) = -oldsn;
                    }
                    const double h = D_(ll) * cs;
                    D_(ll) = h * oldcs;
                    E_(ll) = h * oldsn;
                    dlasr(1, 0, m - ll + 1, n, &W_(nm12 + 1), &W_(nm13 + 1), &AT(VT, ll - 1, 0, ldvt), ldvt);
                    dlasr(0, 0, n, m - ll + 1, &W_(1), &W_(n), &AT(U, 0, ll - 1, ldu), ldu);
                    if (fabs(E_(ll)) <= thresh) E_(ll) = 0.0;
                }
            } else {
                if (idir == 1) {
                    double f = (fabs(D_(ll)) - shift) * (fsign(1.0, D_(ll)) + shift / D_(ll));
                    double g = E_(ll);
                    double cosr, sinr, cosl, sinl;
                    for (int i = ll; i <= m - 1; ++i) {
                        dlartg(f, g, &cosr, &sinr, &r);
                        if (i > ll) E_(i - 1) = r;
                        f = cosr * D_(i) + sinr * E_(i);
                        E_(i) = cosr * E_(i) - sinr * D_(i);
                        g = sinr * D_(i + 1);
                        D_(i + 1) = cosr * D_(i + 1);
                        dlartg(f, g, &cosl, &sinl, &r);
                        D_(i) = r;
                        f = cosl * E_(i) + sinl * D_(i + 1);
                        D_(i + 1) = cosl * D_(i + 1) - sinl * E_(i);
                        if (i < m - 1) {
                            g = sinl * E_(i + 1);
                            E_(i + 1) = cosl * E_(i + 1);
                        }
                        W_(i - ll + 1) = cosr;
                        W_(i - ll + 1 + nm1) = sinr;
                        W_(i - ll + 1 + nm12) = cosl;
                        W_(i - ll + 1 + nm13) = sinl;
                    }
                    E_(m - 1) = f;
                    dlasr(1, 1, m - ll + 1, n, &W_(1), &W_(n), &AT(VT, ll - 1, 0, ldvt), ldvt);
                    dlasr(0, 1, n, m - ll + 1, &W_(nm12 + 1), &W_(nm13 + 1), &AT(U, 0, ll - 1, ldu), ldu);
                    if (fabs(E_(m - 1)) <= thresh) E_(m - 1) = 0.0;
                } else {
                    double f = (fabs(D_(m)) - shift) * (fsign(1.0, D_(m)) + shift / D_(m));
                    double g = E_(m - 1);
                    double cosr, sinr, cosl, sinl;
                    for (int i = m; i >= ll + 1; --i) {
                        dlartg(f, g, &cosr, &sinr, &r);
                        if (i < m) E_(i) = r;
                        f = cosr * D_(i) + sinr * E_(i - 1);
                        E_(i - 1) = cosr * E_(i - 1) - sinr * D_(i);
                        g = sinr * D_(i - 1);
                        D_(i - 1) = cosr * D_(i - 1);
                        dlartg(f, g, &cosl, &sinl, &r);
                        D_(i) = r;
                        f = cosl * E_(i - 1) + sinl * D_(i - 1);
                        D_(i - 1) = cosl * D_(i - 1) - sinl * E_(i - 1);
                        if (i > ll + 1) {
                            g = sinl * E_(i - 2);
                            E_(i - 2) = cosl * E_(i - 2);
                        }
                        W_(i - ll) = cosr;
                        W_(i - ll + nm1) = -sinr;
                        W_(i - ll + nm12) = cosl;
                        W_(i - ll + nm13) = -sinl;
                    }
                    E_(ll) = f;
                    if (fabs(E_(ll)) <= thresh) E_(ll) = 0.0;
                    dlasr(1, 0, m - ll + 1, n, &W_(nm12 + 1), &W_(nm13 + 1), &AT(VT, ll - 1, 0, ldvt), ldvt);
                    dlasr(0, 0, n, m - ll + 1, &W_(1), &W_(n), &AT(U, 0, ll - 1, ldu), ldu);
                }
            }
        }
#undef D_
#undef E_
#undef W_
    }
    /* make singular values positive */
    for (int i = 0; i < n; ++i)
        if (d[i] < 0.0) {
            d[i] = -d[i];
            for (int j = 0; j < n; ++j) AT(VT, i, j, ldvt) *= -1.0; /* dscal(ncvt, -1) */
        }
    /* sort into decreasing order (selection sort, one swap per position; .LE. keeps the last of a tie) */
    for (int i = 1; i <= n - 1; ++i) {
        int isub = 1;
        double smin = d[0];
        for (int j = 2; j <= n + 1 - i; ++j)
            if (d[j - 1] <= smin) { isub = j; smin = d[j - 1]; }
        if (isub != n + 1 - i) {
            d[isub - 1] = d[n - i];
            d[n - i] = smin;
            dswap(n, &AT(VT, isub - 1, 0, ldvt), ldvt, &AT(VT, n - i, 0, ldvt), ldvt);
            dswap(n, &AT(U, 0, isub - 1, ldu), 1, &AT(U, 0, n - i, ldu), 1);
        }
    }
    return 0;
}

/* dbdsdc('U', 'I', n, ...) for n <= SMLSIZ (25): U = VT = I, dlasdq('U', sqre 0)
 * -> dbdsqr (descending), then dlasdq's selection sort into ASCENDING order
 * (strict .LT.), then dbdsdc's selection sort back into descending order (strict
 * .GT.).  Both sorts only swap; they matter for exact ties (zero blocks, rank-
 * deficient blocks), where they fix which singular vector comes first. */
int orc_lp_dbdsdc(int n, double *d, double *e, double *U, int ldu, double *VT, int ldvt)
{
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < n; ++i) { AT(U, i, j, ldu) = (i == j); AT(VT, i, j, ldvt) = (i == j); }
    if (n == 1) {
        AT(U, 0, 0, ldu) = fsign(1.0, d[0]);
        AT(VT, 0, 0, ldvt) = 1.0;
        d[0] = fabs(d[0]);
        return 0;
    }
    const int info = dbdsqr(n, d, e, VT, ldvt, U, ldu);
    /* dlasdq: ascending */
    for (int i = 0; i < n; ++i) {
        int isub = i;
        double smin = d[i];
        for (int j = i + 1; j < n; ++j)
            if (d[j] < smin) { isub = j; smin = d[j]; }
        if (isub != i) {
            d[isub] = d[i];
            d[i] = smin;
            dswap(n, &AT(VT, isub, 0, ldvt), ldvt, &AT(VT, i, 0, ldvt), ldvt);
            dswap(n, &AT(U, 0, isub, ldu), 1, &AT(U, 0, i, ldu), 1);
        }
    }
    /* dbdsdc: descending */
    for (int i = 0; i < n - 1; ++i) {
        int kk = i;
        double p = d[i];
        for (int j = i + 1; j < n; ++j)
            if (d[j] > p) { kk = j; p = d[j]; }
        if (kk != i) {
            d[kk] = d[i];
            d[i] = p;
            dswap(n, &AT(U, 0, i, ldu), 1, &AT(U, 0, kk, ldu), 1);
            dswap(n, &AT(VT, i, 0, ldvt), ldvt, &AT(VT, kk, 0, ldvt), ldvt);
        }
    }
    return info;
}

int orc_lp_dbdsqr(int n, double *d, double *e, double *VT, int ldvt, double *U, int ldu)
{
    return dbdsqr(n, d, e, VT, ldvt, U, ldu);
}

void orc_lp_dgebd2(int m, int n, double *A, int lda, double *d, double *e, double *tauq, double *taup)
{
    dgebd2(m, n, A, lda, d, e, tauq, taup);
}

/* dormbr('Q','L','N', n, n, n, A, tauq, U): dorm2r left, no transpose -> i = k..1 */
void orc_lp_apply_q(int n, const double *A, int lda, const double *tauq, double *U, int ldu)
{
    double Ac[LP_MAXN * LP_MAXN];
    for (int j = 0; j < n; ++j) for (int i = 0; i < n; ++i) Ac[i + j * n] = AT(A, i, j, lda);
    for (int i = n - 1; i >= 0; --i) {
        const double aii = Ac[i + i * n];
        Ac[i + i * n] = 1.0;
        dlarf(1, n - i, n, &Ac[i + i * n], 1, tauq[i], &AT(U, i, 0, ldu), ldu);
        Ac[i + i * n] = aii;
    }
}

/* dormbr('P','R','T', n, n, n, A, taup, VT): nq = n = k, so dormlq('R', 'N', n, n-1,
 * n-1, A(1,2), taup, VT(1,2)) -> dorml2 right, no transpose -> i = k..1 */
void orc_lp_apply_pt(int n, const double *A, int lda, const double *taup, double *VT, int ldvt)
{
    if (n <= 1) return;
    double Ac[LP_MAXN * LP_MAXN];
    for (int j = 0; j < n; ++j) for (int i = 0; i < n; ++i) Ac[i + j * n] = AT(A, i, j, lda);
    double *A2 = Ac + n; /* A(1,2) */
    double *C2 = VT + (size_t)ldvt; /* VT(1,2) */
    const int k = n - 1, nn = n - 1;
    for (int i = k - 1; i >= 0; --i) {
        const double aii = A2[i + (size_t)i * n];
        A2[i + (size_t)i * n] = 1.0;
        dlarf(0, n, nn - i, &A2[i + (size_t)i * n], n, taup[i], C2 + (size_t)i * ldvt, ldvt);
        A2[i + (size_t)i * n] = aii;
    }
}

/* np.linalg.svd(a) for an n x n f64 matrix a (row-major, as numpy holds it):
 * u (row-major, u[i][k]), s (descending), vt (row-major, vt[k][j]).
 * dgesdd JOBZ='A', path 5.  Returns dbdsqr's info (0 = converged). */
int orc_lp_svd(const double *a, int n, double *u, double *s, double *vt)
{
    double A[LP_MAXN * LP_MAXN], U[LP_MAXN * LP_MAXN], VT[LP_MAXN * LP_MAXN];
    double e[LP_MAXN], tauq[LP_MAXN], taup[LP_MAXN];
    if (n <= 0 || n > LP_MAXN) return -1;
    for (int i = 0; i < n; ++i) for (int j = 0; j < n; ++j) A[i + j * n] = a[i * n + j];
    /* dgesdd: anrm = dlange('M'); scale only if anrm is outside [smlnum, bignum] */
    double anrm = 0.0;
    for (int k = 0; k < n * n; ++k) { const double v = fabs(A[k]); if (v > anrm || isnan(v)) anrm = v; }
    if (isnan(anrm)) return -4;
    const double smlnum = sqrt(LP_SAFMIN) / LP_PREC, bignum = 1.0 / smlnum;
    if ((anrm > 0.0 && anrm < smlnum) || anrm > bignum) return -2; /* dlascl path: not restated (never hit by image data) */
    dgebd2(n, n, A, n, s, e, tauq, taup);
    int info = orc_lp_dbdsdc(n, s, e, U, n, VT, n);
    orc_lp_apply_q(n, A, n, tauq, U, n);
    orc_lp_apply_pt(n, A, n, taup, VT, n);
    for (int i = 0; i < n; ++i)
        for (int k = 0; k < n; ++k) { u[i * n + k] = U[i + k * n]; vt[i * n + k] = VT[i + k * n]; }
    return info;
}

/* f32 block -> f32 U, S, Vt exactly as numpy returns them for a float32 input
 * (f64 computation, results cast back with astype(float32)). */
int orc_lp_svd_block_f32(const float *D, int n, float *U, float *S, float *Vt)
{
    double a[LP_MAXN * LP_MAXN], u[LP_MAXN * LP_MAXN], s[LP_MAXN], vt[LP_MAXN * LP_MAXN];
    if (n <= 0 || n > LP_MAXN) return -1;
    for (int k = 0; k < n * n; ++k) a[k] = D[k];
    const int info = orc_lp_svd(a, n, u, s, vt);
    for (int k = 0; k < n * n; ++k) { U[k] = (float)u[k]; Vt[k] = (float)vt[k]; }
    for (int k = 0; k < n; ++k) S[k] = (float)s[k];
    return info;
}

int orc_lp_svd_blocks(const float *D, int64_t nb, int b, float *U, float *S, float *Vt, int nthreads)
{
    int bad = 0;
    if (nthreads < 1) nthreads = 1;
#pragma omp parallel for num_threads(nthreads) schedule(static) reduction(| : bad)
    for (int64_t k = 0; k < nb; ++k)
        bad |= orc_lp_svd_block_f32(D + k * b * b, b, U + k * b * b, S + k * b, Vt + k * b * b) != 0;
    return bad;
}

/* f64 results of the dgesdd route for f32 blocks: u[r][k], s[k], vt[k][j] */
int orc_lp_svd_blocks_f64(const float *D, int64_t nb, int b, double *U, double *S, double *Vt, int nthreads)
{
    int bad = 0;
    if (nthreads < 1) nthreads = 1;
#pragma omp parallel for num_threads(nthreads) schedule(static) reduction(| : bad)
    for (int64_t k = 0; k < nb; ++k) {
        double a[LP_MAXN * LP_MAXN];
        for (int q = 0; q < b * b; ++q) a[q] = D[k * b * b + q];
        bad |= orc_lp_svd(a, b, U + k * b * b, S + k * b, Vt + k * b * b) != 0;
    }
    return bad;
}
