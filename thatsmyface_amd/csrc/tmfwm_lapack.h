// The reference's SVD route on the GPU: np.linalg.svd of a float32 block
// (watermarking.py:195, :279-282) = numpy 2.2.6 -> f64 LAPACK dgesdd (JOBZ='A') from
// scipy-openblas64 0.3.29, i.e. LAPACK 3.12.0 compiled without FMA around the OpenBLAS
// "SkylakeX" BLAS kernels.  Restated operation by operation (oracle/tmfwm_lapack.c is the
// CPU restatement this matches bit for bit):
//
//   dgebd2 (dlarfg + dlarf with iladlc/iladlr trimming) -> dbdsqr (dlartg, dlas2,
//   dlasv2, dlasr, drot) -> dlasdq / dbdsdc selection sorts -> dorm2r / dorml2
//
// BLAS kernels with their exact operation order: dgemv_t (4-lane fma / 2- and 4-lane
// mul+add column kernels, contracted row tail), dgemv_n (4- and 2-column fma kernels,
// mul+add single columns, fma row tail), dger (fma(alpha*y, x, a)), drot (fma pairs) and
// dnrm2 -- OpenBLAS's x87 nrm2.S: squares and sums rounded to a 64-bit mantissa, four
// accumulators, fsqrt, then a second rounding to double -- emulated here in integer
// arithmetic (X80).
//
// Every routine is written over a lane policy P (below): SerialPar runs it on one thread
// (the host build of the CPU tests); WavePar runs one block per 64-lane wave (the fixup
// kernels and the stage entry point).  Under WavePar the scalar parts (dnrm2, dlartg,
// dlasv2, the dbdsqr recurrences, the scans) run uniformly on every lane, and the loops
// over matrix elements -- dgemv columns / rows, dger and the scalings' elements, drot /
// dlasr / dswap positions -- are spread over the lanes (LP_PAR): each element gets the
// same operations in the same order as on one thread, so the bits do not depend on the
// policy.  A loop body touches only its own element(s); P::sync() (a workgroup barrier:
// the workgroup is the one wave) orders a loop's stores before other lanes' loads.
// The fused kernels take this route only for the blocks the conditioning test sends to
// it (embed) or whose sigma_1 enclosure does not decide the f32 value (extract).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tmf {
namespace lp {

// host + device: the CPU test suite compiles this same code for the host
// (tests/native/lp_host.cpp) and checks it against the oracle before any GPU run
// Every routine is inlined: on the GPU a call saves and restores callee-saved registers
// through scratch (global memory), and the route makes hundreds of calls per block -- as
// noinline functions they cost ~1 ms per block (profiles/r03/r03d_*); the working arrays
// are in the caller's LDS workspace, so inlining adds no private memory.
#define TMF_LPI __host__ __device__ inline __attribute__((always_inline))
#define TMF_LPN TMF_LPI

constexpr int kMaxN = 16;
constexpr double kEps = 0x1p-53;                     // dlamch('E')
constexpr double kPrec = 0x1p-52;                    // dlamch('P')
constexpr double kSafmin = 0x1p-1022;                // dlamch('S')
constexpr double kHuge = 0x1.fffffffffffffp+1023;    // dlamch('O')
constexpr double kTolmul = 0x1.8ace5422aa0dbp+6;     // max(10, min(100, eps**-0.125)) (glibc pow, pinned by a CPU test)
constexpr double kRtmax = 0x1.6a09e667f3bcdp+510;    // sqrt(safmax / 2) in dlartg
constexpr double kRtmin = 0x1p-511;                  // sqrt(safmin)

// ---------------------------------------------------------------------------
// lane policies
// ---------------------------------------------------------------------------
struct SerialPar {
    TMF_LPI static int lane() { return 0; }
    static constexpr int kLanes = 1;
    TMF_LPI static void sync() {}
};
// the same loops run backwards (host tests: element bodies must not depend on the order)
struct ReversePar {
    static constexpr int kLanes = 1;
    static constexpr bool kReverse = true;
    TMF_LPI static void sync() {}
};
struct WavePar {  // device code only
    __device__ __forceinline__ static int lane() { return (int)(threadIdx.x & 63u); }
    static constexpr int kLanes = 64;
    __device__ __forceinline__ static void sync() { __syncthreads(); }  // workgroup == one wave
};
// G lanes per block, 64 / G blocks per wave (device code only): every group of G consecutive
// lanes runs the route for its own block, the element loops over the group's lanes and the
// scalar recurrences on each group's lanes alike, so the groups of a wave diverge only where
// their blocks' data do (dbdsqr's iteration counts, splits and shifts).  A group's lanes see
// each other's LDS writes in program order (one wave), so sync() only fences the compiler.
template <int G>
struct GroupPar {
    static_assert(G == 8 || G == 16 || G == 32, "group size");
    __device__ __forceinline__ static int lane() { return (int)(threadIdx.x & (unsigned)(G - 1)); }
    __device__ __forceinline__ static int base() { return (int)(threadIdx.x & ~(unsigned)(G - 1) & 63u); }
    static constexpr int kLanes = G;
    __device__ __forceinline__ static void sync() { asm volatile("" ::: "memory"); }
};

template <class P, class = void>
struct IsReverse { static constexpr bool v = false; };
template <class P>
struct IsReverse<P, decltype((void)P::kReverse)> { static constexpr bool v = P::kReverse; };

// for (int K = first; K < N; K += step) over this lane's share of [0, N)
#define LP_PAR(P, K, N)                                                                                     \
    for (int K##_n = (N), K##_i = IsReverse<P>::v ? K##_n - 1 : lane_of<P>(); IsReverse<P>::v ? K##_i >= 0 : K##_i < K##_n; \
         K##_i += IsReverse<P>::v ? -1 : P::kLanes)                                                          \
        if (const int K = K##_i; true)
template <class P>
TMF_LPI int lane_of()
{
    if constexpr (IsReverse<P>::v) return 0;
    else return P::lane();
}

// A vector of <= 16 doubles that every lane reads and writes alike (dbdsqr's d, e and its
// rotation sequences): a plain array on one thread; under WavePar element i lives in lane
// i's register and is read with readlane (its index is uniform), written with a lane
// select -- the scalar recurrences then wait on register moves, not on LDS round trips.
template <class P>
struct LVec {
    double v[kMaxN];
    TMF_LPI double get(int i) const { return v[i]; }
    TMF_LPI void set(int i, double x) { v[i] = x; }
    TMF_LPI void load(const double *src, int n) { for (int i = 0; i < n; ++i) v[i] = src[i]; }
    TMF_LPI void store_f32(float *dst, int n) const { for (int i = 0; i < n; ++i) dst[i] = (float)v[i]; }
};
template <>
struct LVec<WavePar> {
    double v = 0.0;
    __device__ __forceinline__ double get(int i) const
    {
        const long long b = __builtin_bit_cast(long long, v);
        const int lo = __builtin_amdgcn_readlane((int)b, i), hi = __builtin_amdgcn_readlane((int)(b >> 32), i);
        return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
    }
    __device__ __forceinline__ void set(int i, double x) { v = WavePar::lane() == i ? x : v; }
    __device__ __forceinline__ void load(const double *src, int n) { v = WavePar::lane() < n ? src[WavePar::lane()] : 0.0; }
    __device__ __forceinline__ void store_f32(float *dst, int n) const
    {
        if (WavePar::lane() < n) dst[WavePar::lane()] = (float)v;
    }
};

// Under GroupPar<G> element i of a group's vector lives in the register of the group's lane i;
// the index is uniform within the group but the lane differs between groups, so the read is a
// ds_bpermute (per-lane source) rather than a readlane.
template <int G>
struct LVec<GroupPar<G>> {
    double v = 0.0;
    __device__ __forceinline__ double get(int i) const
    {
        const long long b = __builtin_bit_cast(long long, v);
        const int addr = (GroupPar<G>::base() + i) << 2;
        const int lo = __builtin_amdgcn_ds_bpermute(addr, (int)b), hi = __builtin_amdgcn_ds_bpermute(addr, (int)(b >> 32));
        return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
    }
    __device__ __forceinline__ void set(int i, double x) { v = GroupPar<G>::lane() == i ? x : v; }
    __device__ __forceinline__ void load(const double *src, int n)
    {
        v = GroupPar<G>::lane() < n ? src[GroupPar<G>::lane()] : 0.0;
    }
    __device__ __forceinline__ void store_f32(float *dst, int n) const
    {
        if (GroupPar<G>::lane() < n) dst[GroupPar<G>::lane()] = (float)v;
    }
};

// ---------------------------------------------------------------------------
// x87 extended arithmetic for dnrm2 (non-negative values only: squares and sums)
// value = m * 2^e, m normalised (bit 63 set) or zero.
// ---------------------------------------------------------------------------
struct X80 {
    uint64_t m;
    int e;
};
typedef unsigned __int128 u128;

TMF_LPI int clz128(u128 v)
{
    const uint64_t hi = (uint64_t)(v >> 64);
    return hi ? __builtin_clzll(hi) : 64 + __builtin_clzll((uint64_t)v);
}

// round a 128-bit magnitude (top bit at 127) to 64 bits, RNE: m * 2^(e+64)
TMF_LPI X80 round128(u128 s, int e)
{
    uint64_t m = (uint64_t)(s >> 64);
    const uint64_t rest = (uint64_t)s;
    if (rest > 0x8000000000000000ull || (rest == 0x8000000000000000ull && (m & 1))) {
        ++m;
        if (m == 0) { m = 0x8000000000000000ull; ++e; }
    }
    return {m, e + 64};
}

// x*x rounded to a 64-bit mantissa (x87 fmul of a loaded double)
TMF_LPI X80 x80_sq(double x)
{
    const uint64_t bits = __builtin_bit_cast(uint64_t, x) & 0x7fffffffffffffffull;
    if (bits == 0) return {0, 0};
    int ex = (int)(bits >> 52);
    uint64_t mant = bits & 0xfffffffffffffull;
    if (ex == 0) ex = 1; else mant |= 1ull << 52;  // x = mant * 2^(ex - 1075)
    u128 p = (u128)mant * mant;
    const int sh = clz128(p);
    p <<= sh;  // top bit at 127
    return round128(p, 2 * (ex - 1075) - sh);
}

// a + b, both >= 0, rounded to a 64-bit mantissa (x87 faddp)
TMF_LPI X80 x80_add(X80 a, X80 b)
{
    if (a.m == 0) return b;
    if (b.m == 0) return a;
    if (a.e < b.e) { const X80 t = a; a = b; b = t; }
    const int d = a.e - b.e;
    const u128 A = (u128)a.m << 64;
    u128 Bv;
    if (d >= 128) {
        Bv = 1;  // sticky
    } else {
        const u128 bb = (u128)b.m << 64;
        Bv = bb >> d;
        if (d > 0 && (bb << (128 - d)) != 0) Bv |= 1;  // bits shifted out: sticky
    }
    u128 s = A + Bv;
    int e = a.e - 64;
    if (s < A) {  // carry out of bit 127
        const uint64_t sticky = (uint64_t)s & 1;
        s = (s >> 1) | ((u128)1 << 127) | sticky;
        ++e;
    }
    return round128(s, e);
}

// (double) of the x87 fsqrt of t: sqrt rounded to 64 bits, then to 53 bits (both RNE)
TMF_LPI double x80_sqrt_to_double(X80 t)
{
    if (t.m == 0) return 0.0;
    // N = m * 2^k with k in {63, 64} so that t = N * 2^(e-k), e-k even, sqrt(N) in [2^63, 2^64)
    const int k = ((t.e & 1) == 0) ? 64 : 63;
    const u128 N = (u128)t.m << k;
    const int qe = (t.e - k) / 2;  // sqrt(t) = sqrt(N) * 2^qe
    const double nd = (double)(uint64_t)(N >> 64) * 0x1p64 + (double)(uint64_t)N;
    double rd = __builtin_sqrt(nd);
    uint64_t r = rd >= 0x1p64 ? 0xffffffffffffffffull : (uint64_t)rd;
    // one Newton correction, its step (|step| < ~2^12: rd carries 53 of the 64 bits) rounded in
    // floating point but applied in integer arithmetic -- applied as r + step in a double, the
    // sum would lose the low 11 bits again and leave thousands of fix-up iterations below
    {
        const u128 rr = (u128)r * r;
        const bool over = rr > N;
        const double delta = (double)(over ? rr - N : N - rr) / (2.0 * (double)r);
        const uint64_t step = (uint64_t)__builtin_rint(delta);
        if (over) r = step > r - 0x8000000000000000ull ? 0x8000000000000000ull : r - step;
        else r = step > 0xffffffffffffffffull - r ? 0xffffffffffffffffull : r + step;
    }
    while ((u128)r * r > N) --r;
    while (r != 0xffffffffffffffffull && (u128)(r + 1) * (r + 1) <= N) ++r;
    // r = floor(sqrt(N)); round to nearest (no ties for integer N): up iff N - r^2 > r
    int e = qe;
    if (N - (u128)r * r > (u128)r) {
        ++r;
        if (r == 0) { r = 0x8000000000000000ull; ++e; }  // 2^64 -> 2^63 * 2
    }
    // round the 64-bit mantissa to 53 bits (FST m64 -> double), RNE
    uint64_t m53 = r >> 11;
    const uint64_t drop = r & 0x7ff;
    int e53 = e + 11;
    if (drop > 0x400 || (drop == 0x400 && (m53 & 1))) {
        ++m53;
        if (m53 == (1ull << 53)) { m53 >>= 1; ++e53; }
    }
    return __builtin_ldexp((double)m53, e53);
}

// OpenBLAS dnrm2 (kernel/x86_64/nrm2.S): 4 accumulators over the 8-unrolled body, the
// remainder into accumulator 0, combined d + ((c + a) + b)
TMF_LPN double dnrm2(int n, const double *x, int inc)
{
    if (n <= 0) return 0.0;
    X80 a = {0, 0}, b = {0, 0}, c = {0, 0}, d = {0, 0};
    int i = 0;
    for (int g = 0; g < n / 8; ++g)
        for (int h = 0; h < 2; ++h, i += 4) {
            const X80 q0 = x80_sq(x[i * inc]), q1 = x80_sq(x[(i + 1) * inc]), q2 = x80_sq(x[(i + 2) * inc]),
                      q3 = x80_sq(x[(i + 3) * inc]);
            d = x80_add(d, q3);
            c = x80_add(c, q2);
            b = x80_add(b, q1);
            a = x80_add(a, q0);
        }
    for (; i < n; ++i) a = x80_add(a, x80_sq(x[i * inc]));
    X80 t = x80_add(c, a);
    t = x80_add(t, b);
    t = x80_add(d, t);
    return x80_sqrt_to_double(t);
}

// ---------------------------------------------------------------------------
// OpenBLAS SkylakeX level-2 kernels in the shapes dlarf uses (alpha = 1, beta = 0)
// ---------------------------------------------------------------------------
#define LP_AT(a, i, j, ld) (a)[(i) + (j) * (ld)]

template <class P>
TMF_LPN void gemv_t(int m, int n, const double *A, int lda, const double *x, int incx, double *y)
{
    const int m3 = m & 3, m1 = m - m3, n4 = n & ~3, n2 = n & 3;
    LP_PAR(P, j, n) {
        const double *a = A + j * lda;
        double yy = 0.0;
        if (m1) {
            double t;
            if (j < n4) {
                double l0 = 0, l1 = 0, l2 = 0, l3 = 0;
                for (int r = 0; r < m1; r += 4) {
                    l0 = __builtin_fma(a[r], x[r * incx], l0);
                    l1 = __builtin_fma(a[r + 1], x[(r + 1) * incx], l1);
                    l2 = __builtin_fma(a[r + 2], x[(r + 2) * incx], l2);
                    l3 = __builtin_fma(a[r + 3], x[(r + 3) * incx], l3);
                }
                t = (l0 + l2) + (l1 + l3);
            } else if ((n2 & 2) && j < n4 + 2) {
                double l0 = 0, l1 = 0;
                for (int r = 0; r < m1; r += 2) {
                    l0 = l0 + a[r] * x[r * incx];
                    l1 = l1 + a[r + 1] * x[(r + 1) * incx];
                }
                t = l0 + l1;
            } else {
                double l0 = 0, l1 = 0, l2 = 0, l3 = 0;
                for (int r = 0; r < m1; r += 4) {
                    l0 = l0 + a[r] * x[r * incx];
                    l1 = l1 + a[r + 1] * x[(r + 1) * incx];
                    l2 = l2 + a[r + 2] * x[(r + 2) * incx];
                    l3 = l3 + a[r + 3] * x[(r + 3) * incx];
                }
                t = (l0 + l2) + (l1 + l3);
            }
            yy = __builtin_fma(t, 1.0, yy);
        }
        const double *xt = x + m1 * incx;
        if (m3 == 3)
            yy = yy + __builtin_fma(a[m1 + 2], xt[2 * incx], __builtin_fma(a[m1], xt[0], a[m1 + 1] * xt[incx]));
        else if (m3 == 2)
            yy = yy + __builtin_fma(a[m1], xt[0], a[m1 + 1] * xt[incx]);
        else if (m3 == 1)
            yy = __builtin_fma(a[m1], xt[0], yy);
        y[j] = yy;
    }
    P::sync();
}

template <class P>
TMF_LPN void gemv_n(int m, int n, const double *A, int lda, const double *x, int incx, double *y)
{
    const int m3 = m & 3, m1 = m - m3, n4 = n & ~3;
    LP_PAR(P, r, m) {
        if (r < m1) {
            double yr = 0.0;
            int j = 0;
            for (; j < n4; j += 4) {
                double s = LP_AT(A, r, j + 1, lda) * x[(j + 1) * incx];
                s = __builtin_fma(LP_AT(A, r, j, lda), x[j * incx], s);
                s = __builtin_fma(LP_AT(A, r, j + 2, lda), x[(j + 2) * incx], s);
                s = __builtin_fma(LP_AT(A, r, j + 3, lda), x[(j + 3) * incx], s);
                yr = __builtin_fma(1.0, s, yr);
            }
            if (incx == 1 && (n & 2)) {
                double s = LP_AT(A, r, j + 1, lda) * x[j + 1];
                s = __builtin_fma(LP_AT(A, r, j, lda), x[j], s);
                yr = __builtin_fma(1.0, s, yr);
                j += 2;
            }
            for (; j < n; ++j) yr = yr + LP_AT(A, r, j, lda) * (x[j * incx] * 1.0);
            y[r] = yr;
        } else {
            double t = 0.0;
            for (int j = 0; j < n; ++j) t = __builtin_fma(LP_AT(A, r, j, lda), x[j * incx], t);
            y[r] = __builtin_fma(1.0, t, 0.0);
        }
    }
    P::sync();
}

template <class P>
TMF_LPI void ger(int m, int n, double alpha, const double *x, int incx, const double *y, int incy, double *A, int lda)
{
    if (m <= 0 || n <= 0 || alpha == 0.0) return;
    LP_PAR(P, k, m * n) {
        const int j = k / m, i = k - j * m;
        const double t = alpha * y[j * incy];
        LP_AT(A, i, j, lda) = __builtin_fma(t, x[i * incx], LP_AT(A, i, j, lda));
    }
    P::sync();
}

template <class P>
TMF_LPI void drot(int n, double *x, int incx, double *y, int incy, double c, double s)
{
    LP_PAR(P, i, n) {
        const double xi = x[i * incx], yi = y[i * incy];
        x[i * incx] = __builtin_fma(c, xi, s * yi);
        y[i * incy] = __builtin_fma(c, yi, -(s * xi));
    }
    P::sync();
}

template <class P>
TMF_LPI void dswap(int n, double *x, int incx, double *y, int incy)
{
    LP_PAR(P, i, n) {
        const double t = x[i * incx];
        x[i * incx] = y[i * incy];
        y[i * incy] = t;
    }
    P::sync();
}

// ---------------------------------------------------------------------------
// LAPACK 3.12.0 (plain IEEE double)
// ---------------------------------------------------------------------------
TMF_LPI double fsign(double a, double b) { return __builtin_copysign(__builtin_fabs(a), b); }
TMF_LPI double dmax(double a, double b) { return a > b ? a : b; }
TMF_LPI double dmin(double a, double b) { return a < b ? a : b; }

TMF_LPI double dlapy2(double x, double y)
{
    const double xa = __builtin_fabs(x), ya = __builtin_fabs(y);
    const double w = xa > ya ? xa : ya, z = xa < ya ? xa : ya;
    if (z == 0.0 || w > kHuge) return w;
    const double q = z / w;
    return w * __builtin_sqrt(1.0 + q * q);
}

template <class P>
TMF_LPN void dlarfg(int n, double *alpha, double *x, int incx, double *tau)
{
    // scalars (*alpha, *tau, beta, the norms) are computed, read and written by every lane alike
    if (n <= 1) { *tau = 0.0; return; }
    double xnorm = dnrm2(n - 1, x, incx);
    if (xnorm == 0.0) { *tau = 0.0; return; }
    double beta = -fsign(dlapy2(*alpha, xnorm), *alpha);
    const double safmin = kSafmin / kEps, rsafmn = 1.0 / safmin;
    int knt = 0;
    if (__builtin_fabs(beta) < safmin) {
        do {
            ++knt;
            LP_PAR(P, i, n - 1) x[i * incx] *= rsafmn;
            P::sync();
            beta *= rsafmn;
            *alpha *= rsafmn;
        } while (__builtin_fabs(beta) < safmin && knt < 20);
        xnorm = dnrm2(n - 1, x, incx);
        beta = -fsign(dlapy2(*alpha, xnorm), *alpha);
    }
    *tau = (beta - *alpha) / beta;
    const double sc = 1.0 / (*alpha - beta);
    LP_PAR(P, i, n - 1) x[i * incx] *= sc;
    P::sync();
    for (int j = 0; j < knt; ++j) beta *= safmin;
    *alpha = beta;
}

TMF_LPI int iladlc(int m, int n, const double *A, int lda)
{
    if (n == 0) return 0;
    if (LP_AT(A, 0, n - 1, lda) != 0.0 || LP_AT(A, m - 1, n - 1, lda) != 0.0) return n;
    for (int j = n; j >= 1; --j)
        for (int i = 0; i < m; ++i)
            if (LP_AT(A, i, j - 1, lda) != 0.0) return j;
    return 0;
}

TMF_LPI int iladlr(int m, int n, const double *A, int lda)
{
    if (m == 0) return 0;
    if (LP_AT(A, m - 1, 0, lda) != 0.0 || LP_AT(A, m - 1, n - 1, lda) != 0.0) return m;
    int r = 0;
    for (int j = 0; j < n; ++j) {
        int i = m;
        while (i >= 1 && LP_AT(A, (i > 1 ? i : 1) - 1, j, lda) == 0.0) --i;
        if (i > r) r = i;
    }
    return r;
}

template <class P>
TMF_LPN void dlarf(int left, int m, int n, const double *v, int incv, double tau, double *C, int ldc, double *work)
{
    int lastv = 0, lastc = 0;
    if (tau != 0.0) {
        lastv = left ? m : n;
        int i = incv > 0 ? (lastv - 1) * incv : 0;
        while (lastv > 0 && v[i] == 0.0) { --lastv; i -= incv; }
        lastc = left ? iladlc(lastv, n, C, ldc) : iladlr(m, lastv, C, ldc);
    }
    if (lastv <= 0 || lastc <= 0) return;
    if (left) {
        gemv_t<P>(lastv, lastc, C, ldc, v, incv, work);
        ger<P>(lastv, lastc, -tau, v, incv, work, 1, C, ldc);
    } else {
        gemv_n<P>(lastc, lastv, C, ldc, v, incv, work);
        ger<P>(lastc, lastv, -tau, work, 1, v, incv, C, ldc);
    }
}

template <class P>
TMF_LPN void dgebd2(int n, double *A, int lda, double *d, double *e, double *tauq, double *taup, double *work)
{
    const int m = n;
    for (int i = 0; i < n; ++i) {
        dlarfg<P>(m - i, &LP_AT(A, i, i, lda), &LP_AT(A, (i + 1 < m ? i + 1 : m - 1), i, lda), 1, &tauq[i]);
        d[i] = LP_AT(A, i, i, lda);
        LP_AT(A, i, i, lda) = 1.0;
        if (i < n - 1) dlarf<P>(1, m - i, n - i - 1, &LP_AT(A, i, i, lda), 1, tauq[i], &LP_AT(A, i, i + 1, lda), lda, work);
        LP_AT(A, i, i, lda) = d[i];
        if (i < n - 1) {
            dlarfg<P>(n - i - 1, &LP_AT(A, i, i + 1, lda), &LP_AT(A, i, (i + 2 < n ? i + 2 : n - 1), lda), lda, &taup[i]);
            e[i] = LP_AT(A, i, i + 1, lda);
            LP_AT(A, i, i + 1, lda) = 1.0;
            dlarf<P>(0, m - i - 1, n - i - 1, &LP_AT(A, i, i + 1, lda), lda, taup[i], &LP_AT(A, i + 1, i + 1, lda), lda, work);
            LP_AT(A, i, i + 1, lda) = e[i];
        } else {
            taup[i] = 0.0;
        }
    }
}

TMF_LPN void dlartg(double f, double g, double *c, double *s, double *r)
{
    const double safmin = kSafmin, safmax = 1.0 / kSafmin;
    const double f1 = __builtin_fabs(f), g1 = __builtin_fabs(g);
    if (g == 0.0) {
        *c = 1.0; *s = 0.0; *r = f;
    } else if (f == 0.0) {
        *c = 0.0; *s = fsign(1.0, g); *r = g1;
    } else if (f1 > kRtmin && f1 < kRtmax && g1 > kRtmin && g1 < kRtmax) {
        const double d = __builtin_sqrt(f * f + g * g);
        *c = f1 / d;
        *r = fsign(d, f);
        *s = g / *r;
    } else {
        double u = f1 > g1 ? f1 : g1;
        if (safmin > u) u = safmin;
        if (u > safmax) u = safmax;
        const double fs = f / u, gs = g / u;
        const double d = __builtin_sqrt(fs * fs + gs * gs);
        *c = __builtin_fabs(fs) / d;
        *r = fsign(d, f);
        *s = gs / *r;
        *r = *r * u;
    }
}

TMF_LPN void dlas2(double f, double g, double h, double *ssmin, double *ssmax)
{
    const double fa = __builtin_fabs(f), ga = __builtin_fabs(g), ha = __builtin_fabs(h);
    const double fhmn = fa < ha ? fa : ha, fhmx = fa > ha ? fa : ha;
    if (fhmn == 0.0) {
        *ssmin = 0.0;
        if (fhmx == 0.0) {
            *ssmax = ga;
        } else {
            const double mx = fhmx > ga ? fhmx : ga, mn = fhmx < ga ? fhmx : ga;
            const double q = mn / mx;
            *ssmax = mx * __builtin_sqrt(1.0 + q * q);
        }
    } else if (ga < fhmx) {
        const double as = 1.0 + fhmn / fhmx, at = (fhmx - fhmn) / fhmx;
        const double au0 = ga / fhmx, au = au0 * au0;
        const double c = 2.0 / (__builtin_sqrt(as * as + au) + __builtin_sqrt(at * at + au));
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
            const double c = 1.0 / (__builtin_sqrt(1.0 + p * p) + __builtin_sqrt(1.0 + q * q));
            const double mn = (fhmn * c) * au;
            *ssmin = mn + mn;
            *ssmax = ga / (c + c);
        }
    }
}

TMF_LPN void dlasv2(double f, double g, double h, double *ssmin, double *ssmax, double *snr, double *csr, double *snl, double *csl)
{
    double ft = f, fa = __builtin_fabs(ft), ht = h, ha = __builtin_fabs(h);
    int pmax = 1;
    const bool swap = ha > fa;
    if (swap) {
        pmax = 3;
        double t = ft; ft = ht; ht = t;
        t = fa; fa = ha; ha = t;
    }
    const double gt = g, ga = __builtin_fabs(gt);
    double clt = 1.0, crt = 1.0, slt = 0.0, srt = 0.0;
    if (ga == 0.0) {
        *ssmin = ha;
        *ssmax = fa;
    } else {
        bool gasmal = true;
        if (ga > fa) {
            pmax = 2;
            if (fa / ga < kEps) {
                gasmal = false;
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
            const double s = __builtin_sqrt(tt + mm);
            const double r = (l == 0.0) ? __builtin_fabs(mm0) : __builtin_sqrt(l * l + mm);
            const double a = 0.5 * (s + r);
            *ssmin = ha / a;
            *ssmax = fa * a;
            if (mm == 0.0) {
                if (l == 0.0) t = fsign(2.0, ft) * fsign(1.0, gt);
                else t = gt / fsign(dd, ft) + mm0 / t;
            } else {
                t = (mm0 / (s + t) + mm0 / (r + l)) * (1.0 + a);
            }
            l = __builtin_sqrt(t * t + 4.0);
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

// dlasr, PIVOT = 'V': left -> rows j, j+1 of an m x n A; right -> columns j, j+1; the
// rotations (c, s) are elements [0, k-1) of two LVecs.  A lane keeps one column (left) /
// row (right) through every rotation of the sequence.
template <class P>
TMF_LPN void dlasr(bool left, bool fwd, int m, int n, const LVec<P> &c, const LVec<P> &s, double *A, int lda)
{
    const int k = left ? m : n;
    LP_PAR(P, i, left ? n : m) {
        for (int q = 0; q < k - 1; ++q) {
            const int j = fwd ? q : k - 2 - q;
            const double ct = c.get(j), st = s.get(j);
            if (ct == 1.0 && st == 0.0) continue;
            if (left) {
                const double t = LP_AT(A, j + 1, i, lda);
                LP_AT(A, j + 1, i, lda) = ct * t - st * LP_AT(A, j, i, lda);
                LP_AT(A, j, i, lda) = st * t + ct * LP_AT(A, j, i, lda);
            } else {
                const double t = LP_AT(A, i, j + 1, lda);
                LP_AT(A, i, j + 1, lda) = ct * t - st * LP_AT(A, i, j, lda);
                LP_AT(A, i, j, lda) = st * t + ct * LP_AT(A, i, j, lda);
            }
        }
    }
    P::sync();
}

// dbdsqr('U', n, ncvt = n, nru = n, ncc = 0).  WANT_V = false skips the vector
// updates only (the d / e recurrences do not read the vectors, so the singular values
// are those of the vector-carrying run -- not dlasq1's, which LAPACK would use without
// vectors and numpy never does).  Returns 0, or 1 if not converged.
template <bool WANT_V, class P>
TMF_LPN int dbdsqr(int n, LVec<P> &d, LVec<P> &e, double *VT, int ldvt, double *U, int ldu)
{
    const int maxitr = 6;
    if (n == 0) return 0;
    if (n > 1) {
        LVec<P> w0, w1, w2, w3;  // LAPACK's WORK(1..4(n-1)) as its four (n-1)-long sequences
        const double eps = kEps, unfl = kSafmin;
        const double tol = kTolmul * eps;
        double smax = 0.0;
        for (int i = 0; i < n; ++i) smax = dmax(smax, __builtin_fabs(d.get(i)));
        for (int i = 0; i < n - 1; ++i) smax = dmax(smax, __builtin_fabs(e.get(i)));
        double sminoa = __builtin_fabs(d.get(0));
        if (sminoa != 0.0) {
            double mu = sminoa;
            for (int i = 1; i < n; ++i) {
                mu = __builtin_fabs(d.get(i)) * (mu / (mu + __builtin_fabs(e.get(i - 1))));
                sminoa = dmin(sminoa, mu);
                if (sminoa == 0.0) break;
            }
        }
        sminoa = sminoa / __builtin_sqrt((double)n);
        double thresh;
        {
            const double a = tol * sminoa, b = (double)maxitr * ((double)n * ((double)n * unfl));
            thresh = a > b ? a : b;
        }
        const int maxitdivn = maxitr * n;
        int iterdivn = 0, iter = -1, oldll = -1, oldm = -1, idir = 0;
        int m = n;
#define D_(i) d.get((i) - 1)
#define E_(i) e.get((i) - 1)
        for (;;) {
            if (m <= 1) break;
            if (iter >= n) {
                iter -= n;
                ++iterdivn;
                if (iterdivn >= maxitdivn) return 1;
            }
            double smin = 0.0;
            smax = __builtin_fabs(D_(m));
            int ll = 0;
            bool split = false;
            for (int lll = 1; lll <= m - 1; ++lll) {
                ll = m - lll;
                const double abss = __builtin_fabs(D_(ll)), abse = __builtin_fabs(E_(ll));
                if (abse <= thresh) { split = true; break; }
                smax = dmax(smax, dmax(abss, abse));
            }
            if (split) {
                e.set((ll) - 1, 0.0);
                if (ll == m - 1) { m = m - 1; continue; }
            } else {
                ll = 0;
            }
            ll = ll + 1;
            if (ll == m - 1) {
                double sigmn, sigmx, sinr, cosr, sinl, cosl;
                dlasv2(D_(m - 1), E_(m - 1), D_(m), &sigmn, &sigmx, &sinr, &cosr, &sinl, &cosl);
                d.set((m - 1) - 1, sigmx);
                e.set((m - 1) - 1, 0.0);
                d.set((m) - 1, sigmn);
                if (WANT_V) {
                    drot<P>(n, &LP_AT(VT, m - 2, 0, ldvt), ldvt, &LP_AT(VT, m - 1, 0, ldvt), ldvt, cosr, sinr);
                    drot<P>(n, &LP_AT(U, 0, m - 2, ldu), 1, &LP_AT(U, 0, m - 1, ldu), 1, cosl, sinl);
                }
                m = m - 2;
                continue;
            }
            if (ll > oldm || m < oldll) idir = __builtin_fabs(D_(ll)) >= __builtin_fabs(D_(m)) ? 1 : 2;
            bool conv = false;
            if (idir == 1) {
                if (__builtin_fabs(E_(m - 1)) <= __builtin_fabs(tol) * __builtin_fabs(D_(m))) { e.set((m - 1) - 1, 0.0); continue; }
                double mu = __builtin_fabs(D_(ll));
                smin = mu;
                for (int lll = ll; lll <= m - 1; ++lll) {
                    if (__builtin_fabs(E_(lll)) <= tol * mu) { e.set((lll) - 1, 0.0); conv = true; break; }
                    mu = __builtin_fabs(D_(lll + 1)) * (mu / (mu + __builtin_fabs(E_(lll))));
                    smin = dmin(smin, mu);
                }
            } else {
                if (__builtin_fabs(E_(ll)) <= __builtin_fabs(tol) * __builtin_fabs(D_(ll))) { e.set((ll) - 1, 0.0); continue; }
                double mu = __builtin_fabs(D_(m));
                smin = mu;
                for (int lll = m - 1; lll >= ll; --lll) {
                    if (__builtin_fabs(E_(lll)) <= tol * mu) { e.set((lll) - 1, 0.0); conv = true; break; }
                    mu = __builtin_fabs(D_(lll)) * (mu / (mu + __builtin_fabs(E_(lll))));
                    smin = dmin(smin, mu);
                }
            }
            if (conv) continue;
            oldll = ll;
            oldm = m;
            double shift, r;
            {
                const double lhs = (double)n * tol * (smin / smax);
                const double rhs = eps > 0.01 * tol ? eps : 0.01 * tol;
                if (lhs <= rhs) {
                    shift = 0.0;
                } else {
                    double sll;
                    if (idir == 1) { sll = __builtin_fabs(D_(ll)); dlas2(D_(m - 1), E_(m - 1), D_(m), &shift, &r); }
                    else { sll = __builtin_fabs(D_(m)); dlas2(D_(ll), E_(ll), D_(ll + 1), &shift, &r); }
                    if (sll > 0.0) {
                        const double qq = shift / sll;
                        if (qq * qq < eps) shift = 0.0;
                    }
                }
            }
            iter = iter + m - ll;
            if (shift == 0.0) {
                if (idir == 1) {
                    double cs = 1.0, oldcs = 1.0, sn = 0.0, oldsn = 0.0;
                    for (int i = ll; i <= m - 1; ++i) {
                        dlartg(D_(i) * cs, E_(i), &cs, &sn, &r);
                        if (i > ll) e.set((i - 1) - 1, oldsn * r);
                        { double di; dlartg(oldcs * r, D_(i + 1) * sn, &oldcs, &oldsn, &di); d.set(i - 1, di); }
                        w0.set(i - ll, cs);
                        w1.set(i - ll, sn);
                        w2.set(i - ll, oldcs);
                        w3.set(i - ll, oldsn);
                    }
                    const double h = D_(m) * cs;
                    d.set((m) - 1, h * oldcs);
                    e.set((m - 1) - 1, h * oldsn);
                    if (WANT_V) {
                        dlasr<P>(true, true, m - ll + 1, n, w0, w1, &LP_AT(VT, ll - 1, 0, ldvt), ldvt);
                        dlasr<P>(false, true, n, m - ll + 1, w2, w3, &LP_AT(U, 0, ll - 1, ldu), ldu);
                    }
                    if (__builtin_fabs(E_(m - 1)) <= thresh) e.set((m - 1) - 1, 0.0);
                } else {
                    double cs = 1.0, oldcs = 1.0, sn = 0.0, oldsn = 0.0;
                    for (int i = m; i >= ll + 1; --i) {
                        dlartg(D_(i) * cs, E_(i - 1), &cs, &sn, &r);
                        if (i < m) e.set((i) - 1, oldsn * r);
                        { double di; dlartg(oldcs * r, D_(i - 1) * sn, &oldcs, &oldsn, &di); d.set(i - 1, di); }
                        w0.set(i - ll - 1, cs);
                        w1.set(i - ll - 1, -sn);
                        w2.set(i - ll - 1, oldcs);
                        w3.set(i - ll - 1, -oldsn);
                    }
                    const double h = D_(ll) * cs;
                    d.set((ll) - 1, h * oldcs);
                    e.set((ll) - 1, h * oldsn);
                    if (WANT_V) {
                        dlasr<P>(true, false, m - ll + 1, n, w2, w3, &LP_AT(VT, ll - 1, 0, ldvt), ldvt);
                        dlasr<P>(false, false, n, m - ll + 1, w0, w1, &LP_AT(U, 0, ll - 1, ldu), ldu);
                    }
                    if (__builtin_fabs(E_(ll)) <= thresh) e.set((ll) - 1, 0.0);
                }
            } else {
                if (idir == 1) {
                    double f = (__builtin_fabs(D_(ll)) - shift) * (fsign(1.0, D_(ll)) + shift / D_(ll));
                    double g = E_(ll);
                    double cosr, sinr, cosl, sinl;
                    for (int i = ll; i <= m - 1; ++i) {
                        dlartg(f, g, &cosr, &sinr, &r);
                        if (i > ll) e.set((i - 1) - 1, r);
                        f = cosr * D_(i) + sinr * E_(i);
                        e.set((i) - 1, cosr * E_(i) - sinr * D_(i));
                        g = sinr * D_(i + 1);
                        d.set((i + 1) - 1, cosr * D_(i + 1));
                        dlartg(f, g, &cosl, &sinl, &r);
                        d.set((i) - 1, r);
                        f = cosl * E_(i) + sinl * D_(i + 1);
                        d.set((i + 1) - 1, cosl * D_(i + 1) - sinl * E_(i));
                        if (i < m - 1) {
                            g = sinl * E_(i + 1);
                            e.set((i + 1) - 1, cosl * E_(i + 1));
                        }
                        w0.set(i - ll, cosr);
                        w1.set(i - ll, sinr);
                        w2.set(i - ll, cosl);
                        w3.set(i - ll, sinl);
                    }
                    e.set((m - 1) - 1, f);
                    if (WANT_V) {
                        dlasr<P>(true, true, m - ll + 1, n, w0, w1, &LP_AT(VT, ll - 1, 0, ldvt), ldvt);
                        dlasr<P>(false, true, n, m - ll + 1, w2, w3, &LP_AT(U, 0, ll - 1, ldu), ldu);
                    }
                    if (__builtin_fabs(E_(m - 1)) <= thresh) e.set((m - 1) - 1, 0.0);
                } else {
                    double f = (__builtin_fabs(D_(m)) - shift) * (fsign(1.0, D_(m)) + shift / D_(m));
                    double g = E_(m - 1);
                    double cosr, sinr, cosl, sinl;
                    for (int i = m; i >= ll + 1; --i) {
                        dlartg(f, g, &cosr, &sinr, &r);
                        if (i < m) e.set((i) - 1, r);
                        f = cosr * D_(i) + sinr * E_(i - 1);
                        e.set((i - 1) - 1, cosr * E_(i - 1) - sinr * D_(i));
                        g = sinr * D_(i - 1);
                        d.set((i - 1) - 1, cosr * D_(i - 1));
                        dlartg(f, g, &cosl, &sinl, &r);
                        d.set((i) - 1, r);
                        f = cosl * E_(i - 1) + sinl * D_(i - 1);
                        d.set((i - 1) - 1, cosl * D_(i - 1) - sinl * E_(i - 1));
                        if (i > ll + 1) {
                            g = sinl * E_(i - 2);
                            e.set((i - 2) - 1, cosl * E_(i - 2));
                        }
                        w0.set(i - ll - 1, cosr);
                        w1.set(i - ll - 1, -sinr);
                        w2.set(i - ll - 1, cosl);
                        w3.set(i - ll - 1, -sinl);
                    }
                    e.set((ll) - 1, f);
                    if (__builtin_fabs(E_(ll)) <= thresh) e.set((ll) - 1, 0.0);
                    if (WANT_V) {
                        dlasr<P>(true, false, m - ll + 1, n, w2, w3, &LP_AT(VT, ll - 1, 0, ldvt), ldvt);
                        dlasr<P>(false, false, n, m - ll + 1, w0, w1, &LP_AT(U, 0, ll - 1, ldu), ldu);
                    }
                }
            }
        }
#undef D_
#undef E_
    }
    for (int i = 0; i < n; ++i)
        if (d.get(i) < 0.0) {
            d.set(i, -d.get(i));
            if (WANT_V) {
                LP_PAR(P, j, n) LP_AT(VT, i, j, ldvt) *= -1.0;
                P::sync();
            }
        }
    // dbdsqr: descending selection sort (.LE.: the last of a tie moves)
    for (int i = 1; i <= n - 1; ++i) {
        int isub = 1;
        double smin = d.get(0);
        for (int j = 2; j <= n + 1 - i; ++j)
            if (d.get(j - 1) <= smin) { isub = j; smin = d.get(j - 1); }
        if (isub != n + 1 - i) {
            d.set(isub - 1, d.get(n - i));
            d.set(n - i, smin);
            if (WANT_V) {
                dswap<P>(n, &LP_AT(VT, isub - 1, 0, ldvt), ldvt, &LP_AT(VT, n - i, 0, ldvt), ldvt);
                dswap<P>(n, &LP_AT(U, 0, isub - 1, ldu), 1, &LP_AT(U, 0, n - i, ldu), 1);
            }
        }
    }
    return 0;
}

// dbdsdc('U', 'I') for n <= 25: U = VT = I, dlasdq -> dbdsqr, dlasdq's ascending
// selection sort (.LT.), dbdsdc's descending selection sort (.GT.)
template <bool WANT_V, class P>
TMF_LPN int dbdsdc(int n, LVec<P> &d, LVec<P> &e, double *U, int ldu, double *VT, int ldvt)
{
    if (WANT_V) {
        LP_PAR(P, k, n * n) {
            const int j = k / n, i = k - j * n;
            LP_AT(U, i, j, ldu) = (i == j) ? 1.0 : 0.0;
            LP_AT(VT, i, j, ldvt) = (i == j) ? 1.0 : 0.0;
        }
        P::sync();
    }
    if (n == 1) {
        if (WANT_V) { LP_AT(U, 0, 0, ldu) = fsign(1.0, d.get(0)); LP_AT(VT, 0, 0, ldvt) = 1.0; }
        d.set(0, __builtin_fabs(d.get(0)));
        return 0;
    }
    const int info = dbdsqr<WANT_V, P>(n, d, e, VT, ldvt, U, ldu);
    for (int i = 0; i < n; ++i) {
        int isub = i;
        double smin = d.get(i);
        for (int j = i + 1; j < n; ++j)
            if (d.get(j) < smin) { isub = j; smin = d.get(j); }
        if (isub != i) {
            d.set(isub, d.get(i));
            d.set(i, smin);
            if (WANT_V) {
                dswap<P>(n, &LP_AT(VT, isub, 0, ldvt), ldvt, &LP_AT(VT, i, 0, ldvt), ldvt);
                dswap<P>(n, &LP_AT(U, 0, isub, ldu), 1, &LP_AT(U, 0, i, ldu), 1);
            }
        }
    }
    for (int i = 0; i < n - 1; ++i) {
        int kk = i;
        double p = d.get(i);
        for (int j = i + 1; j < n; ++j)
            if (d.get(j) > p) { kk = j; p = d.get(j); }
        if (kk != i) {
            d.set(kk, d.get(i));
            d.set(i, p);
            if (WANT_V) {
                dswap<P>(n, &LP_AT(U, 0, i, ldu), 1, &LP_AT(U, 0, kk, ldu), 1);
                dswap<P>(n, &LP_AT(VT, i, 0, ldvt), ldvt, &LP_AT(VT, kk, 0, ldvt), ldvt);
            }
        }
    }
    return info;
}

// dormbr('Q','L','N') -> dorm2r: H(k) ... H(1) applied backwards to U
template <class P>
TMF_LPN void apply_q(int n, double *A, const double *tauq, double *U, double *work)
{
    for (int i = n - 1; i >= 0; --i) {
        const double aii = LP_AT(A, i, i, n);
        LP_AT(A, i, i, n) = 1.0;
        dlarf<P>(1, n - i, n, &LP_AT(A, i, i, n), 1, tauq[i], &LP_AT(U, i, 0, n), n, work);
        LP_AT(A, i, i, n) = aii;
    }
}

// dormbr('P','R','T'), nq = k = n -> dorml2('R','N', n, n-1, n-1, A(1,2), taup, VT(1,2))
template <class P>
TMF_LPN void apply_pt(int n, double *A, const double *taup, double *VT, double *work)
{
    if (n <= 1) return;
    double *A2 = A + n;
    double *C2 = VT + n;
    for (int i = n - 2; i >= 0; --i) {
        const double aii = A2[i + i * n];
        A2[i + i * n] = 1.0;
        dlarf<P>(0, n, n - 1 - i, &A2[i + i * n], n, taup[i], C2 + i * n, n, work);
        A2[i + i * n] = aii;
    }
}

// Working set of one block's dgesdd: A, U, VT (n x n), d, e, tauq, taup (n), and the BLAS /
// dbdsqr work vectors (n + 4n) -- in doubles.  The fixup kernels carve it out of LDS.  Without
// vectors (JOBZ = 'N', extract) U and VT are not part of it: A, then the vectors.
TMF_LPI constexpr int ws_doubles(int n) { return 3 * n * n + 9 * n; }
TMF_LPI constexpr int ws_doubles_s(int n) { return n * n + 9 * n; }
// the compact layout (svd_f32_ws<true, P, true>): no work slot of its own -- dgebd2's dlarf vector
// sits in U's slot (free until dbdsdc sets U to the identity), apply_q / apply_pt's in d's (d and
// e are in registers by then) -- so A, U, VT, d, e, tauq, taup: 3 n^2 + 4 n
TMF_LPI constexpr int ws_doubles_compact(int n) { return 3 * n * n + 4 * n; }
template <bool WANT_V>
TMF_LPI constexpr int ws_doubles_for(int n) { return WANT_V ? ws_doubles(n) : ws_doubles_s(n); }

// np.linalg.svd of one float32 n x n block (row-major D): f32 U (row-major u[r][k]),
// S, Vt (row-major vt[k][j]) exactly as numpy returns them, in the caller's workspace
// ws (ws_doubles_for<WANT_V>(n)).  Returns dbdsqr's info (0, or 1: not converged -- np.linalg.svd
// raises LinAlgError there).  Under WavePar every lane of the wave calls it for the same
// block, with ws, D and the outputs in LDS or global memory visible to the whole wave.
template <bool WANT_V, class P = SerialPar, bool COMPACT = false>
TMF_LPN int svd_f32_ws(const float *D, int n, float *Uo, float *So, float *Vto, double *ws)
{
    static_assert(!COMPACT || WANT_V, "the compact layout borrows U's slot");
    double *A = ws, *U = WANT_V ? A + n * n : nullptr, *VT = WANT_V ? U + n * n : nullptr, *d = A + (WANT_V ? 3 : 1) * n * n,
           *e = d + n, *tauq = e + n, *taup = tauq + n, *work = COMPACT ? U : taup + n;
    LP_PAR(P, k, n * n) {
        const int j = k / n, i = k - j * n;
        A[i + j * n] = (double)D[i * n + j];
    }
    P::sync();
    // dgesdd scales only when max|a| is outside [sqrt(safmin)/prec, its inverse]: never for f32 data
    dgebd2<P>(n, A, n, d, e, tauq, taup, work);
    LVec<P> dv, ev;
    dv.load(d, n);
    ev.load(e, n - 1);
    const int info = dbdsdc<WANT_V, P>(n, dv, ev, U, n, VT, n);
    if (WANT_V) {
        double *work2 = COMPACT ? d : work;
        apply_q<P>(n, A, tauq, U, work2);
        apply_pt<P>(n, A, taup, VT, work2);
        if (Uo) {  // NULL: the caller reads U (ws + n^2) and VT (ws + 2 n^2), column-major f64, itself
            LP_PAR(P, q, n * n) {
                const int i = q / n, k = q - i * n;
                Uo[i * n + k] = (float)U[i + k * n];
                Vto[i * n + k] = (float)VT[i + k * n];
            }
        }
    }
    dv.store_f32(So, n);
    P::sync();
    return info;
}

// the same with a private workspace (host builds)
template <bool WANT_V, class P = SerialPar>
TMF_LPN int svd_f32(const float *D, int n, float *Uo, float *So, float *Vto)
{
    double ws[ws_doubles(kMaxN)];
    return svd_f32_ws<WANT_V, P>(D, n, Uo, So, Vto, ws);
}

}  // namespace lp
}  // namespace tmf
