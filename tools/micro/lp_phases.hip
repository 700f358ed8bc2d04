// Latency of one block's dgesdd route under lp::WavePar, by phase (s_memtime cycles):
// dgebd2, dbdsdc (dbdsqr + sorts), apply_q, apply_pt; and one dnrm2 of 7 elements.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o lp_phases lp_phases.hip
#include <cstdio>
#include <vector>
#include "../../thatsmyface_amd/csrc/tmfwm_lapack.h"

using namespace tmf::lp;

__global__ __launch_bounds__(64) void k_phases(const float *D, int n, unsigned long long *out)
{
    __shared__ double ws[ws_doubles(kMaxN)];
    using P = WavePar;
    double *A = ws, *U = A + n * n, *VT = U + n * n, *d = VT + n * n, *e = d + n, *tauq = e + n, *taup = tauq + n, *work = taup + n;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    LP_PAR(P, k, n * n) {
        const int j = k / n, i = k - j * n;
        A[i + j * n] = (double)D[i * n + j];
    }
    P::sync();
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    dgebd2<P>(n, A, n, d, e, tauq, taup, work);
    unsigned long long t2 = __builtin_amdgcn_s_memtime();
    {
        LVec<P> dv, ev;
        dv.load(d, n);
        ev.load(e, n - 1);
        dbdsdc<true, P>(n, dv, ev, U, n, VT, n);
    }
    unsigned long long t3 = __builtin_amdgcn_s_memtime();
    apply_q<P>(n, A, tauq, U, work);
    unsigned long long t4 = __builtin_amdgcn_s_memtime();
    apply_pt<P>(n, A, taup, VT, work);
    unsigned long long t5 = __builtin_amdgcn_s_memtime();
    double x = dnrm2(n - 1, A, 1);
    unsigned long long t6 = __builtin_amdgcn_s_memtime();
    // dgebd2's first steps, timed one by one: dlarfg (column), dlarf left, dlarfg (row), dlarf right
    LP_PAR(P, k, n * n) {
        const int j = k / n, i = k - j * n;
        A[i + j * n] = (double)D[i * n + j];
    }
    P::sync();
    unsigned long long s0 = __builtin_amdgcn_s_memtime();
    dlarfg<P>(n, &A[0], &A[1], 1, &tauq[0]);
    unsigned long long s1 = __builtin_amdgcn_s_memtime();
    const double a00 = A[0];
    A[0] = 1.0;
    dlarf<P>(1, n, n - 1, &A[0], 1, tauq[0], &A[n], n, work);
    A[0] = a00;
    unsigned long long s2 = __builtin_amdgcn_s_memtime();
    dlarfg<P>(n - 1, &A[n], &A[2 * n], n, &taup[0]);
    unsigned long long s3 = __builtin_amdgcn_s_memtime();
    const double xn = dlapy2(A[1], A[2]);
    unsigned long long s4 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {
        out[0] = t1 - t0; out[1] = t2 - t1; out[2] = t3 - t2; out[3] = t4 - t3; out[4] = t5 - t4; out[5] = t6 - t5;
        out[6] = (unsigned long long)(x != x) + (unsigned long long)(xn != xn);
        out[7] = s1 - s0; out[8] = s2 - s1; out[9] = s3 - s2; out[10] = s4 - s3;
    }
}

int main()
{
    for (int n : {8, 16}) {
        std::vector<float> h(n * n);
        unsigned s = 12345;
        for (auto &v : h) { s = s * 1664525u + 1013904223u; v = (float)((s >> 8) & 0xFFFF) / 65536.0f - 0.5f; }
        float *D; unsigned long long *o;
        hipMalloc(&D, n * n * 4); hipMalloc(&o, 16 * 8);
        hipMemcpy(D, h.data(), n * n * 4, hipMemcpyHostToDevice);
        for (int rep = 0; rep < 3; ++rep) {
            hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
            hipEventRecord(a);
            hipLaunchKernelGGL(k_phases, dim3(1), dim3(64), 0, 0, D, n, o);
            hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b);
            unsigned long long r[16]; hipMemcpy(r, o, 128, hipMemcpyDeviceToHost);
            printf("n=%d rep %d: kernel %.1f us | cycles: load %llu dgebd2 %llu dbdsdc %llu apply_q %llu apply_pt %llu dnrm2(%d) %llu\n",
                   n, rep, ms * 1000, r[0], r[1], r[2], r[3], r[4], n - 1, r[5]);
            printf("   dlarfg(col) %llu dlarf(left) %llu dlarfg(row) %llu dlapy2 %llu\n", r[7], r[8], r[9], r[10]);
        }
        hipFree(D); hipFree(o);
    }
    return 0;
}
