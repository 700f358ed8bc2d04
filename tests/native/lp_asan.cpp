// TEST-ONLY: bounds check of the dgesdd route's workspace indexing (thatsmyface_amd/csrc/
// tmfwm_lapack.h) under AddressSanitizer on the host.  Every array -- D, U, S, Vt and the
// workspace of exactly ws_doubles_for<want_v>(n) doubles, the size the fixup kernels give it in LDS --
// is its own heap allocation of exactly its size, so any read or write past an end aborts.
// Built and run by tests/test_lapack_device_code.py::test_workspace_bounds_asan; never shipped.
#include "../../thatsmyface_amd/csrc/tmfwm_lapack.h"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <vector>

using namespace tmf::lp;

static unsigned long long g_rng = 0x9E3779B97F4A7C15ull;
static double uni()
{
    g_rng ^= g_rng << 13;
    g_rng ^= g_rng >> 7;
    g_rng ^= g_rng << 17;
    return (double)(g_rng >> 11) * 0x1p-53;
}

// cover-like test matrices: 0 noise, 1 rank-deficient (repeated columns), 2 zero,
// 3 tiny scale, 4 small integers (ties), 5 one nonzero, 6 huge scale, 7 graded rows
static void fill(float *D, int n, int kind)
{
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            double v = 2.0 * uni() - 1.0;
            if (kind == 1) v = std::sin(1.0 + i * 0.7) * ((j % 3) + 1);
            if (kind == 2) v = 0.0;
            if (kind == 3) v *= 1e-30;
            if (kind == 4) v = (double)(int)(3.0 * uni()) - 1.0;
            if (kind == 5) v = (i == n / 2 && j == n / 3) ? 0.5 : 0.0;
            if (kind == 6) v *= 1e30;
            if (kind == 7) v *= std::ldexp(1.0, -3 * i);
            D[i * n + j] = (float)v;
        }
}

template <class P>
static int run(int n, int kind, bool want_v)
{
    float *D = new float[n * n];
    fill(D, n, kind);
    float *U = want_v ? new float[n * n] : nullptr, *Vt = want_v ? new float[n * n] : nullptr;
    float *S = new float[n];
    double *ws = new double[want_v ? ws_doubles_for<true>(n) : ws_doubles_for<false>(n)];  // as the fixup kernels size it
    const int info = want_v ? svd_f32_ws<true, P>(D, n, U, S, Vt, ws) : svd_f32_ws<false, P>(D, n, nullptr, S, nullptr, ws);
    delete[] ws;
    delete[] S;
    delete[] Vt;
    delete[] U;
    delete[] D;
    return info;
}

// The compact layout as the b > 8 embed pass uses it (tmfwm_fixup.h FixLds<B, true>): a workspace of
// exactly ws_doubles_compact(n), D waiting in its U slot and S written into its e slot -- bounds
// under ASan, and the same U, S, Vt bits as the standard layout.  Returns the mismatches (or 1000
// when dbdsqr did not converge).
template <class P>
static int run_compact(int n, int kind)
{
    float *D = new float[n * n];
    fill(D, n, kind);
    float *U0 = new float[n * n], *V0 = new float[n * n], *S0 = new float[n], *U1 = new float[n * n], *V1 = new float[n * n];
    double *ws0 = new double[ws_doubles(n)];
    const int i0 = svd_f32_ws<true, P>(D, n, U0, S0, V0, ws0);
    double *ws = new double[ws_doubles_compact(n)];
    float *Din = reinterpret_cast<float *>(ws + n * n), *S1 = reinterpret_cast<float *>(ws + 3 * n * n + n);
    for (int k = 0; k < n * n; ++k) Din[k] = D[k];
    const int i1 = svd_f32_ws<true, P, true>(Din, n, U1, S1, V1, ws);
    int bad = (i0 || i1) ? 1000 : 0;
    for (int k = 0; k < n * n; ++k) bad += (std::memcmp(&U0[k], &U1[k], 4) != 0) + (std::memcmp(&V0[k], &V1[k], 4) != 0);
    for (int k = 0; k < n; ++k) bad += std::memcmp(&S0[k], &S1[k], 4) != 0;
    delete[] ws;
    delete[] ws0;
    delete[] V1;
    delete[] U1;
    delete[] S0;
    delete[] V0;
    delete[] U0;
    delete[] D;
    return bad;
}

int main()
{
    int cases = 0, bad = 0;
    for (int n = 1; n <= kMaxN; ++n)
        for (int kind = 0; kind < 8; ++kind)
            for (int rep = 0; rep < 4; ++rep)
                for (int v = 0; v < 2; ++v) {
                    bad += run<SerialPar>(n, kind, v) != 0;
                    bad += run<ReversePar>(n, kind, v) != 0;
                    cases += 2;
                }
    int compact_cases = 0, compact_bad = 0;
    for (int n = 1; n <= kMaxN; ++n)
        for (int kind = 0; kind < 8; ++kind) {
            compact_bad += run_compact<SerialPar>(n, kind) + run_compact<ReversePar>(n, kind);
            compact_cases += 2;
        }
    std::printf("{\"cases\": %d, \"not_converged\": %d, \"compact_cases\": %d, \"compact_mismatches\": %d}\n", cases, bad,
                compact_cases, compact_bad);
    return 0;
}
