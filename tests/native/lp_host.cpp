// TEST-ONLY: the device LAPACK route (thatsmyface_amd/csrc/tmfwm_lapack.h) compiled for
// the host CPU, so that tests/test_lapack_device_code.py can check the GPU code path
// against the oracle without a GPU.  Built by that test with hipcc; never shipped.
#include "../../thatsmyface_amd/csrc/tmfwm_lapack.h"

extern "C" {

// reverse != 0: every element loop runs backwards (ReversePar) -- the per-element bodies
// must not depend on the order in which the lanes of a wave would take them
int lp_host_svd_blocks(const float *D, long long nb, int b, float *U, float *S, float *Vt, int want_v, int reverse)
{
    using namespace tmf::lp;
    int bad = 0;
    for (long long k = 0; k < nb; ++k) {
        const float *d = D + k * b * b;
        float *u = U ? U + k * b * b : nullptr, *v = Vt ? Vt + k * b * b : nullptr, *s = S + k * b;
        int rc;
        if (reverse) rc = want_v ? svd_f32<true, ReversePar>(d, b, u, s, v) : svd_f32<false, ReversePar>(d, b, u, s, v);
        else rc = want_v ? svd_f32<true>(d, b, u, s, v) : svd_f32<false>(d, b, u, s, v);
        bad |= rc != 0;
    }
    return bad;
}

double lp_host_dnrm2(int n, const double *x, int inc) { return tmf::lp::dnrm2(n, x, inc); }

}
