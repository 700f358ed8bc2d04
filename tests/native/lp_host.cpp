// TEST-ONLY: the device LAPACK route (thatsmyface_amd/csrc/tmfwm_lapack.h) compiled for
// the host CPU, so that tests/test_lapack_device_code.py can check the GPU code path
// against the oracle without a GPU.  Built by that test with hipcc; never shipped.
#include "../../thatsmyface_amd/csrc/tmfwm_lapack.h"

extern "C" {

int lp_host_svd_blocks(const float *D, long long nb, int b, float *U, float *S, float *Vt, int want_v)
{
    int bad = 0;
    for (long long k = 0; k < nb; ++k) {
        const int rc = want_v ? tmf::lp::svd_f32<true>(D + k * b * b, b, U + k * b * b, S + k * b, Vt + k * b * b)
                              : tmf::lp::svd_f32<false>(D + k * b * b, b, U + k * b * b, S + k * b, Vt + k * b * b);
        bad |= rc != 0;
    }
    return bad;
}

double lp_host_dnrm2(int n, const double *x, int inc) { return tmf::lp::dnrm2(n, x, inc); }

}
