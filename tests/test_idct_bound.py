"""The rank-1 pre-pass's IDCT tables (csrc/tmfwm_idct_bounds.h), made by
tools/exp/idct_bound.py: its transcription of pocketfft's f32 DCT-III is the device's op sequence
(bit for bit against the oracle's IDCT), the shipped header is what the tool generates, and the
rounding bound |IDCT_fl(x)_p - (C' x)_p| <= 2^-24 sum_i E[p][i] |x_i| holds on random and
adversarial inputs (C' x evaluated exactly in rationals)."""
import os
import sys
from fractions import Fraction

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "tools", "exp"))

import idct_bound as IB  # noqa: E402

SIZES = [4, 6, 8, 10, 12, 14, 16]


@pytest.mark.parametrize("n", SIZES)
def test_transcription_is_the_device_op_sequence(n):
    rng = np.random.default_rng(n)
    smp = (rng.standard_normal((4, n, n)) * rng.uniform(0.01, 30, (4, 1, 1))).astype(np.float32)
    res, _, _ = IB.analyse(n, smp)
    assert res["f32_values_equal_oracle"], res
    assert res["max_C_prime_minus_C"] < 1e-7, res


def test_shipped_header_is_generated(tmp_path):
    out = tmp_path / "h.h"
    IB.emit(str(out))
    with open(os.path.join(ROOT, "thatsmyface_amd", "csrc", "tmfwm_idct_bounds.h")) as f:
        assert f.read() == out.read_text()


@pytest.mark.parametrize("n", SIZES)
def test_rounding_bound_holds(n):
    _, Cp, E = IB.analyse(n)
    absc, err = (np.array(t) for t in IB.tables(n))
    assert np.all(absc >= np.abs(Cp)) and np.all(err >= E)
    rng = np.random.default_rng(100 + n)
    z = np.zeros(n)
    cq = [[Fraction(float(c)) for c in row] for row in Cp]
    worst = 0.0
    for t in range(300):
        # random magnitudes, and vectors concentrated on one coefficient (where |C| is smallest)
        x = rng.standard_normal(n) * 10.0 ** rng.uniform(-3, 2)
        if t % 3 == 0:
            x = np.zeros(n)
            x[rng.integers(n)] = rng.uniform(-40, 40)
            x += rng.standard_normal(n) * 1e-3
        x = x.astype(np.float32)
        y = [o.v for o in IB.dct3([IB.V(x[i], z, z) for i in range(n)], n)]
        for p in range(n):
            exact = sum(cq[p][i] * Fraction(float(x[i])) for i in range(n))
            bound = 2.0**-24 * float(err[p] @ np.abs(x.astype(np.float64)))
            dev = abs(float(Fraction(float(y[p])) - exact))
            assert dev <= bound, (n, p, dev, bound)
            if bound > 0:
                worst = max(worst, dev / bound)
    assert worst > 0.0
