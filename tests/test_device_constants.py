"""Constants and short formulas of the device code checked exhaustively on the CPU (the GPU
suite checks the kernels that use them: test_colour_tables_exhaustive_gpu)."""
import os
import re
from fractions import Fraction

import numpy as np

HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "thatsmyface_amd", "csrc", "tmfwm_device.h")


def _rn32(v: Fraction) -> np.float32:
    """round-to-nearest-even of an exact rational to float32"""
    f = np.float32(float(v))
    cands = sorted({f, np.nextafter(f, np.float32(-np.inf)), np.nextafter(f, np.float32(np.inf))}, key=float)
    best = min(cands, key=lambda c: (abs(Fraction(float(c)) - v), int(np.float32(c).view(np.uint32)) & 1))
    return np.float32(best)


def test_unit_from_u8_two_ops_is_the_ieee_divide():
    """unit_from_u8: fma(x, Hi, x * Lo) == f32(v) / 255.0f for every byte (watermarking.py:29)."""
    src = open(HDR).read()
    hi = np.float32(re.search(r"kUnitHi = ([-0-9.e]+)f;", src).group(1))
    lo = np.float32(re.search(r"kUnitLo = ([-0-9.e]+)f;", src).group(1))
    assert hi == np.float32(1.0 / 255.0) and lo == np.float32(1.0 / 255.0 - float(hi))
    for v in range(256):
        x = np.float32(v)
        p = np.float32(x * lo)  # the f32 multiply
        got = _rn32(Fraction(float(x)) * Fraction(float(hi)) + Fraction(float(p)))  # the fma: one rounding
        assert got == x / np.float32(255.0), v
