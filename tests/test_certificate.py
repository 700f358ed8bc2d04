"""CPU tests of the hybrid route's byte certificate (oracle/tmfwm_cert.cpp orc_cert_block, the
restatement of the device's in thatsmyface_amd/csrc/tmfwm_blocks.h).

The certificate carries each block's factor uncertainty (K = 256 units of 2^-53 sigma_1 / g_k) as
f32 intervals through the reconstruction's fmaf chain, pocketfft's IDCT and the inverse colour,
and sends a block to the dgesdd route unless every byte is decided.  Pinned here:
  * the interval IDCT on point intervals is the IDCT, bit for bit (the interval passes restate
    pocketfft's op order, watermarking.py:204);
  * the exact cases: zero and flat (DC-only) blocks are certain, alpha < 0 pushing S'[0] below 0
    is not;
  * on camera-like covers with the app's binary (QR) watermark -- the hardest case for the
    certificate -- the oracle's hybrid route gives numpy's own dgesdd bytes (tests/lapack_path.py,
    watermarking.py:195-216), and on the bench's noise covers it decides >= 99.9 % of blocks.
"""
import ctypes

import numpy as np
import pytest

from oracle import oracle as O
from lapack_path import embed_lapack, photo_cover
from golden.gen_golden import wmark


def _f32(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _f64(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


@pytest.mark.parametrize("b", [4, 6, 8, 10, 12, 14, 16])
def test_interval_idct_on_points_is_the_idct(b):
    rng = np.random.default_rng(100 + b)
    blk = (rng.standard_normal((16, b, b)) * 60.0).astype(np.float32)
    want = O.dct2d_blocks(blk, inverse=True)
    for i in range(blk.shape[0]):
        x = np.ascontiguousarray(blk[i])
        O.lib().orc_cert_idct_point(_f32(x), b)
        assert not np.isnan(x).any(), "a point interval widened"
        assert np.array_equal(x.view(np.uint32), want[i].view(np.uint32)), i


def _cert(D, w, alpha, cb=None, cr=None):
    """orc_cert_block on one b x b DCT block with the Jacobi route's f64 factors: 0 = the bytes
    are decided, 1 = the dgesdd route."""
    b = D.shape[-1]
    D = np.ascontiguousarray(D, np.float32)
    U, S, V = O.svd_blocks_f64(D[None])
    U, S, V = np.ascontiguousarray(U[0]), np.ascontiguousarray(S[0]), np.ascontiguousarray(V[0])
    cb = np.full((b, b), 0.5, np.float32) if cb is None else np.ascontiguousarray(cb, np.float32)
    cr = np.full((b, b), 0.5, np.float32) if cr is None else np.ascontiguousarray(cr, np.float32)
    st = np.zeros(8, np.int64)
    return O.lib().orc_cert_block(_f32(D), _f64(U), _f64(S), _f64(V), b, w, float(alpha), _f32(cb), _f32(cr),
                                  st.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)))


@pytest.mark.parametrize("b", [8, 16])
def test_exact_cases(b):
    zero = np.zeros((b, b), np.float32)
    assert _cert(zero, 200, 0.1) == 0
    flat = np.zeros((b, b), np.float32)
    flat[0, 0] = 3.25
    assert _cert(flat, 200, 0.1) == 0
    rng = np.random.default_rng(b)
    D = O.dct2d_blocks((rng.random((b, b)) * 0.8 + 0.1).astype(np.float32))
    assert _cert(D, 255, -1e6) == 1  # S'[0] < 0: outside the certificate's sign rule


@pytest.mark.parametrize("b", [8, 16])
def test_camera_like_qr_watermark_matches_numpy(b):
    H, W = 144, 256
    cov = photo_cover(H, W, 21)
    tile = wmark("qr", H // b, W // b, 5)
    for alpha in (0.01, 0.1, 0.2):
        st = {}
        got = O.embed_frame(cov, tile, b, alpha, route="hybrid", stats=st)
        assert np.array_equal(got, embed_lapack(cov, tile, b, alpha)), alpha
        assert st["fallback_blocks"] < (H // b) * (W // b)  # the certificate decides blocks at all


def test_noise_covers_decided():
    b, H, W = 8, 272, 480
    rng = np.random.default_rng(7)
    cov = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    tile = rng.integers(0, 256, (H // b, W // b), dtype=np.uint8)
    st = {}
    O.embed_frame(cov, tile, b, 0.1, route="hybrid", stats=st)
    assert st["fallback_blocks"] <= 0.001 * (H // b) * (W // b) + 1, st


def test_device_and_oracle_share_the_bound():
    """The device certificate (tmfwm_blocks.h) and its oracle restatement (tmfwm_cert.cpp) use the
    same K (kCertScale = K 2^-53 = 2^-45) and hold E_k as f32(tE / g_k) on both sides."""
    import os
    import re

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    dev = open(os.path.join(root, "thatsmyface_amd", "csrc", "tmfwm_blocks.h")).read()
    orc = open(os.path.join(root, "oracle", "tmfwm_cert.cpp")).read()
    rx = re.compile(r"kCertScale\s*=\s*([0-9a-fx.p+-]+)")
    assert rx.search(dev).group(1) == rx.search(orc).group(1) == "0x1p-45"
    assert "(float)(tE / gk[k])" in dev
    assert re.search(r"\(double\)\(float\)\(t / g\)", orc)
