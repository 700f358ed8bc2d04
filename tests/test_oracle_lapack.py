"""Pin the oracle's restatement of the reference's SVD (oracle/tmfwm_lapack.c).

The reference calls np.linalg.svd on float32 blocks (watermarking.py:195, :279-282):
numpy 2.2.6 -> f64 LAPACK dgesdd from scipy-openblas64 0.3.29 (LAPACK 3.12.0 Fortran
plus the OpenBLAS kernels of the CPU's DYNAMIC_ARCH core).  The restatement is pinned
bit for bit here against numpy itself (f64 factors and the f32 factors the reference
consumes) and against the library's own BLAS entry points.  The OpenBLAS kernels it
restates are the "SkylakeX" core's, the one this container's CPU selects; on another
core numpy's own bits differ, so these tests skip there.
"""
import ctypes
import glob
import os

import numpy as np
import pytest

from oracle import oracle as O


def _openblas():
    import numpy

    libs = glob.glob(os.path.join(os.path.dirname(numpy.__file__), os.pardir, "numpy.libs", "libscipy_openblas64_*.so"))
    if not libs:
        return None, None
    L = ctypes.CDLL(libs[0])
    f = L.scipy_openblas_get_corename64_
    f.restype = ctypes.c_char_p
    return L, f().decode()


_LIB, _CORE = _openblas()
needs_skylakex = pytest.mark.skipif(_CORE != "SkylakeX", reason=f"OpenBLAS core {_CORE!r}: the restated kernels are SkylakeX's")


def _same(a, b):
    return np.array_equal(np.ascontiguousarray(a).view(np.uint64), np.ascontiguousarray(b).view(np.uint64))


@needs_skylakex
def test_dnrm2_x87_vs_openblas():
    """OpenBLAS dnrm2 (dlarfg's column norm): x87 extended, four accumulators."""
    fn = _LIB.scipy_dnrm2_64_
    fn.restype = ctypes.c_double
    rng = np.random.default_rng(5)
    for inc in (1, 3, 16):
        for n in range(0, 41):
            for t in range(200):
                x = rng.standard_normal(max(n * inc, 1)) * 10.0 ** rng.integers(-4, 5)
                got = O.lp_dnrm2(x[: n * inc], inc)
                ref = fn(ctypes.byref(ctypes.c_int64(n)), x.ctypes.data_as(ctypes.c_void_p), ctypes.byref(ctypes.c_int64(inc)))
                assert _same(np.float64(got), np.float64(ref)), (n, inc, t)


def _matrices(n, rng):
    """Dense random, f32-representable, sparse rank-1, single entries, small integers,
    binary 0/255 (QR-like), identities / permutations / repeated diagonals (exact ties)."""
    yield np.eye(n)
    yield -np.eye(n)
    yield np.diag(rng.permutation(n).astype(float))
    yield np.diag(np.repeat([3.0, 1.0], (n + 1) // 2)[:n])
    yield np.eye(n)[rng.permutation(n)] * 2.0
    yield np.zeros((n, n))
    for _ in range(40):
        yield rng.standard_normal((n, n))
        yield rng.standard_normal((n, n)).astype(np.float32).astype(np.float64)
        a = np.outer(rng.standard_normal(n), rng.standard_normal(n))
        a[rng.random((n, n)) < 0.1] = 0
        yield a
        a = np.zeros((n, n))
        k = rng.integers(1, n + 1)
        a[rng.integers(0, n, k), rng.integers(0, n, k)] = rng.choice([-2.0, -1.0, 0.5, 1.0, 2.0], k)
        yield a
        yield rng.integers(-2, 3, (n, n)).astype(np.float64)
        yield rng.integers(0, 2, (n, n)).astype(np.float64) * 255
        yield np.tile(rng.standard_normal(n), (n, 1))


@needs_skylakex
@pytest.mark.parametrize("n", list(range(1, 17)))
def test_svd_f64_bit_identical_to_numpy(n):
    rng = np.random.default_rng(100 + n)
    for k, a in enumerate(_matrices(n, rng)):
        u, s, vt = O.lp_svd(a)
        U, S, VT = np.linalg.svd(a)
        assert _same(s, S) and _same(u, U) and _same(vt, VT), (n, k)


def _cover_blocks(kind, b, H=272, W=480, seed=11):
    from golden.gen_golden import cover
    from lapack_path import _blocks, photo_cover

    cov = photo_cover(H, W, seed) if kind == "photo" else cover(kind, H, W, seed)
    return O.dct2d_blocks(_blocks(O.rgb_to_ycbcr(cov)[..., 0], b))


KINDS = ["noise", "photo", "smooth", "blocky", "qr", "diagonal", "flat", "black"]


@needs_skylakex
@pytest.mark.parametrize("b", [4, 6, 8, 10, 12, 14, 16])
def test_svd_blocks_f32_bit_identical_to_numpy(b):
    """The factors the reference consumes: np.linalg.svd of the float32 DCT blocks."""
    for kind in KINDS:
        D = _cover_blocks(kind, b)
        U, S, Vt = O.lp_svd_blocks(D)
        u, s, vt = np.linalg.svd(D)
        for x, y in ((U, u), (S, s), (Vt, vt)):
            assert np.array_equal(x.view(np.uint32), y.view(np.uint32)), (b, kind)


@pytest.mark.parametrize("b", [8, 12, 16])
def test_hybrid_flag_covers_every_divergent_block(b):
    """Where the Jacobi route's reconstructed block differs from the dgesdd route's at
    all (any bit of the IDCT output, a stricter test than the bytes), the hybrid
    route's conditioning test must have flagged the block."""
    from golden.gen_golden import wmark

    for kind in ["noise", "photo", "smooth", "blocky", "qr", "diagonal"]:
        D = _cover_blocks(kind, b)
        tile = wmark("qr", 272 // b, 480 // b, 3).reshape(-1)
        J = O.svd_blocks(D)[:3]
        Lp = O.lp_svd_blocks(D)
        Yj, Yl = (O.dct2d_blocks(O.blend_reconstruct_blocks(*f, tile, 0.1), inverse=True) for f in (J, Lp))
        diff = ~np.all((Yj.view(np.uint32) == Yl.view(np.uint32)).reshape(len(D), -1), axis=1)
        _, sig, _ = O.svd_blocks_f64(D)
        flags = np.array([O.svd_flag(s) for s in sig])
        assert not (diff & ~flags).any(), (b, kind, int((diff & ~flags).sum()))


def test_hybrid_flag_rates():
    """The dgesdd route is the exception on natural-looking covers: < 0.1 % of blocks on
    uniform-noise covers (the bench workload), < 2 % on camera-like covers."""
    for kind, cap in (("noise", 1e-3), ("photo", 2e-2)):
        for b in (8, 16):
            _, sig, _ = O.svd_blocks_f64(_cover_blocks(kind, b, 544, 960))
            rate = np.mean([O.svd_flag(s) for s in sig])
            assert rate <= cap, (kind, b, rate)


@pytest.mark.parametrize("b,frames", [(8, 4), (16, 1)])
def test_hybrid_flag_margin_at_scale(b, frames):
    """The conditioning flag's margin over whole 4K frames: per kind,
    `frames` noise frames (the bench's generator) and `frames` camera-like covers -- at b = 8
    1.04 M blocks.  Unflagged blocks whose output bytes differ between the Jacobi and dgesdd
    routes: must be 0.  Unflagged blocks whose IDCT output *bits* differ (a factor element
    rounded to the other side of an f32 boundary; no byte changed) are counted: measured
    (tools/exp/flag_margin.py) 1 of 1,036,800 at b = 8 and 20 of 259,200 at
    b = 16, at amplifications sigma_1 / m of 6e3 and <= 2.4e5 -- rounding coincidences, not
    conditioning: the flag (2^20 = 1.05e6) is never what separates them."""
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "exp"))
    import flag_margin as FM

    H, W = 2160, 3840
    bytediff = ydiff = blocks = 0
    for kind in ("noise", "photo"):
        for f in range(frames):
            from lapack_path import photo_cover

            cov = (O.synth_bytes(0x5EED0001, f, 1, H * W * 3).reshape(H, W, 3) if kind == "noise"
                   else photo_cover(H, W, 100 + f))
            tile = O.synth_bytes(0x5EED0002, f, 1, (H // b) * (W // b)).reshape(H // b, W // b)
            nb, flags, yd, bd, _ = FM.frame_stats(cov, tile, b)
            blocks += nb
            bytediff += int((bd & ~flags).sum())
            ydiff += int((yd & ~flags).sum())
    assert bytediff == 0
    assert ydiff <= 1e-4 * blocks, (ydiff, blocks)
