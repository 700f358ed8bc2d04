"""CPU tests of the round-4 parity studies: the rounding certificate of the
hybrid route (tools/exp/cert_study.py) and the certified rank-1 embed (tools/exp/fastpath_study.py).
Small frames; the 4K numbers are in profiles/r04/."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools", "exp"))

from oracle import oracle as O  # noqa: E402


def _covers(H, W, seed):
    from lapack_path import photo_cover

    return {"noise": O.synth_bytes(0x5EED0001, seed, 1, H * W * 3).reshape(H, W, 3), "photo": photo_cover(H, W, seed)}


@pytest.mark.parametrize("b", [8, 16])
def test_certificate_catches_every_divergence(b):
    """The reconstruction-level certificate (interval fmaf chain) with the calibrated bound flags
    every block whose IDCT bits differ between the Jacobi and dgesdd routes; the element-level
    test at K = 256 covers every block whose f32 factors differ."""
    import cert_study as C

    for kind, cov in _covers(136, 240, 11).items():
        r2 = C.study2(cov, O.synth_bytes(0x5EED0002, 11, 1, (136 // b) * (240 // b)).reshape(136 // b, 240 // b), b, (256,))
        assert r2["K256"]["missed"] == 0, (kind, r2)
        r1 = C.study(cov, b, (256,))
        assert r1["K256"]["missed"] == 0, (kind, r1)
        # the per-route disagreement the bound must cover stays well inside it
        assert max(r1["ru_max"], r1["rv_max"], r1["rs_max"]) < 256 / 2, (kind, r1)


def test_fast_path_certificate_is_sound():
    """Every block the rank-1 fast path certifies has the dgesdd route's bytes (np.linalg.svd's
    arithmetic); the exact-path fraction is what DESIGN.md 5 reports (noise covers need the
    exact path for most blocks, camera-like covers for a minority)."""
    import fastpath_study as F

    b = 8
    covs = _covers(136, 240, 12)
    tile = O.synth_bytes(0x5EED0002, 12, 1, (136 // b) * (240 // b)).reshape(136 // b, 240 // b)
    res = {k: F.certify(c, tile, b) for k, c in covs.items()}
    for k, r in res.items():
        assert r["certified_blocks_differing_from_lapack"] == 0, (k, r)
    assert res["noise"]["frac_exact_path"] > 0.4
    assert res["photo"]["frac_exact_path"] < 0.3


@pytest.mark.parametrize("b", [4, 6, 8, 10, 12, 14, 16])
def test_rank1_prepass_bound_is_sound(b):
    """The shipped rank-1 pre-pass's bound (csrc/tmfwm_rank1.hip) restated in numpy
    (fastpath_study.certify_rank1, the IDCT's rounding through tools/exp/idct_bound.py's tables):
    every block it decides has the dgesdd route's bytes, at every slider size, with the noise and
    a binary (0 / 255) watermark; it decides most camera-like blocks under the noise watermark
    (and, at b = 8 / 16, few noise-cover blocks)."""
    import fastpath_study as F

    H, W = 272, 480
    covs = _covers(H, W, 13)
    tn = O.synth_bytes(0x5EED0002, 13, 1, (H // b) * (W // b)).reshape(H // b, W // b)
    for wm, tile in (("noise", tn), ("qr", (tn & 1) * 255)):
        res = {k: F.certify_rank1(c, tile, b) for k, c in covs.items()}
        for k, r in res.items():
            assert r["decided_blocks_differing"] == 0, (wm, k, r)
        if wm == "noise":
            assert res["photo"]["undecided"] < 0.35, res
            assert b not in (8, 16) or res["noise"]["undecided"] > 0.4, res
