"""The byte certificate's one assumption, measured directly.

The hybrid route's certificate (thatsmyface_amd/csrc/tmfwm_blocks.h `kCertScale`, oracle
tmfwm_cert.cpp) assumes that for a block that passes the conditioning test, LAPACK's f64 factors
(dgesdd as np.linalg.svd runs it at watermarking.py:195) and the Jacobi route's lie within
    E_k = K 2^-53 sigma_1 / g_k   per element of U[:, k] and V[:, k],
    E_s = K 2^-53 sigma_1         per singular value,
K = 256.  This module measures that quantity itself -- the direct Jacobi-vs-dgesdd difference,
orc_svd_blocks_f64 against orc_lp_svd_blocks_f64, sign-aligned per triplet -- in those units, on
seeded cover classes: pixel-derived DCT blocks (noise, camera-like, QR-module covers, flat + eps,
gradients) and DCT-domain constructions (near ties just above the 2^-20 conditioning cut, graded
spectra, clusters, rank-deficient blocks).  Test infrastructure: imports the oracle only.
"""
from __future__ import annotations

import os
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_ROOT = os.path.dirname(_HERE)
for _p in (_ROOT, _HERE):
    if _p not in sys.path:
        sys.path.insert(0, _p)

from oracle import oracle as O  # noqa: E402
from lapack_path import _blocks, photo_cover  # noqa: E402

EPS = 2.0 ** -53
K_CERT = 256  # kCertScale = 2^-45 = K 2^-53


def lapack_f64(D: np.ndarray):
    """np.linalg.svd's f64 factors on the restated dgesdd route: U (u[r][k]), S, V (v[r][k])."""
    import ctypes
    D = np.ascontiguousarray(D, np.float32)
    nb, b = D.shape[0], D.shape[-1]
    U = np.empty(D.shape, np.float64)
    Vt = np.empty(D.shape, np.float64)
    S = np.empty((nb, b), np.float64)
    f64p = ctypes.POINTER(ctypes.c_double)
    f32p = ctypes.POINTER(ctypes.c_float)
    fn = O.lib().orc_lp_svd_blocks_f64
    fn.restype = ctypes.c_int
    rc = fn(D.ctypes.data_as(f32p), ctypes.c_int64(nb), b, U.ctypes.data_as(f64p), S.ctypes.data_as(f64p),
            Vt.ctypes.data_as(f64p), O.default_threads())
    if rc:
        raise ValueError("lapack restatement did not converge")
    return U, S, np.swapaxes(Vt, 1, 2)


def ratios(D: np.ndarray):
    """Per block: (certified, ru, rv, rs) -- `certified` = the device's cert condition (non-zero,
    not flat, not flagged); ru / rv = max over output triplets k and rows of |F_J - F_L| in units of
    2^-53 s1 / g_k; rs = max over every k of |sigma_J - sigma_L| in units of 2^-53 s1.  g_k and the
    flag as tmfwm_blocks.h computes them from the Jacobi route's sigmas."""
    D = np.ascontiguousarray(D, np.float32)
    n, b = D.shape[0], D.shape[-1]
    Uj, sj, Vj = O.svd_blocks_f64(D)
    Ul, sl, Vl = lapack_f64(D)
    s1 = sj.max(axis=1)
    d = np.abs(sj[:, :, None] - sj[:, None, :])
    d[:, np.arange(b), np.arange(b)] = np.inf
    g = np.minimum(sj, d.min(axis=2))
    out = sj.astype(np.float32) != 0
    m = np.where(out, g, np.inf).min(axis=1)
    m = np.minimum(m, s1)
    flag = m * 2.0 ** 20 < s1
    off = D.reshape(n, -1)[:, 1:]
    flat = ~np.any(off != 0, axis=1)
    cert = (s1 > 0) & ~flat & ~flag
    sg = np.sign(np.einsum("nrk,nrk->nk", Uj, Ul))
    sg[sg == 0] = 1
    du = np.abs(Uj - Ul * sg[:, None, :]).max(axis=1)
    dv = np.abs(Vj - Vl * sg[:, None, :]).max(axis=1)
    with np.errstate(divide="ignore", invalid="ignore"):
        ek = EPS * s1[:, None] / g
        ru = np.where(out & cert[:, None], du / ek, 0.0).max(axis=1)
        rv = np.where(out & cert[:, None], dv / ek, 0.0).max(axis=1)
        rs = np.where(cert[:, None], np.abs(sj - sl) / (EPS * s1[:, None]), 0.0).max(axis=1)
    return cert, ru, rv, rs


# The rank-1 pre-pass's LAPACK constants (csrc/tmfwm_rank1.hip: gamma' = 2^-40 s1, the top pair
# within 1024 2^-53 s1 / (s1 - s2)), measured by tools/exp/lapack_bounds.py
RESID_UNITS = 8192
PAIR_UNITS = 1024


def residual_units(D, U, S, V):
    """max_ij |(U S V^T)_ij - D_ij| / (2^-53 sigma_1) per block, in extended precision."""
    Ul, Sl, Vl = (x.astype(np.longdouble) for x in (U, S, V))
    M = np.einsum("nik,nk,njk->nij", Ul, Sl, Vl)
    r = np.abs(M - D.astype(np.longdouble)).reshape(len(D), -1).max(axis=1).astype(np.float64)
    s1 = S.max(axis=1)
    with np.errstate(divide="ignore", invalid="ignore"):
        return np.where(s1 > 0, r / (EPS * s1), 0.0)


def top_pair_units(D, S_l, U_l, V_l):
    """max |F_J - F_L| over the top triplet's elements, units 2^-53 s1 / (s1 - s2)."""
    Uj, sj, Vj = O.svd_blocks_f64(D)
    n = len(D)
    kj = np.argmax(sj, axis=1)
    kl = np.argmax(S_l, axis=1)
    uj, vj = Uj[np.arange(n), :, kj], Vj[np.arange(n), :, kj]
    ul, vl = U_l[np.arange(n), :, kl], V_l[np.arange(n), :, kl]
    sg = np.sign(np.einsum("nr,nr->n", uj, ul))
    sg[sg == 0] = 1
    d = np.maximum(np.abs(uj - ul * sg[:, None]).max(axis=1), np.abs(vj - vl * sg[:, None]).max(axis=1))
    s = np.sort(sj, axis=1)
    s1, s2 = s[:, -1], s[:, -2]
    ok = s1 > s2
    with np.errstate(divide="ignore", invalid="ignore"):
        return ok, np.where(ok, d / (EPS * s1 / np.where(ok, s1 - s2, 1.0)), 0.0)



# ---- cover classes ----------------------------------------------------------------------

def _rand_orth(rng, n, b):
    q, r = np.linalg.qr(rng.standard_normal((n, b, b)))
    return q * np.sign(np.einsum("nii->ni", r))[:, None, :]


def _from_sigmas(rng, sig):
    n, b = sig.shape
    Q1, Q2 = _rand_orth(rng, n, b), _rand_orth(rng, n, b)
    return np.einsum("nik,nk,njk->nij", Q1, sig, Q2).astype(np.float32)


def _luma_blocks(rgb: np.ndarray, b: int) -> np.ndarray:
    return O.dct2d_blocks(_blocks(O.rgb_to_ycbcr(rgb)[..., 0], b))


def _qr_cover(rng, H, W):
    """Covers made of QR symbols (the app's watermark as an image): modules of random integer and
    non-integer pixel pitch at random offsets, some with a camera-like blur and grain."""
    from thatsmyface_amd import qrcode_generator as qg
    img = np.full((H, W), 255.0)
    y = 0
    while y < H:
        x = 0
        pitch = rng.uniform(1.3, 11.0)
        mods = qg.qr_matrix(rng.integers(0, 256, int(rng.integers(4, 60))).astype(np.uint8).tobytes())
        side = int(np.ceil((mods.shape[0] + 8) * pitch))
        while x < W:
            idx = ((np.arange(side) / pitch).astype(int) - 4)
            ok = (idx >= 0) & (idx < mods.shape[0])
            tile = np.full((side, side), 255.0)
            ii = np.clip(idx, 0, mods.shape[0] - 1)
            sub = np.where(mods[np.ix_(ii, ii)] != 0, 0.0, 255.0)
            tile[np.ix_(ok, ok)] = sub[np.ix_(ok, ok)]
            h, w = min(side, H - y), min(side, W - x)
            img[y:y + h, x:x + w] = tile[:h, :w]
            x += side + int(rng.integers(0, 9))
        y += side + int(rng.integers(0, 9))
    if rng.random() < 0.5:
        for ax in (0, 1):
            img = (np.roll(img, 1, ax) + np.roll(img, -1, ax) + 2 * img) / 4.0
        img = img + rng.normal(0, 1.5, img.shape)
    g = np.clip(img, 0, 255).astype(np.uint8)
    tint = rng.integers(-20, 21, 3)
    return np.clip(g[..., None].astype(int) + tint, 0, 255).astype(np.uint8)


def _flat_eps_cover(rng, H, W):
    """Flat colour with +-1..2 changes on a fraction of the pixels (near-flat DCT blocks: one
    dominant sigma, the others ~1e-3 of it; sparse changes leave rank-deficient blocks, which the
    conditioning test sends to the dgesdd route)."""
    base = rng.integers(0, 256, 3)
    img = np.broadcast_to(base, (H, W, 3)).astype(int).copy()
    mask = rng.random((H, W)) < rng.uniform(0.3, 1.0)
    img[mask] += rng.integers(-2, 3, (int(mask.sum()), 3))
    return np.clip(img, 0, 255).astype(np.uint8)


def _gradient_cover(rng, H, W):
    """Smooth ramps and steps (graphics): low-rank blocks with exact structural zeros."""
    y, x = np.meshgrid(np.arange(H), np.arange(W), indexing="ij")
    img = np.zeros((H, W, 3))
    for c in range(3):
        a, bb, cc = rng.uniform(-0.6, 0.6, 3)
        img[..., c] = 128 + a * x + bb * y + cc * ((x // 37 + y // 23) % 2) * 40
    return np.clip(img, 0, 255).astype(np.uint8)


def pixel_class(kind: str, b: int, seed: int, H: int = 544, W: int = 960) -> np.ndarray:
    rng = np.random.default_rng(seed)
    if kind == "noise":
        rgb = O.synth_bytes(0x5EED0001 ^ seed, 0, 1, H * W * 3).reshape(H, W, 3)
    elif kind == "photo":
        rgb = photo_cover(H, W, seed)
    elif kind == "qr":
        rgb = _qr_cover(rng, H, W)
    elif kind == "flat_eps":
        rgb = _flat_eps_cover(rng, H, W)
    elif kind == "gradient":
        rgb = _gradient_cover(rng, H, W)
    else:
        raise ValueError(kind)
    return _luma_blocks(rgb, b)


def dct_class(kind: str, b: int, n: int, seed: int) -> np.ndarray:
    """DCT-domain constructions aimed at the bound (f32 blocks D = Q1 diag(s) Q2^T)."""
    rng = np.random.default_rng(seed)
    s1 = np.exp(rng.uniform(np.log(0.05), np.log(40.0), n))  # the DCT's sigma_1 range (ortho, b <= 16)
    if kind == "near_tie":
        # one pair separated by 1..16 x the 2^-20 s1 cut, the rest random
        sig = np.sort(rng.uniform(0.02, 1.0, (n, b)), axis=1)[:, ::-1].copy()
        k = rng.integers(0, b - 1, n)
        gap = 2.0 ** -20 * np.exp(rng.uniform(0, np.log(16.0), n))
        sig[np.arange(n), k + 1] = sig[np.arange(n), k] - gap
        sig = np.sort(sig, axis=1)[:, ::-1]
    elif kind == "graded":
        # sigma_k = 2^-e_k, e_k spread over [0, E], E up to 19 (the smallest above the cut)
        E = rng.uniform(2.0, 19.0, n)
        e = np.sort(rng.uniform(0, 1, (n, b)), axis=1) * E[:, None]
        e[:, 0] = 0.0
        sig = 2.0 ** -e
    elif kind == "graded_diag":
        # graded, unrotated or rotated on one side only (structured zeros in D)
        E = rng.uniform(2.0, 19.0, n)
        sig = 2.0 ** -(np.linspace(0, 1, b)[None, :] * E[:, None])
        D = np.zeros((n, b, b))
        perm = np.argsort(rng.random((n, b)), axis=1)
        D[np.arange(n)[:, None], np.arange(b)[None, :], perm] = sig
        half = rng.random(n) < 0.5
        Q = _rand_orth(rng, n, b)
        D[half] = np.einsum("nik,nkj->nij", Q[half], D[half])
        return (D * s1[:, None, None]).astype(np.float32)
    elif kind == "cluster":
        # three to b/2 sigmas in a cluster with gaps 1..64 x the cut
        sig = np.sort(rng.uniform(0.02, 1.0, (n, b)), axis=1)[:, ::-1].copy()
        for i in range(n):
            c = int(rng.integers(3, b // 2 + 2))
            k0 = int(rng.integers(0, b - c + 1))
            steps = 2.0 ** -20 * np.exp(rng.uniform(0, np.log(64.0), c - 1))
            sig[i, k0 + 1:k0 + c] = sig[i, k0] - np.cumsum(steps)
        sig = np.sort(np.abs(sig), axis=1)[:, ::-1]
    elif kind == "rank_def":
        # rank r < b: exact zeros through f32 rounding where they survive (else the flag fires)
        sig = np.sort(rng.uniform(0.02, 1.0, (n, b)), axis=1)[:, ::-1].copy()
        r = rng.integers(1, b, n)
        sig[np.arange(b)[None, :] >= r[:, None]] = 0.0
        D = _from_sigmas(rng, sig * s1[:, None]).astype(np.float64)
        # most of them with structurally zero columns (exact zeros of the Jacobi route's sigmas:
        # a zero column is never rotated, so those triplets do not reach the output) or rows
        z = rng.random(n)
        for i in np.nonzero(z < 0.8)[0]:
            k = int(rng.integers(1, b))
            if z[i] < 0.6:
                D[i, :, rng.permutation(b)[:k]] = 0.0
            else:
                D[i, rng.permutation(b)[:k], :] = 0.0
        return D.astype(np.float32)
    elif kind == "dc_dominant":
        # the bench's noise shape pushed further: a huge D[0][0], tiny AC (flat + eps in DCT terms)
        D = rng.standard_normal((n, b, b)) * (2.0 ** rng.uniform(-19, -4, n))[:, None, None]
        D[:, 0, 0] = 1.0
        return (D * s1[:, None, None]).astype(np.float32)
    else:
        raise ValueError(kind)
    return _from_sigmas(rng, sig * s1[:, None])


PIXEL_KINDS = ("noise", "photo", "qr", "flat_eps", "gradient")
DCT_KINDS = ("near_tie", "graded", "graded_diag", "cluster", "rank_def", "dc_dominant")


def corpus(kind: str, b: int, seed: int, n: int = 20000) -> np.ndarray:
    if kind in PIXEL_KINDS:
        return pixel_class(kind, b, seed)
    return dct_class(kind, b, n, seed)
