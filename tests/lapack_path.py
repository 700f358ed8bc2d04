"""Reference-structured embed with LAPACK's own SVD -- test infrastructure only.

The reference computes, per b x b block of the Y plane (watermarking.py:183-210),
``U, S, Vt = np.linalg.svd(dct_block)`` -- numpy upcasts the f32 block to f64,
runs LAPACK dgesdd and casts the factors back to f32.  This
module composes the oracle's pinned stages (colour N1/N2/N9, pocketfft DCT N3,
blend + sgemm-order reconstruct N7/N8) around *numpy's LAPACK SVD itself*, i.e.
the reference's exact arithmetic, vectorised over all blocks of a frame so that
whole 1080p / 4K frames can be checked in seconds.  It is the yardstick for the
oracle's own (Jacobi) SVD at sizes the per-block golden fixtures do not reach
(tests/test_oracle_vs_lapack.py).

Only tests/ use this module.
"""
from __future__ import annotations

import numpy as np

from oracle import oracle as O


def _blocks(plane: np.ndarray, b: int) -> np.ndarray:
    H, W = plane.shape
    nbh, nbw = H // b, W // b
    return np.ascontiguousarray(plane[: nbh * b, : nbw * b].reshape(nbh, b, nbw, b).transpose(0, 2, 1, 3).reshape(-1, b, b))


def _unblocks(blocks: np.ndarray, nbh: int, nbw: int, b: int) -> np.ndarray:
    return blocks.reshape(nbh, nbw, b, b).transpose(0, 2, 1, 3).reshape(nbh * b, nbw * b)


def lapack_svd(D: np.ndarray):
    """np.linalg.svd of f32 blocks exactly as watermarking.py:195 gets it (f64 dgesdd -> f32)."""
    u, s, vt = np.linalg.svd(D.astype(np.float64))
    return u.astype(np.float32), s.astype(np.float32), vt.astype(np.float32)


def embed_lapack(rgb: np.ndarray, tile: np.ndarray, b: int, alpha: float) -> np.ndarray:
    """embed_watermark's bytes (watermarking.py:163-219) for an RGB u8 frame and a resized tile."""
    rgb = np.ascontiguousarray(rgb, np.uint8)
    H, W = rgb.shape[:2]
    nbh, nbw = H // b, W // b
    ycc = O.rgb_to_ycbcr(rgb)
    if nbh and nbw:
        D = O.dct2d_blocks(_blocks(ycc[..., 0], b))
        U, S, Vt = lapack_svd(D)
        M = O.blend_reconstruct_blocks(U, S, Vt, np.ascontiguousarray(tile, np.uint8).reshape(-1), alpha)
        ycc[: nbh * b, : nbw * b, 0] = _unblocks(O.dct2d_blocks(M, inverse=True), nbh, nbw, b)
    return O.ycbcr_to_rgb(ycc)


def sigma1_lapack(rgb: np.ndarray, b: int) -> np.ndarray:
    """f32(sigma_1) per block as extract_watermark gets it (watermarking.py:262-282)."""
    ycc = O.rgb_to_ycbcr(np.ascontiguousarray(rgb, np.uint8))
    D = O.dct2d_blocks(_blocks(ycc[..., 0], b))
    return np.linalg.svd(D.astype(np.float64), compute_uv=False)[:, 0].astype(np.float32)


def extract_lapack(wrgb: np.ndarray, orgb: np.ndarray, b: int, alpha: float) -> np.ndarray:
    """extract_watermark's tile bytes (watermarking.py:285-289, numpy-2 NEP 50 promotion)."""
    H, W = wrgb.shape[:2]
    sw, so = sigma1_lapack(wrgb, b), sigma1_lapack(orgb, b)
    e = (sw - so) / np.float32(alpha)
    return (np.clip(e.astype(np.float64), 0, 1) * 255.0).astype(np.uint8).reshape(H // b, W // b)


def photo_cover(H: int, W: int, seed: int) -> np.ndarray:
    """Camera-like synthetic cover: low-pass noise field + gradients + fine grain.

    DCT blocks of such frames have the decaying spectra of natural images (a strong
    DC term, smooth AC roll-off), unlike uniform noise (flat spectra)."""
    rng = np.random.default_rng(seed)
    f = rng.standard_normal((H // 16 + 2, W // 16 + 2, 3))
    f = np.kron(f, np.ones((16, 16, 1)))[:H, :W]
    for ax in (0, 1):  # cheap separable box blur, twice
        for _ in range(2):
            f = (np.roll(f, 5, ax) + np.roll(f, -5, ax) + f) / 3.0
    y, x = np.meshgrid(np.linspace(0, 1, H), np.linspace(0, 1, W), indexing="ij")
    img = 128 + 45 * f + 60 * (x[..., None] - 0.5) + 30 * (y[..., None] - 0.5) + rng.normal(0, 2.0, (H, W, 3))
    return np.clip(img, 0, 255).astype(np.uint8)
