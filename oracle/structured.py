"""ORACLE -- TEST INFRASTRUCTURE ONLY: the reference's COST MODEL, for bench.py's CPU baseline.

SURVEY 8(d)(i) "reference-structured mode": the same loops and library calls as the
reference, restated on numpy arrays so they run where /root/reference does not exist (the
GPU box): a Python loop over pixels with one np.dot (OpenBLAS dgemv) per pixel for each
colour conversion (/root/reference/modules/watermarking.py:43-45, :64-67), and a Python loop
over blocks with scipy.fftpack DCTs, np.linalg.svd and np.dot per block (:183-210 embed,
:262-285 extract).  It is timed, never shipped: only bench.py's cpu_baseline leg and tests/
import it.  Its arithmetic is numpy's / scipy's, i.e. the reference's own libraries, so on a
host whose OpenBLAS picks the SkylakeX kernels (this container) its bytes are the
reference's (tests/test_structured.py checks that against the golden fixtures); on another
OpenBLAS core the dgemv / sgemm FMA patterns can differ, which is why the bench reports how
many of its frames match instead of requiring it.
"""
from __future__ import annotations

import numpy as np
from scipy.fftpack import dct, idct

FWD = np.array([[0.299, 0.587, 0.114], [-0.169, -0.331, 0.5], [0.5, -0.419, -0.081]])  # :37-39
INV = np.array([[1.0, 0.0, 1.403], [1.0, -0.344, -0.714], [1.0, 1.773, 0.0]])  # :61


def ycc_of(rgb_u8: np.ndarray) -> np.ndarray:
    """:23-50 -- f32 pixels / 255, one f64 matrix-vector product per pixel, stored f32."""
    px = rgb_u8[..., :3].astype(np.float32) / 255.0
    out = np.zeros_like(px)
    h, w = px.shape[:2]
    for y in range(h):
        row, orow = px[y], out[y]
        for x in range(w):
            orow[x] = np.dot(FWD, row[x])
    out[:, :, 1:] += 0.5
    return out


def rgb_of(ycc: np.ndarray) -> np.ndarray:
    """:53-73 -- Cb, Cr - 0.5, one product per pixel, clip, * 255, truncate."""
    t = ycc.copy()
    t[:, :, 1:] -= 0.5
    out = np.zeros_like(t)
    h, w = t.shape[:2]
    for y in range(h):
        row, orow = t[y], out[y]
        for x in range(w):
            orow[x] = np.dot(INV, row[x])
    return (np.clip(out, 0, 1) * 255).astype(np.uint8)


def _dct2(blk):  # :76-78, axis 0 first
    return dct(dct(blk.T, norm="ortho").T, norm="ortho")


def _idct2(blk):  # :81-83
    return idct(idct(blk.T, norm="ortho").T, norm="ortho")


def embed(cover_u8: np.ndarray, tile_u8: np.ndarray, b: int, alpha: float) -> np.ndarray:
    """embed_watermark's body (:163-219) on an RGB uint8 array and the resized tile."""
    ycc = ycc_of(cover_u8)
    Y = ycc[:, :, 0]
    wm = tile_u8 / 255.0
    for i in range(Y.shape[0] // b):
        for j in range(Y.shape[1] // b):
            view = Y[i * b:(i + 1) * b, j * b:(j + 1) * b]
            u, s, vt = np.linalg.svd(_dct2(view), full_matrices=True)
            s[0] += alpha * wm[i, j]
            view[...] = _idct2(np.dot(u, np.dot(np.diag(s), vt)))
    return rgb_of(ycc)


def extract(marked_u8: np.ndarray, cover_u8: np.ndarray, b: int, alpha: float) -> np.ndarray:
    """extract_watermark's body (:246-292)."""
    Yw, Yo = ycc_of(marked_u8)[:, :, 0], ycc_of(cover_u8)[:, :, 0]
    nbh, nbw = Yw.shape[0] // b, Yw.shape[1] // b
    e = np.zeros((nbh, nbw))
    for i in range(nbh):
        for j in range(nbw):
            sw = np.linalg.svd(_dct2(Yw[i * b:(i + 1) * b, j * b:(j + 1) * b]), full_matrices=True)[1]
            so = np.linalg.svd(_dct2(Yo[i * b:(i + 1) * b, j * b:(j + 1) * b]), full_matrices=True)[1]
            e[i, j] = (sw[0] - so[0]) / alpha
    return (np.clip(e, 0, 1) * 255).astype(np.uint8)


def _worker(args):
    import os
    import time

    cover, tile, b, alpha = args
    t0 = time.perf_counter()
    out = embed(cover, tile, b, alpha)
    ext = extract(out, cover, b, alpha)
    return time.perf_counter() - t0, out, ext, os.getpid()


def run_pool(covers, tiles, b: int, alpha: float, procs: int):
    """Embed + extract of each (cover, tile) in a pool of `procs` single-threaded processes
    (OPENBLAS_NUM_THREADS=1 in the children): [(seconds, embedded, extracted)], wall time."""
    import multiprocessing as mp
    import os
    import time

    old = os.environ.get("OPENBLAS_NUM_THREADS")
    os.environ["OPENBLAS_NUM_THREADS"] = "1"  # read by OpenBLAS when a child imports numpy
    try:
        ctx = mp.get_context("spawn")
        t0 = time.perf_counter()
        with ctx.Pool(procs) as pool:
            res = pool.map(_worker, [(c, t, b, alpha) for c, t in zip(covers, tiles)], chunksize=1)
        wall = time.perf_counter() - t0
    finally:
        if old is None:
            os.environ.pop("OPENBLAS_NUM_THREADS", None)
        else:
            os.environ["OPENBLAS_NUM_THREADS"] = old
    return [(r[0], r[1], r[2]) for r in res], wall
