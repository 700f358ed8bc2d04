"""ORACLE -- test infrastructure only.

ctypes wrapper around ``oracle/_build/libtmfwm_oracle.so`` (the plain-C
restatement in ``tmfwm_oracle.c`` of /root/reference/modules/watermarking.py).
Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg import this module, and only as the checker / CPU
baseline.  The product package ``thatsmyface_amd`` never imports it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libtmfwm_oracle.so")
_lib = None
# gfx950 v_rsq_f32 truth table (phase 1 of the Jacobi route, tmfwm_oracle.c rsq_hw): deltas in
# ulps against f32(1 / sqrt(f64(x))) on the 2^24 canonical inputs, measured on the GPU by
# tools/trans_table.py
_TRANS_NPZ = os.path.join(os.path.dirname(_HERE), "tests", "golden", "gfx950_trans_delta.npz")
_rsq_delta = None

_u8p = ctypes.POINTER(ctypes.c_uint8)
_f32p = ctypes.POINTER(ctypes.c_float)
_i32p = ctypes.POINTER(ctypes.c_int32)
_f64p = ctypes.POINTER(ctypes.c_double)


def build(force: bool = False) -> str:
    """Compile the oracle with its Makefile (gcc); returns the .so path."""
    if force or not os.path.exists(_LIB_PATH) or (
        os.path.getmtime(_LIB_PATH) < max(os.path.getmtime(os.path.join(_HERE, f)) for f in ("tmfwm_oracle.c", "tmfwm_lapack.c", "tmfwm_cert.cpp", "orc_plan.h"))
    ):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_LIB_PATH)
        I64, I32, D = ctypes.c_int64, ctypes.c_int, ctypes.c_double
        sig = {
            "orc_rgb_to_ycbcr": (None, [_u8p, I64, _f32p]),
            "orc_ycbcr_to_rgb": (None, [_f32p, I64, _u8p]),
            "orc_rgb_to_ycbcr_f32": (None, [_f32p, I64, _f32p]),
            "orc_ycbcr_to_rgb_f64": (None, [ctypes.c_void_p, I64, _u8p]),
            "orc_ycbcr_to_rgb_f16": (None, [ctypes.c_void_p, I64, _u8p]),
            "orc_dct2d_blocks": (None, [_f32p, I64, I32, I32]),
            "orc_dct_rows": (None, [_f32p, I64, I32, I32]),
            "orc_svd_blocks": (I32, [_f32p, I64, I32, _f32p, _f32p, _f32p, _i32p]),
            "orc_sigma1_block": (ctypes.c_float, [_f32p, I32]),
            "orc_blend_reconstruct": (None, [_f32p, _f32p, _f32p, I32, ctypes.c_uint8, D, _f32p]),
            "orc_blend_reconstruct_blocks": (None, [_f32p, _f32p, _f32p, I64, I32, _u8p, D, _f32p]),
            "orc_gather_blocks": (None, [_f32p, I32, I32, I32, _f32p]),
            "orc_scatter_blocks": (None, [_f32p, I32, I32, I32, _f32p]),
            "orc_embed_frame": (I32, [_u8p, I32, I32, _u8p, I32, D, _u8p, I32]),
            "orc_extract_frame": (I32, [_u8p, _u8p, I32, I32, I32, D, _u8p, I32]),
            "orc_embed_batch": (I32, [_u8p, I64, I32, I32, _u8p, I32, D, _u8p, I32]),
            "orc_extract_batch": (I32, [_u8p, _u8p, I64, I32, I32, I32, D, _u8p, I32]),
            "orc_synth_bytes": (None, [ctypes.c_uint64, I64, I64, I64, _u8p]),
            "orc_resize_lanczos": (I32, [_u8p, I32, I32, I32, I32, _u8p, I32]),
            "orc_prepare_tile": (I32, [_u8p, I32, I32, I32, I32, I32, _u8p]),
            "orc_embed_frame_mode": (I32, [_u8p, I32, I32, _u8p, I32, D, _u8p, I32, I32, ctypes.POINTER(I64)]),
            "orc_extract_frame_mode": (I32, [_u8p, _u8p, I32, I32, I32, D, _u8p, I32, I32]),
            "orc_svd_flag": (I32, [_f64p, I32]),
            "orc_cert_block": (I32, [_f32p, _f64p, _f64p, _f64p, I32, ctypes.c_uint8, D, _f32p, _f32p, ctypes.POINTER(I64)]),
            "orc_cert_idct_point": (None, [_f32p, I32]),
            "orc_rsq_hw": (ctypes.c_float, [ctypes.c_float]),
            "orc_svd_blocks_f64": (None, [_f32p, I64, I32, _f64p, _f64p, _f64p, I32]),
            "orc_lp_dnrm2": (D, [I32, _f64p, I32]),
            "orc_lp_svd_blocks": (I32, [_f32p, I64, I32, _f32p, _f32p, _f32p, I32]),
            "orc_lp_svd": (I32, [_f64p, I32, _f64p, _f64p, _f64p]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        global _rsq_delta
        with np.load(_TRANS_NPZ) as z:
            _rsq_delta = np.ascontiguousarray(z["rsq"], dtype=np.int8)
        if _rsq_delta.shape != (1 << 24,):
            raise RuntimeError(f"{_TRANS_NPZ}: rsq table has shape {_rsq_delta.shape}")
        L.orc_set_rsq_table.restype = None
        L.orc_set_rsq_table.argtypes = [ctypes.c_void_p]
        L.orc_set_rsq_table(_rsq_delta.ctypes.data)
        _lib = L
    return _lib


def _p(a: np.ndarray, typ):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(typ)


def default_threads() -> int:
    try:
        return max(1, len(os.sched_getaffinity(0)))
    except AttributeError:  # pragma: no cover
        return os.cpu_count() or 1


# --- stages ---------------------------------------------------------------
def rgb_to_ycbcr(rgb: np.ndarray) -> np.ndarray:
    """watermarking.py:23-50.  uint8 pixels, or any other numeric array through the
    reference's own cast np.array(img, dtype=np.float32) (:29)."""
    rgb = np.asarray(rgb)
    out = np.empty(rgb.shape[:-1] + (3,), np.float32)
    if rgb.dtype == np.uint8:
        rgb = np.ascontiguousarray(rgb)
        lib().orc_rgb_to_ycbcr(_p(rgb, _u8p), rgb.size // 3, _p(out, _f32p))
    else:
        rgb = np.ascontiguousarray(rgb, dtype=np.float32)
        lib().orc_rgb_to_ycbcr_f32(_p(rgb, _f32p), rgb.size // 3, _p(out, _f32p))
    return out


def ycbcr_to_rgb(ycc: np.ndarray) -> np.ndarray:
    """watermarking.py:53-73 in the input's own float type (float16 / 32 / 64)."""
    ycc = np.asarray(ycc)
    out = np.empty(ycc.shape, np.uint8)
    if ycc.dtype == np.float64 or ycc.dtype == np.float16:
        ycc = np.ascontiguousarray(ycc)
        fn = lib().orc_ycbcr_to_rgb_f64 if ycc.dtype == np.float64 else lib().orc_ycbcr_to_rgb_f16
        fn(ycc.ctypes.data, ycc.size // 3, _p(out, _u8p))
    else:
        if ycc.dtype != np.float32:
            raise TypeError(f"ycbcr_to_rgb takes float16/32/64 arrays, got {ycc.dtype}")
        ycc = np.ascontiguousarray(ycc)
        lib().orc_ycbcr_to_rgb(_p(ycc, _f32p), ycc.size // 3, _p(out, _u8p))
    return out


def dct_rows(x: np.ndarray, inverse: bool = False) -> np.ndarray:
    x = np.array(x, dtype=np.float32, order="C", copy=True)
    n = x.shape[-1]
    lib().orc_dct_rows(_p(x, _f32p), x.size // n, n, int(inverse))
    return x


def dct2d_blocks(blocks: np.ndarray, inverse: bool = False) -> np.ndarray:
    x = np.array(blocks, dtype=np.float32, order="C", copy=True)
    b = x.shape[-1]
    lib().orc_dct2d_blocks(_p(x, _f32p), x.size // (b * b), b, int(inverse))
    return x


def svd_blocks(D: np.ndarray):
    D = np.ascontiguousarray(D, dtype=np.float32)
    b = D.shape[-1]
    nb = D.size // (b * b)
    U = np.empty(D.shape, np.float32)
    Vt = np.empty(D.shape, np.float32)
    S = np.empty(D.shape[:-1], np.float32)
    sw = np.empty(max(nb, 1), np.int32)
    lib().orc_svd_blocks(_p(D, _f32p), nb, b, _p(U, _f32p), _p(S, _f32p), _p(Vt, _f32p), _p(sw, _i32p))
    return U, S, Vt, sw[:nb]


def lp_svd_blocks(D: np.ndarray, nthreads: int | None = None):
    """numpy.linalg.svd of float32 blocks as the reference gets it (LAPACK dgesdd route,
    tmfwm_lapack.c): f32 U, S, Vt."""
    D = np.ascontiguousarray(D, dtype=np.float32)
    b = D.shape[-1]
    nb = D.size // (b * b)
    U = np.empty(D.shape, np.float32)
    Vt = np.empty(D.shape, np.float32)
    S = np.empty(D.shape[:-1], np.float32)
    if lib().orc_lp_svd_blocks(_p(D, _f32p), nb, b, _p(U, _f32p), _p(S, _f32p), _p(Vt, _f32p), nthreads or default_threads()):
        raise ValueError("lapack restatement did not converge")
    return U, S, Vt


def svd_blocks_f64(D: np.ndarray, nthreads: int | None = None):
    """The Jacobi route's f64 factors before rounding: U (u[r][k]), sig, V (v[r][k]), sorted."""
    D = np.ascontiguousarray(D, dtype=np.float32)
    b = D.shape[-1]
    nb = D.size // (b * b)
    U = np.empty(D.shape, np.float64)
    V = np.empty(D.shape, np.float64)
    S = np.empty(D.shape[:-1], np.float64)
    lib().orc_svd_blocks_f64(_p(D, _f32p), nb, b, _p(U, _f64p), _p(S, _f64p), _p(V, _f64p), nthreads or default_threads())
    return U, S, V


def lp_dnrm2(x: np.ndarray, inc: int = 1) -> float:
    """OpenBLAS dnrm2 (x87 extended, four accumulators) as restated for LAPACK's dlarfg."""
    x = np.ascontiguousarray(x, np.float64)
    n = (x.size + inc - 1) // inc if x.size else 0
    return float(lib().orc_lp_dnrm2(n, _p(x, _f64p), inc))


def lp_svd(a: np.ndarray):
    """numpy.linalg.svd of one f64 n x n matrix (dgesdd route restated): u, s, vt in f64."""
    a = np.ascontiguousarray(a, dtype=np.float64)
    n = a.shape[0]
    u, vt, s = np.empty((n, n)), np.empty((n, n)), np.empty(n)
    rc = lib().orc_lp_svd(_p(a, _f64p), n, _p(u, _f64p), _p(s, _f64p), _p(vt, _f64p))
    if rc:
        raise ValueError(f"lapack restatement rc={rc}")
    return u, s, vt


def sigma1(D: np.ndarray) -> float:
    D = np.ascontiguousarray(D, dtype=np.float32)
    return float(lib().orc_sigma1_block(_p(D, _f32p), D.shape[-1]))


def blend_reconstruct_blocks(U, S, Vt, w: np.ndarray, alpha: float) -> np.ndarray:
    """N7 + N8 over nb blocks; w holds one watermark byte per block."""
    U = np.ascontiguousarray(U, np.float32)
    S = np.ascontiguousarray(S, np.float32)
    Vt = np.ascontiguousarray(Vt, np.float32)
    w = np.ascontiguousarray(w, np.uint8)
    b = U.shape[-1]
    nb = U.size // (b * b)
    assert w.size == nb and S.size == nb * b and Vt.shape == U.shape
    M = np.empty_like(U)
    lib().orc_blend_reconstruct_blocks(_p(U, _f32p), _p(S, _f32p), _p(Vt, _f32p), nb, b, _p(w, _u8p), float(alpha), _p(M, _f32p))
    return M


def blend_reconstruct(U, S, Vt, w: int, alpha: float) -> np.ndarray:
    U = np.ascontiguousarray(U, np.float32)
    S = np.ascontiguousarray(S, np.float32)
    Vt = np.ascontiguousarray(Vt, np.float32)
    M = np.empty_like(U)
    lib().orc_blend_reconstruct(_p(U, _f32p), _p(S, _f32p), _p(Vt, _f32p), U.shape[-1], int(w), float(alpha), _p(M, _f32p))
    return M


# --- whole-frame paths ------------------------------------------------------
# SVD routes (tmfwm_oracle.c ORC_SVD_*): "lapack" = the reference's own dgesdd arithmetic
# (tmfwm_lapack.c); "jacobi" / "hybrid" = the specified device routes.  None = the route
# libtmfwm.so implements (the contract the GPU tests compare against).
ROUTES = {"jacobi": 0, "lapack": 1, "hybrid": 2}


def embed_frame(rgb: np.ndarray, wm_tile: np.ndarray, block: int, alpha: float, nthreads: int | None = None,
                route: str | None = None, stats: dict | None = None) -> np.ndarray:
    rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
    H, W = rgb.shape[:2]
    wm_tile = np.ascontiguousarray(wm_tile, dtype=np.uint8)
    assert wm_tile.shape == (H // block, W // block), (wm_tile.shape, H, W, block)
    out = np.empty_like(rgb)
    nfb = ctypes.c_int64(0)
    if route is None:
        rc = lib().orc_embed_frame(_p(rgb, _u8p), H, W, _p(wm_tile, _u8p), block, float(alpha), _p(out, _u8p), nthreads or default_threads())
    else:
        rc = lib().orc_embed_frame_mode(_p(rgb, _u8p), H, W, _p(wm_tile, _u8p), block, float(alpha), _p(out, _u8p),
                                        nthreads or default_threads(), ROUTES[route], ctypes.byref(nfb))
    if rc:
        raise ValueError(f"oracle embed failed rc={rc}")
    if stats is not None:
        stats["fallback_blocks"] = int(nfb.value)
    return out


def extract_frame(wrgb: np.ndarray, orgb: np.ndarray, block: int, alpha: float, nthreads: int | None = None,
                  route: str | None = None) -> np.ndarray:
    wrgb = np.ascontiguousarray(wrgb, dtype=np.uint8)
    orgb = np.ascontiguousarray(orgb, dtype=np.uint8)
    H, W = wrgb.shape[:2]
    assert orgb.shape == wrgb.shape
    out = np.empty((H // block, W // block), np.uint8)
    if route is None:
        rc = lib().orc_extract_frame(_p(wrgb, _u8p), _p(orgb, _u8p), H, W, block, float(alpha), _p(out, _u8p), nthreads or default_threads())
    else:
        rc = lib().orc_extract_frame_mode(_p(wrgb, _u8p), _p(orgb, _u8p), H, W, block, float(alpha), _p(out, _u8p),
                                          nthreads or default_threads(), ROUTES[route])
    if rc:
        raise ValueError(f"oracle extract failed rc={rc}")
    return out


def svd_flag(sig: np.ndarray) -> bool:
    """The hybrid route's conditioning test on one block's f64 singular values."""
    sig = np.ascontiguousarray(sig, np.float64)
    return bool(lib().orc_svd_flag(_p(sig, _f64p), sig.size))


def embed_batch(rgb: np.ndarray, wm_tile: np.ndarray, block: int, alpha: float, nthreads: int | None = None) -> np.ndarray:
    rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
    n, H, W = rgb.shape[:3]
    wm_tile = np.ascontiguousarray(wm_tile, dtype=np.uint8)
    out = np.empty_like(rgb)
    rc = lib().orc_embed_batch(_p(rgb, _u8p), n, H, W, _p(wm_tile, _u8p), block, float(alpha), _p(out, _u8p), nthreads or default_threads())
    if rc:
        raise ValueError(f"oracle embed failed rc={rc}")
    return out


def extract_batch(wrgb: np.ndarray, orgb: np.ndarray, block: int, alpha: float, nthreads: int | None = None) -> np.ndarray:
    wrgb = np.ascontiguousarray(wrgb, dtype=np.uint8)
    orgb = np.ascontiguousarray(orgb, dtype=np.uint8)
    n, H, W = wrgb.shape[:3]
    out = np.empty((n, H // block, W // block), np.uint8)
    rc = lib().orc_extract_batch(_p(wrgb, _u8p), _p(orgb, _u8p), n, H, W, block, float(alpha), _p(out, _u8p), nthreads or default_threads())
    if rc:
        raise ValueError(f"oracle extract failed rc={rc}")
    return out


def synth_bytes(seed: int, frame0: int, nframes: int, frame_bytes: int) -> np.ndarray:
    out = np.empty(nframes * frame_bytes, np.uint8)
    lib().orc_synth_bytes(ctypes.c_uint64(seed), frame0, nframes, frame_bytes, _p(out, _u8p))
    return out


# --- watermark preparation (watermarking.py:102-132 after convert("L")) ------
def resize_lanczos(img: np.ndarray, oh: int, ow: int) -> np.ndarray:
    img = np.ascontiguousarray(img, np.uint8)
    out = np.empty((oh, ow), np.uint8)
    if lib().orc_resize_lanczos(_p(img, _u8p), img.shape[0], img.shape[1], oh, ow, _p(out, _u8p), ow):
        raise ValueError("empty size")
    return out


def prepare_tile(wm_l: np.ndarray, th: int, tw: int, preserve_ratio: bool) -> np.ndarray:
    wm_l = np.ascontiguousarray(wm_l, np.uint8)
    out = np.empty((th, tw), np.uint8)
    if lib().orc_prepare_tile(_p(wm_l, _u8p), wm_l.shape[0], wm_l.shape[1], th, tw, int(bool(preserve_ratio)), _p(out, _u8p)):
        raise ValueError("empty size")
    return out
