"""Drop-in for ``modules/watermarking.py`` of ThatsMyFace, running on MI355X.

Same module surface and signatures as the reference
(/root/reference/modules/watermarking.py): ``get_watermark_settings`` (:10),
``rgb_to_ycbcr`` (:23), ``ycbcr_to_rgb`` (:53), ``apply_dct_to_block`` (:76),
``apply_idct_to_block`` (:81), ``resize_watermark`` (:86), ``embed_watermark``
(:135), ``extract_watermark`` (:224).  The host keeps PIL for image decode and
mode conversion only; the watermark's LANCZOS resample and every per-pixel and
per-block loop run in libtmfwm.so's HIP kernels and return the reference's
bytes.  There is no CPU fallback: without the
built library or a GPU these functions raise.

Deviations: block sizes other than the app's slider values
(4..16 step 2) raise NotImplementedError; an original image smaller than the watermarked one raises
ValueError (the reference raises for a full block of shortfall and silently
computes partial blocks for less); array inputs to the helper functions must be
uint8 RGB(A) / float32 as the reference itself produces them.
"""
from __future__ import annotations

import ctypes
import hashlib
import io
import os
import sys
import threading
import weakref

import numpy as np
from PIL import Image

from . import _lib
from .constants import ALPHA, BLOCK_SIZE, SVD_ROUTE

__all__ = [
    "get_watermark_settings",
    "rgb_to_ycbcr",
    "ycbcr_to_rgb",
    "apply_dct_to_block",
    "apply_idct_to_block",
    "resize_watermark",
    "embed_watermark",
    "extract_watermark",
]


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data_as(ctypes.c_void_p).value or 0


def get_watermark_settings():
    """watermarking.py:10-20: session-state settings, else the module defaults.

    streamlit is imported lazily (the reference imports it at module top, :5, but
    uses it only here), so the module also works outside a Streamlit app.
    """
    try:
        import streamlit as st  # noqa: PLC0415
    except ImportError:
        return {"block_size": BLOCK_SIZE, "alpha": ALPHA}
    state = getattr(st, "session_state", {})
    if "custom_settings" in state:
        settings = state.custom_settings if hasattr(state, "custom_settings") else state["custom_settings"]
        return {
            "block_size": settings.get("block_size", BLOCK_SIZE),
            "alpha": settings.get("alpha", ALPHA),
        }
    return {"block_size": BLOCK_SIZE, "alpha": ALPHA}


def _rgb_pixels(img) -> np.ndarray:
    """rgb_to_ycbcr's input as the reference reads it (:26-34): PIL -> convert("RGB");
    uint8 arrays stay uint8 (the fast path), any other numeric array gets the
    reference's own cast np.array(img, dtype=np.float32) (:29); RGBA -> first three
    channels (:32-34)."""
    if isinstance(img, Image.Image):
        img = img.convert("RGB")
    arr = np.asarray(img)
    if arr.dtype != np.uint8:
        arr = np.asarray(arr, dtype=np.float32)
    if arr.ndim != 3 or arr.shape[-1] not in (3, 4):
        raise ValueError(f"expected an (H, W, 3|4) image, got shape {arr.shape}")
    if arr.shape[-1] == 4:
        arr = arr[..., :3]
    return np.ascontiguousarray(arr)


def rgb_to_ycbcr(img) -> np.ndarray:
    """watermarking.py:23-50 on the GPU: (H, W, 3) float32 (Y, Cb + 0.5, Cr + 0.5).
    uint8 / PIL inputs go as bytes; other numeric arrays as their float32 cast."""
    rgb = _rgb_pixels(img)
    out = np.empty(rgb.shape[:2] + (3,), np.float32)
    L = _lib.load()
    fn = L.tmfwm_rgb_to_ycbcr if rgb.dtype == np.uint8 else L.tmfwm_rgb_to_ycbcr_f32
    _lib.check(fn(_ptr(rgb), rgb.shape[0] * rgb.shape[1], _ptr(out), _lib.MEM_HOST, None), "rgb_to_ycbcr")
    return out


_YCC_DTYPES = {np.dtype(np.float16): _lib.DT_F16, np.dtype(np.float32): _lib.DT_F32, np.dtype(np.float64): _lib.DT_F64}


def ycbcr_to_rgb(img) -> np.ndarray:
    """watermarking.py:53-73 on the GPU: (H, W, 3) float16/32/64 -> (H, W, 3) uint8, in
    the input's own float type as the reference computes (:55 img.copy())."""
    ycc = np.asarray(img)
    if ycc.dtype.kind == "f" and not ycc.dtype.isnative:
        # a byte-swapped float ('>f4' ...) holds the same values: compute on the native layout
        ycc = ycc.astype(ycc.dtype.newbyteorder("="))
    if ycc.dtype not in _YCC_DTYPES:
        # the reference's in-place "-= 0.5" (:58) refuses non-float arrays; longdouble has no
        # type of its own here (the reference would compute in it)
        raise TypeError(f"expected a float16/32/64 array, got {ycc.dtype}")
    if ycc.ndim != 3 or ycc.shape[-1] != 3:
        raise ValueError(f"expected an (H, W, 3) array, got shape {ycc.shape}")
    ycc = np.ascontiguousarray(ycc)
    out = np.empty(ycc.shape, np.uint8)
    L = _lib.load()
    _lib.check(L.tmfwm_ycbcr_to_rgb_typed(_ptr(ycc), _YCC_DTYPES[ycc.dtype], ycc.shape[0] * ycc.shape[1], _ptr(out),
                                          _lib.MEM_HOST, None), "ycbcr_to_rgb")
    return out


def _dct_blocks(block, inverse: bool) -> np.ndarray:
    arr = np.asarray(block)
    if arr.dtype != np.float32:
        raise NotImplementedError(f"DCT blocks are float32 on this path (got {arr.dtype})")
    if arr.ndim < 2 or arr.shape[-1] != arr.shape[-2]:
        raise NotImplementedError(f"square b x b blocks only (got {arr.shape})")
    out = np.array(arr, dtype=np.float32, order="C", copy=True)
    b = out.shape[-1]
    L = _lib.load()
    _lib.check(L.tmfwm_dct2d_blocks(_ptr(out), out.size // (b * b), b, int(inverse), _lib.MEM_HOST, None),
               "apply_idct_to_block" if inverse else "apply_dct_to_block")
    return out


def apply_dct_to_block(block) -> np.ndarray:
    """watermarking.py:76-78: 2-D orthonormal DCT-II, axis 0 then axis 1 (also on a stack of blocks)."""
    return _dct_blocks(block, False)


def apply_idct_to_block(block) -> np.ndarray:
    """watermarking.py:81-83: 2-D orthonormal DCT-III, axis 0 then axis 1."""
    return _dct_blocks(block, True)


def resize_watermark(watermark, target_height, target_width, preserve_ratio=False):
    """watermarking.py:86-132.  PNG decode and convert("L") (:98-103) stay with PIL on
    the host; the LANCZOS resample and the white-canvas paste (:105-130) run on the GPU
    (tmfwm_prepare_tile), byte-identical to Pillow's fixed-point resampler."""
    watermark_img = Image.open(io.BytesIO(watermark)) if isinstance(watermark, bytes) else watermark
    grey = np.ascontiguousarray(np.asarray(watermark_img.convert("L"), dtype=np.uint8))
    th, tw = int(target_height), int(target_width)
    if th <= 0 or tw <= 0 or grey.size == 0:
        raise ValueError("height and width must be > 0")
    tile = np.empty((th, tw), np.uint8)
    L = _lib.load()
    _lib.check(L.tmfwm_prepare_tile(_ptr(grey), grey.shape[0], grey.shape[1], th, tw, int(bool(preserve_ratio)), _ptr(tile),
                                    _lib.MEM_HOST, None), "resize_watermark")
    return Image.fromarray(tile, "L")


def _settings(custom_settings):
    settings = custom_settings if custom_settings else get_watermark_settings()
    return settings.get("block_size", BLOCK_SIZE), settings.get("alpha", ALPHA)


def _route(custom_settings) -> int:
    """The SVD route of one drop-in call: custom_settings["svd_route"] if given,
    else the TMFWM_SVD_ROUTE environment variable, else constants.SVD_ROUTE.  "reference"
    computes every block's SVD with np.linalg.svd's own arithmetic (the dgesdd route), so
    the bytes are the reference's by construction; "hybrid" is the batch path's route."""
    r = (custom_settings or {}).get("svd_route") if isinstance(custom_settings, dict) else None
    return _lib.route_code(r or os.environ.get("TMFWM_SVD_ROUTE") or SVD_ROUTE)


def _rgb_image(img):
    """img.convert("RGB") as the reference calls it (:154, :242-243), without its copy when the
    image already is RGB (the pixels are only read)."""
    return img if img.mode == "RGB" else img.convert("RGB")


# Prepared watermark tiles of PNG-bytes watermarks, keyed by the bytes' digest and the tile
# geometry: the app embeds one QR code into every uploaded image (embed_watermark_page.py:
# 492-558), and its decode + resample would otherwise be redone per image.
_TILE_CACHE_MAX = 16
_tile_cache: "dict[tuple, np.ndarray]" = {}
_tile_lock = threading.Lock()
# Per-thread output staging of embed_watermark's copying path: Image.fromarray copies an RGB
# array into PIL's own storage, so the array is reused by the thread's next call.
_tls = threading.local()

# Zero-copy PIL path: PIL holds a mode-"RGB" image as 4 bytes per pixel; pyarrow
# hands that memory over (Image.__arrow_c_array__) and Image.fromarrow wraps 4-byte output
# memory as an RGB image, so tmfwm_embed_px / tmfwm_extract_px read and write PIL's own layout
# and the host never packs or unpacks pixels.  Inputs Pillow stores in several blocks (large
# images) and read-only (mapped / arrow-backed) images -- Pillow 12.2's __arrow_c_array__
# crashes on those -- take np.asarray instead.  TMFWM_PIL_ZERO_COPY=0 turns the path off.
_zero_copy = os.environ.get("TMFWM_PIL_ZERO_COPY", "1") != "0"
_pa = None
_POOL_KEEP = 4  # output buffers kept per size
_out_pool: "dict[int, list[np.ndarray]]" = {}
_out_free: "set[int]" = set()  # ids of pooled buffers whose image has been collected
_pool_lock = threading.Lock()


def _arrow():
    """pyarrow when the zero-copy path can run: it also needs Pillow's Arrow interface
    (Image.fromarrow and Image.__arrow_c_array__, Pillow >= 11.2; the reference asks for
    Pillow >= 9, requirements.txt:3), otherwise every call takes the copying path."""
    global _pa, _zero_copy
    if _pa is None and _zero_copy:
        if not (hasattr(Image, "fromarrow") and hasattr(Image.Image, "__arrow_c_array__")):
            _zero_copy = False
            return None
        try:
            import pyarrow  # noqa: PLC0415

            _pa = pyarrow
        except ImportError:
            _zero_copy = False
    return _pa if _zero_copy else None


def _rgbx_view(image):
    """(address, keepalive) of PIL's own 4-byte pixels of an RGB image, or None."""
    own = getattr(image, "_tmfwm_rgbx", None)  # an embed_watermark output: its buffer as it is,
    if own is not None and image.readonly:  # unless PIL copied it (every in-place edit does first)
        return _ptr(own), own
    pa = _arrow()
    if pa is None or image.readonly or not hasattr(image, "__arrow_c_array__"):
        return None
    try:
        arr = pa.array(image)
    except (ValueError, TypeError, NotImplementedError):  # several memory blocks
        return None
    vals = arr.values
    if len(vals) != image.width * image.height * 4:
        return None
    return vals.buffers()[1].address + vals.offset, arr


def _release(buf: np.ndarray) -> None:
    # Lock-free: a finalizer runs in whichever thread triggers the collection, possibly one that
    # already holds _pool_lock.  dict.get, iterating a list another thread may append to, and
    # set.add are each atomic under the GIL; _take_out re-checks pool membership under the lock.
    if any(b is buf for b in _out_pool.get(buf.size, ())):  # pooled: free for the next call
        _out_free.add(id(buf))


def _take_out(nbytes: int) -> np.ndarray:
    """An RGBX output buffer: a pooled one whose image has been collected (weakref.finalize on
    the image, _rgb_from_rgbx) and that nothing else still references, else a new one (its pages
    are then faulted in once; page-locked buffers measured no faster, r04k)."""
    with _pool_lock:
        lst = _out_pool.setdefault(nbytes, [])
        for b in lst:
            # the finalizer is the signal; the reference count only vetoes (an Arrow export of
            # the image taken by the caller keeps the buffer: the list, this name, the argument)
            if id(b) in _out_free and sys.getrefcount(b) <= 3:
                _out_free.discard(id(b))
                return b
        b = np.empty(nbytes, np.uint8)
        if len(lst) < _POOL_KEEP:
            _out_free.discard(id(b))  # a stale id of a collected, unpooled buffer at this address
            lst.append(b)
        return b


def _give_back(buf: np.ndarray) -> None:
    """A buffer from _take_out that no image was built around (the call failed): free again."""
    _release(buf)


def _rgb_from_rgbx(buf: np.ndarray, width: int, height: int):
    """Image.fromarrow over the RGBX buffer: a mode-"RGB" image sharing its memory."""
    pa = _pa
    vals = pa.Array.from_buffers(pa.uint8(), width * height * 4, [None, pa.py_buffer(buf)])
    img = Image.fromarrow(pa.FixedSizeListArray.from_arrays(vals, 4), "RGB", (width, height))
    img._tmfwm_rgbx = buf  # extract_watermark reads it back without an export
    weakref.finalize(img, _release, buf)  # the pool may hand the buffer out again
    return img


def _tile_for(watermark_data, nbh, nbw, preserve_ratio) -> np.ndarray:
    if not isinstance(watermark_data, bytes):
        return np.ascontiguousarray(np.asarray(resize_watermark(watermark_data, nbh, nbw, preserve_ratio), dtype=np.uint8))
    key = (hashlib.sha256(watermark_data).digest(), nbh, nbw, bool(preserve_ratio))
    with _tile_lock:
        t = _tile_cache.get(key)
    if t is None:
        t = np.ascontiguousarray(np.asarray(resize_watermark(Image.open(io.BytesIO(watermark_data)), nbh, nbw, preserve_ratio),
                                            dtype=np.uint8))
        t.setflags(write=False)
        with _tile_lock:
            if len(_tile_cache) >= _TILE_CACHE_MAX:
                _tile_cache.pop(next(iter(_tile_cache)))
            _tile_cache[key] = t
    return t


def embed_watermark(image, watermark_data, preserve_ratio=False, custom_settings=None):
    """watermarking.py:135-221: returns a new RGB PIL image of the same size."""
    block_size, alpha = _settings(custom_settings)
    image = _rgb_image(image)
    block_size = int(block_size)
    if block_size <= 0:
        raise ValueError(f"block_size must be positive, got {block_size}")
    width, height = image.size
    nbh, nbw = height // block_size, width // block_size
    tile = _tile_for(watermark_data, nbh, nbw, preserve_ratio)
    route = _route(custom_settings)
    if _arrow() is not None and height > 0 and width > 0:
        view = _rgbx_view(image)
        if view is not None:
            src, src_px, keep = view[0], _lib.PIX_RGBX, view[1]
        else:
            keep = np.ascontiguousarray(np.asarray(image, dtype=np.uint8))
            src, src_px = _ptr(keep), _lib.PIX_RGB
        out = _take_out(height * width * 4)
        L = _lib.load()
        try:
            _lib.check(
                L.tmfwm_embed_px(src, src_px, height * width * src_px, 1, height, width, _ptr(tile), block_size, float(alpha),
                                 _ptr(out), _lib.PIX_RGBX, height * width * 4, _lib.MEM_HOST, None, route, None),
                "embed_watermark",
            )
        except BaseException:
            _give_back(out)
            raise
        del keep
        return _rgb_from_rgbx(out, width, height)
    rgb = np.ascontiguousarray(np.asarray(image, dtype=np.uint8))
    out = getattr(_tls, "out", None)
    if out is None or out.shape != rgb.shape:
        out = np.empty_like(rgb)
    _tls.out = None  # owned by this call until PIL has copied it
    L = _lib.load()
    _lib.check(
        L.tmfwm_embed_route(_ptr(rgb), 1, height, width, rgb.size, _ptr(tile), block_size, float(alpha), _ptr(out), _lib.MEM_HOST,
                            None, route, None),
        "embed_watermark",
    )
    img = Image.fromarray(out)
    if not getattr(img, "readonly", 0):  # PIL copied the pixels: the array is free again
        _tls.out = out
    return img


def extract_watermark(watermarked_image, original_image, custom_settings=None):
    """watermarking.py:224-294: returns the (W/b) x (H/b) mode-"L" extracted watermark."""
    block_size, alpha = _settings(custom_settings)
    block_size = int(block_size)
    if block_size <= 0:
        raise ValueError(f"block_size must be positive, got {block_size}")
    wimg, oimg = _rgb_image(watermarked_image), _rgb_image(original_image)
    width, height = wimg.size
    nbh, nbw = height // block_size, width // block_size
    route = _route(custom_settings)
    if _arrow() is not None and nbh > 0 and nbw > 0 and oimg.size == wimg.size:
        ins = []
        for img in (wimg, oimg):
            view = _rgbx_view(img)
            if view is None:
                arr = np.ascontiguousarray(np.asarray(img, dtype=np.uint8))
                view = (_ptr(arr), arr)
                px = _lib.PIX_RGB
            else:
                px = _lib.PIX_RGBX
            ins.append((view[0], px, view[1]))
        out = np.empty((nbh, nbw), np.uint8)
        L = _lib.load()
        (wp, wpx, _), (op, opx, _) = ins
        _lib.check(
            L.tmfwm_extract_px(wp, wpx, height * width * wpx, op, opx, height * width * opx, 1, height, width, block_size,
                               float(alpha), _ptr(out), _lib.MEM_HOST, None, route, None),
            "extract_watermark",
        )
        del ins
        return Image.fromarray(out)
    w = np.asarray(wimg, dtype=np.uint8)
    o = np.asarray(oimg, dtype=np.uint8)
    if nbh == 0 or nbw == 0:
        return Image.fromarray(np.zeros((nbh, nbw), np.uint8))
    if o.shape[0] < height or o.shape[1] < width:
        raise ValueError(
            f"original image {o.shape[1]}x{o.shape[0]} is smaller than the watermarked image {width}x{height}"
        )
    w = np.ascontiguousarray(w)
    o = np.ascontiguousarray(o[:height, :width])  # the reference slices the original with the watermarked grid
    out = np.empty((nbh, nbw), np.uint8)
    L = _lib.load()
    _lib.check(
        L.tmfwm_extract_route(_ptr(w), _ptr(o), 1, height, width, w.size, block_size, float(alpha), _ptr(out), _lib.MEM_HOST,
                              None, route, None),
        "extract_watermark",
    )
    return Image.fromarray(out)
