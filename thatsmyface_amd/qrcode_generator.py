"""Drop-in for the reference's modules/qrcode_generator.py (text_to_qrcode :10-44,
qrcode_to_text :47-76) on libtmfwm.so's host QR codec (include/tmfwm.h tmfwm_qr_*), so the
pages work without python-qrcode / pyzbar (neither is in this image).

text_to_qrcode: bytes are base64-encoded first (:23-24); error correction H, the smallest
version >= 1 that fits (QRCode(version=1, ...).make(fit=True)), python-qrcode's segmentation
and mask choice, 10-pixel modules with a 4-module white border drawn in a mode-"1" image
(make_image(fill_color="black", back_color="white")), resized to `size` -- Pillow resamples
mode "1" images with NEAREST whatever filter is asked, so LANCZOS at :41 is NEAREST.
qrcode_to_text: the first decodable symbol's text, base64-decoded when that succeeds (:60-69),
None when nothing decodes or on any error (:70-76).
"""
from __future__ import annotations

import base64
import ctypes
from typing import Tuple, Union

import numpy as np
from PIL import Image

from . import _lib

EC_L, EC_M, EC_Q, EC_H = 0, 1, 2, 3
BOX_SIZE, BORDER = 10, 4  # qrcode_generator.py:30-31


def qr_matrix(data: bytes, ec_level: int = EC_H, min_version: int = 1, mask: int = -1) -> np.ndarray:
    """Module matrix (True = dark) of `data` (tmfwm_qr_encode)."""
    L = _lib.load()
    size = ctypes.c_int32(0)
    buf = (ctypes.c_uint8 * 1)()
    rc = L.tmfwm_qr_encode(data, len(data), ec_level, min_version, mask, buf, 0, ctypes.byref(size))
    if size.value == 0:
        _lib.check(rc, "qr_encode")
    out = np.empty((size.value, size.value), np.uint8)
    _lib.check(L.tmfwm_qr_encode(data, len(data), ec_level, min_version, mask, out.ctypes.data, out.size,
                                 ctypes.byref(size)), "qr_encode")
    return out.astype(bool)


def render(modules: np.ndarray, box_size: int = BOX_SIZE, border: int = BORDER) -> Image.Image:
    """python-qrcode's PilImage for black on white: a mode-"1" image, dark boxes on white."""
    n = modules.shape[0]
    grid = np.pad(modules, border, constant_values=False)
    px = np.where(np.kron(grid, np.ones((box_size, box_size), bool)), 0, 255).astype(np.uint8)
    assert px.shape == ((n + 2 * border) * box_size,) * 2
    return Image.fromarray(px, "L").convert("1")


def text_to_qrcode(text: Union[str, bytes], size: Tuple[int, int] = (300, 300)) -> Image.Image:
    if isinstance(text, bytes):
        text = base64.b64encode(text).decode("utf-8")
    img = render(qr_matrix(text.encode("utf-8"), EC_H, 1))
    return img.resize(size, Image.LANCZOS)


def decode_image(gray: np.ndarray) -> bytes | None:
    """Payload of the first decodable upright QR symbol in an (h, w) uint8 grey image, or None."""
    g = np.ascontiguousarray(gray, dtype=np.uint8)
    if g.ndim != 2 or g.size == 0:
        raise ValueError("decode_image needs a non-empty (h, w) uint8 image")
    L = _lib.load()
    cap = 4096
    out = np.empty(cap, np.uint8)
    n = ctypes.c_int32(0)
    rc = L.tmfwm_qr_decode(g.ctypes.data, g.shape[0], g.shape[1], g.strides[0], out.ctypes.data, cap, ctypes.byref(n))
    if rc == _lib.ERR_NODATA:
        return None
    _lib.check(rc, "qr_decode")
    return out[: n.value].tobytes()


def decode_tiles(tiles: np.ndarray, capacity: int = 512) -> list:
    """Payloads of a batch of extracted tiles (n, h, w) uint8, decoded on host threads
    (tmfwm_qr_decode_batch); None where a tile holds no decodable symbol."""
    t = np.ascontiguousarray(tiles, dtype=np.uint8)
    if t.ndim != 3:
        raise ValueError("tiles must be (n, h, w) uint8")
    out = np.empty((len(t), capacity), np.uint8)
    lens = np.empty(len(t), np.int32)
    _lib.check(_lib.load().tmfwm_qr_decode_batch(t.ctypes.data, len(t), t.shape[1], t.shape[2], out.ctypes.data, capacity,
                                                 lens.ctypes.data), "qr_decode_batch")
    return [out[i, :k].tobytes() if k >= 0 else None for i, k in enumerate(lens)]


def qrcode_to_text(qr_image: Image.Image):
    try:
        data = decode_image(np.asarray(qr_image.convert("L")))
        if data is not None:
            text = data.decode("utf-8")
            try:
                return base64.b64decode(text)
            except Exception:
                return text
        return None
    except Exception as e:  # the reference prints and returns None (:74-76)
        print(f"Error decoding QR code: {str(e)}")
        return None
