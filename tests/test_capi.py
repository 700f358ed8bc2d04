"""CPU checks of the C-ABI boundary: libtmfwm.so loads, exports exactly what
include/tmfwm.h declares, validates arguments, and fails loudly without a GPU
(no CPU fallback).  No compute runs here."""
import ctypes
import os
import re

import numpy as np
import pytest

from thatsmyface_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    with open(os.path.join(ROOT, "include", "tmfwm.h")) as f:
        text = f.read()
    return sorted(set(re.findall(r"\b(tmfwm_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_header_symbol():
    L = _lib.load()
    names = header_functions()
    assert len(names) >= 10
    for n in names:
        assert hasattr(L, n), n
    assert set(names) == set(_lib.SIGNATURES), "ctypes signatures out of sync with include/tmfwm.h"


def test_nm_exports_match_header():
    import subprocess

    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = sorted(set(re.findall(r" T (tmfwm_[a-z0-9_]+)", out)))
    assert exported == header_functions()


def test_abi_version_and_device_count():
    L = _lib.load()
    assert L.tmfwm_abi_version() == _lib.ABI_VERSION == 10
    assert _lib.device_count() >= 0


def test_argument_validation_before_device():
    L = _lib.load()
    a = np.zeros((16, 16, 3), np.uint8)
    t = np.zeros((2, 2), np.uint8)
    o = np.empty_like(a)
    p = lambda x: x.ctypes.data  # noqa: E731
    for bad_block in (7, 18, 2):  # the app's slider offers 4..16 step 2; nothing else is supported
        with pytest.raises(NotImplementedError):
            _lib.check(L.tmfwm_embed(p(a), 1, 16, 16, a.size, p(t), bad_block, 0.1, p(o), _lib.MEM_HOST, None), "embed")
    with pytest.raises(ValueError):  # negative size
        _lib.check(L.tmfwm_embed(p(a), -1, 16, 16, a.size, p(t), 8, 0.1, p(o), _lib.MEM_HOST, None), "embed")
    with pytest.raises(ValueError):  # frame stride shorter than a frame
        _lib.check(L.tmfwm_embed(p(a), 2, 16, 16, 10, p(t), 8, 0.1, p(o), _lib.MEM_HOST, None), "embed")
    with pytest.raises(ValueError):  # alpha NaN
        _lib.check(L.tmfwm_embed(p(a), 1, 16, 16, a.size, p(t), 8, float("nan"), p(o), _lib.MEM_HOST, None), "embed")
    assert "frame_stride" in _lib.last_error() or "alpha" in _lib.last_error()
    for bad_route in (-1, 4):  # TMFWM_ROUTE_HYBRID / _REFERENCE / _RANK1 / _RANK1_REFERENCE only
        with pytest.raises(ValueError, match="route"):
            _lib.check(L.tmfwm_embed_route(p(a), 1, 16, 16, a.size, p(t), 8, 0.1, p(o), _lib.MEM_HOST, None, bad_route, None), "e")
        with pytest.raises(ValueError, match="route"):
            _lib.check(L.tmfwm_extract_route(p(a), p(a), 1, 16, 16, a.size, 8, 0.1, p(t), _lib.MEM_HOST, None, bad_route, None), "x")
    assert [L.tmfwm_embed_list_pass(k) for k in (4, 6, 8, 10, 12, 14, 16, 7, 18)] == [0, 0, 1, 0, 0, 0, 0, 0, 0]
    # 4-byte pixel entry points (ABI 8): layouts and strides checked before any device work
    a4 = np.zeros((16, 16, 4), np.uint8)
    o4 = np.empty_like(a4)
    for px in (2, 5):
        with pytest.raises(ValueError, match="pixel bytes"):
            _lib.check(L.tmfwm_embed_px(p(a4), px, a4.size, 1, 16, 16, p(t), 8, 0.1, p(o4), 4, o4.size, _lib.MEM_HOST, None, 0,
                                        None), "embed_px")
    with pytest.raises(ValueError, match="frame_stride"):  # a 4-byte frame needs H*W*4 bytes
        _lib.check(L.tmfwm_embed_px(p(a4), 4, a.size, 1, 16, 16, p(t), 8, 0.1, p(o4), 4, o4.size, _lib.MEM_HOST, None, 0, None),
                   "embed_px")
    with pytest.raises(ValueError, match="one frame_stride"):  # 3 -> 3 is tmfwm_embed_route
        _lib.check(L.tmfwm_embed_px(p(a), 3, a.size, 1, 16, 16, p(t), 8, 0.1, p(o), 3, a.size + 4, _lib.MEM_HOST, None, 0, None),
                   "embed_px")
    with pytest.raises(NotImplementedError):
        _lib.check(L.tmfwm_embed_px(p(a4), 4, a4.size, 1, 16, 16, p(t), 7, 0.1, p(o4), 4, o4.size, _lib.MEM_HOST, None, 0, None),
                   "embed_px")
    with pytest.raises(ValueError, match="alpha"):
        _lib.check(L.tmfwm_extract_px(p(a4), 4, a4.size, p(a), 3, a.size, 1, 16, 16, 8, 0.0, p(t), _lib.MEM_HOST, None, 0, None),
                   "extract_px")
    with pytest.raises(ValueError, match="original frame_stride"):
        _lib.check(L.tmfwm_extract_px(p(a4), 4, a4.size, p(a), 4, a.size, 1, 16, 16, 8, 0.1, p(t), _lib.MEM_HOST, None, 0, None),
                   "extract_px")
    with pytest.raises(ValueError):
        _lib.route_code("exact")
    assert (_lib.route_code("hybrid"), _lib.route_code("reference")) == (_lib.ROUTE_HYBRID, _lib.ROUTE_REFERENCE) == (0, 1)


@pytest.mark.skipif(_lib.device_count() > 0, reason="CPU-only check")
def test_fails_loudly_without_gpu():
    from thatsmyface_amd import watermarking as W

    with pytest.raises(_lib.TmfwmError, match="no HIP device"):
        W.rgb_to_ycbcr(np.zeros((4, 4, 3), np.uint8))
    from PIL import Image

    with pytest.raises(_lib.TmfwmError):
        W.embed_watermark(Image.new("RGB", (16, 16)), Image.new("L", (2, 2)), False, {"block_size": 8, "alpha": 0.1})


def test_product_never_imports_oracle():
    pkg = os.path.join(ROOT, "thatsmyface_amd")
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                with open(os.path.join(dp, f)) as fh:
                    src = fh.read()
                assert not re.search(r"^\s*(from|import)\s+oracle\b", src, re.M), f
                assert "tmfwm_oracle" not in src, f
                assert "libtmfwm_oracle" not in src, f


def test_multi_entry_points_validate_then_need_a_device():
    """tmfwm_embed_multi / tmfwm_extract_multi: arguments are checked first; without a GPU
    the call fails with TMFWM_ERR_NODEVICE (no CPU fallback)."""
    from thatsmyface_amd import multi

    a = np.zeros((2, 16, 16, 3), np.uint8)
    t = np.zeros((2, 2), np.uint8)
    with pytest.raises(NotImplementedError):
        multi.embed_multi(a, t, 7, 0.1)
    with pytest.raises(ValueError):
        multi.embed_multi(a, np.zeros((3, 3), np.uint8), 8, 0.1)
    L = _lib.load()
    p = lambda x: x.ctypes.data  # noqa: E731
    with pytest.raises(ValueError, match="route"):
        multi.embed_multi(a, t, 8, 0.1, route="exact")
    with pytest.raises(ValueError, match="route"):
        _lib.check(_lib.load().tmfwm_embed_multi_route(a.ctypes.data, 2, 16, 16, 16 * 16 * 3, t.ctypes.data, 8, 0.1, a.ctypes.data,
                                                       None, 0, 4, None), "embed_multi_route")
    with pytest.raises(ValueError):  # alpha = 0 divides by zero in extract (watermarking.py:285)
        _lib.check(L.tmfwm_extract_multi(p(a), p(a), 2, 16, 16, 16 * 16 * 3, 8, 0.0, p(t), None, 0, None), "extract_multi")
    if _lib.device_count() == 0:
        with pytest.raises(_lib.TmfwmError, match="no HIP device"):
            multi.embed_multi(a, t, 8, 0.1)
        with pytest.raises(_lib.TmfwmError, match="no HIP device"):
            multi.extract_multi(a, a, 8, 0.1, devices=[0, 0])
