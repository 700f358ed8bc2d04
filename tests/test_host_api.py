"""Host-side logic of the drop-in module (no GPU): settings resolution
(watermarking.py:10-20), watermark resize (:86-132) against the reference's
tiles, and the argument checks that run before any kernel."""
import gc
import io
import sys
import types

import numpy as np
import pytest
from PIL import Image

from thatsmyface_amd import watermarking as W


def test_settings_defaults_without_streamlit(monkeypatch):
    monkeypatch.setitem(sys.modules, "streamlit", None)  # import fails -> defaults
    assert W.get_watermark_settings() == {"block_size": 8, "alpha": 0.1}


def test_settings_from_session_state(monkeypatch):
    class State(dict):
        def __getattr__(self, k):
            return self[k]

    st = types.ModuleType("streamlit")
    st.session_state = State(custom_settings={"block_size": 16})
    monkeypatch.setitem(sys.modules, "streamlit", st)
    assert W.get_watermark_settings() == {"block_size": 16, "alpha": 0.1}
    st.session_state = State()
    assert W.get_watermark_settings() == {"block_size": 8, "alpha": 0.1}


def test_extract_rejects_smaller_original():
    big = Image.new("RGB", (64, 64))
    with pytest.raises(ValueError, match="smaller"):
        W.extract_watermark(big, Image.new("RGB", (56, 64)), {"block_size": 8, "alpha": 0.1})


def test_extract_tiny_image_is_empty_like_reference():
    img = Image.new("RGB", (5, 5))
    out = W.extract_watermark(img, img, {"block_size": 8, "alpha": 0.1})
    assert np.asarray(out).shape == (0, 0)


def test_embed_tiny_image_raises_like_reference():
    # the reference's PIL resize raises "height and width must be > 0"
    with pytest.raises(ValueError):
        W.embed_watermark(Image.new("RGB", (5, 5)), Image.new("L", (4, 4)), False, {"block_size": 8, "alpha": 0.1})


def test_helper_input_checks():
    with pytest.raises(ValueError):
        W.rgb_to_ycbcr(np.zeros((2, 2), np.float32))
    with pytest.raises(TypeError):  # the reference's in-place "-= 0.5" (:58) refuses integers
        W.ycbcr_to_rgb(np.zeros((2, 2, 3), np.uint8))
    with pytest.raises(NotImplementedError):
        W.apply_dct_to_block(np.zeros((8, 8), np.float64))
    with pytest.raises(NotImplementedError):
        W.apply_dct_to_block(np.zeros((8, 4), np.float32))


def test_module_path_shim():
    from thatsmyface_amd.modules import constants, watermarking

    assert watermarking.embed_watermark is W.embed_watermark
    assert constants.BLOCK_SIZE == 8 and constants.ALPHA == 0.1


def test_zero_copy_pil_helpers():
    """Host side of the drop-in's zero-copy PIL path, no GPU needed: PIL's own
    4-byte memory of a single-block RGB image is handed over (its bytes are the pixels plus a
    pad byte), read-only and multi-block images are not, embed_watermark's own outputs hand over
    their buffer while PIL has not copied them, and pooled buffers come back only once nothing
    references them."""
    import gc

    pytest.importorskip("pyarrow")
    if not W._zero_copy:
        pytest.skip("TMFWM_PIL_ZERO_COPY=0")
    rng = np.random.default_rng(5)
    arr = rng.integers(0, 256, (48, 80, 3), dtype=np.uint8)
    img = Image.fromarray(arr)
    addr, keep = W._rgbx_view(img)
    import ctypes

    got = np.frombuffer((ctypes.c_uint8 * (48 * 80 * 4)).from_address(addr), np.uint8).reshape(48, 80, 4)
    assert np.array_equal(got[..., :3], arr)
    del keep
    assert W._rgbx_view(Image.new("RGB", (3840, 2160))) is None  # several memory blocks
    # an output buffer wrapped as an RGB image: same pixels, read-only, its buffer handed back
    buf = W._take_out(48 * 80 * 4)
    buf.reshape(48, 80, 4)[..., :3] = arr
    out = W._rgb_from_rgbx(buf, 80, 48)
    assert out.mode == "RGB" and out.readonly and np.array_equal(np.asarray(out), arr)
    assert W._rgbx_view(out)[0] == buf.ctypes.data
    assert W._take_out(48 * 80 * 4) is not buf  # still referenced by the image
    out.paste((1, 2, 3), (0, 0, 4, 4))  # PIL copies first: the buffer is no longer the image's
    assert not out.readonly and W._rgbx_view(out)[0] != buf.ctypes.data
    where = buf.ctypes.data
    del out, buf  # the pool counts every reference, this test's own included
    gc.collect()
    assert W._take_out(48 * 80 * 4).ctypes.data == where


def test_pool_finalizer_runs_under_the_pool_lock():
    """an output image in a reference cycle is finalized by whichever thread triggers
    the cyclic GC -- possibly one that holds _pool_lock (in _take_out).  The finalizer must not
    take the lock (a plain Lock would deadlock the thread on itself)."""
    import threading

    if W._arrow() is None:
        pytest.skip("zero-copy path unavailable (pyarrow / Pillow Arrow interface)")
    buf = W._take_out(16 * 16 * 4)
    img = W._rgb_from_rgbx(buf, 16, 16)
    cyc = [img]
    cyc.append(cyc)  # collectable only by the cyclic GC
    del img, cyc, buf
    done = threading.Event()

    def run():
        with W._pool_lock:
            gc.collect()  # the image's finalizer runs here, inside the locked region
        done.set()

    t = threading.Thread(target=run, daemon=True)
    t.start()
    assert done.wait(10), "finalizer deadlocked on _pool_lock"
    assert W._take_out(16 * 16 * 4) is not None


def test_pool_buffer_returned_after_failed_call(monkeypatch):
    """a pooled buffer whose C call raised (no image built) is free again."""
    if W._arrow() is None:
        pytest.skip("zero-copy path unavailable (pyarrow / Pillow Arrow interface)")
    n = 24 * 40 * 4
    W._out_pool.pop(n, None)
    buf = W._take_out(n)
    where = buf.ctypes.data
    W._give_back(buf)
    del buf
    gc.collect()
    assert W._take_out(n).ctypes.data == where


def test_zero_copy_needs_pillow_arrow(monkeypatch):
    """Pillow < 11.2 has no Image.fromarrow / __arrow_c_array__ (the reference allows Pillow >= 9,
    requirements.txt:3): the drop-in must then take the copying path, pyarrow or not."""
    monkeypatch.setattr(W, "_pa", None)
    monkeypatch.setattr(W, "_zero_copy", True)
    monkeypatch.delattr(Image, "fromarrow", raising=False)
    assert W._arrow() is None and W._zero_copy is False
    assert W._rgbx_view(Image.new("RGB", (8, 8))) is None
