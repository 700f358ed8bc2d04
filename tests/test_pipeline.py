"""Batched app pipeline (thatsmyface_amd/pipeline.py): order, bytes and PNG output.

CPU: the oracle stands in for the device stage (test infrastructure only), so the
decode / ordered-device / encode overlap logic is checked without a GPU.
GPU: the real (HIP) stage against the oracle's prepare_tile + embed_frame + PNG per image.
"""
import io

import numpy as np
import pytest
from PIL import Image

from oracle import oracle as O
from thatsmyface_amd import pipeline


def _images(n, seed=0):
    from lapack_path import photo_cover

    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        h, w = [(96, 128), (120, 90), (96, 128), (64, 200)][i % 4]
        arr = photo_cover(h, w, seed + i) if i % 2 else rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        buf = io.BytesIO()
        Image.fromarray(arr).save(buf, format="PNG")
        out.append(buf.getvalue() if i % 3 else Image.fromarray(arr))
    return out


def _wm_png():
    buf = io.BytesIO()
    Image.fromarray((np.random.default_rng(9).integers(0, 2, (29, 29)) * 255).astype(np.uint8), "L").save(buf, format="PNG")
    return buf.getvalue()


def _oracle_stage(wm_png, block, alpha, preserve_ratio):
    grey = np.asarray(Image.open(io.BytesIO(wm_png)).convert("L"))

    def stage(rgb):
        tile = O.prepare_tile(grey, rgb.shape[0] // block, rgb.shape[1] // block, preserve_ratio)
        return O.embed_frame(rgb, tile, block, alpha), None

    return stage


def test_pipeline_order_and_png_cpu():
    imgs, wm = _images(7), _wm_png()
    res = pipeline.embed_images(imgs, wm, True, {"block_size": 8, "alpha": 0.1}, workers=4,
                                device_stage=_oracle_stage(wm, 8, 0.1, True))
    assert len(res) == len(imgs)
    for src, r in zip(imgs, res):
        rgb = pipeline._decode(src)
        grey = np.asarray(Image.open(io.BytesIO(wm)).convert("L"))
        ref = O.embed_frame(rgb, O.prepare_tile(grey, rgb.shape[0] // 8, rgb.shape[1] // 8, True), 8, 0.1)
        assert np.array_equal(r.pixels, ref)
        assert np.array_equal(np.asarray(Image.open(io.BytesIO(r.png))), ref)


@pytest.mark.gpu
def test_pipeline_matches_oracle_gpu():
    """The HIP device stage (prepare_tile + embed on the GPU) against the oracle's
    prepare_tile + embed_frame, and the PNG round trip of the result."""
    torch = pytest.importorskip("torch")
    assert torch.cuda.is_available()

    imgs, wm = _images(9, seed=5), _wm_png()
    grey = np.asarray(Image.open(io.BytesIO(wm)).convert("L"))
    for b, pr in ((8, True), (12, False)):
        settings = {"block_size": b, "alpha": 0.15}
        res = pipeline.embed_images(imgs, wm, pr, settings)
        for src, r in zip(imgs, res):
            rgb = pipeline._decode(src)
            tile = O.prepare_tile(grey, rgb.shape[0] // b, rgb.shape[1] // b, pr)
            from thatsmyface_amd.constants import SVD_ROUTE

            ref = O.embed_frame(rgb, tile, b, 0.15, route={"reference": "lapack", "hybrid": None}[SVD_ROUTE])
            assert np.array_equal(r.pixels, ref), (b, pr)
            assert np.array_equal(np.asarray(Image.open(io.BytesIO(r.png))), ref)
