#!/usr/bin/env python3
"""Latency of the app's per-image calls through the drop-in (host PIL images in, PIL out):
embed_watermark(img, qr_png_bytes, preserve_ratio=True) as the embed page calls it
(internal_pages/embed_watermark_page.py:529-531) and extract_watermark(wm, orig)
(extract_watermark_page.py:293-296), on a camera-like 1080p image and a QR watermark.
Also the same embed as a device-resident batch of one frame (batch.embed_batch), which
excludes PIL and PCIe.  Prints one JSON line (median ms over --reps calls after one warm-up)."""
import argparse
import io
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
from PIL import Image  # noqa: E402

from thatsmyface_amd import batch  # noqa: E402
from thatsmyface_amd import watermarking as W  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--reps", type=int, default=20)
    p.add_argument("--height", type=int, default=1080)
    p.add_argument("--width", type=int, default=1920)
    p.add_argument("--block", type=int, default=8)
    a = p.parse_args()
    from golden.gen_golden import wmark
    from lapack_path import photo_cover

    cover = Image.fromarray(photo_cover(a.height, a.width, 5))
    qr = Image.fromarray(wmark("qr", 300, 300, 3))
    buf = io.BytesIO()
    qr.save(buf, format="PNG")
    png = buf.getvalue()
    cs = {"block_size": a.block, "alpha": 0.1}

    def timed(fn):
        fn()
        t = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            fn()
            t.append((time.perf_counter() - t0) * 1e3)
        return round(statistics.median(t), 3)

    out = {}
    wm_img = W.embed_watermark(cover, png, True, cs)
    out["embed_watermark_ms"] = timed(lambda: W.embed_watermark(cover, png, True, cs))
    out["extract_watermark_ms"] = timed(lambda: W.extract_watermark(wm_img, cover, cs))
    rs = dict(cs, svd_route="reference")
    out["embed_watermark_reference_route_ms"] = timed(lambda: W.embed_watermark(cover, png, True, rs))
    out["extract_watermark_reference_route_ms"] = timed(lambda: W.extract_watermark(wm_img, cover, rs))
    r1 = dict(cs, svd_route="rank1_reference")  # round 6: the rank-1 pre-pass in front of the dgesdd route
    out["embed_watermark_rank1_reference_route_ms"] = timed(lambda: W.embed_watermark(cover, png, True, r1))
    out["extract_watermark_rank1_reference_route_ms"] = timed(lambda: W.extract_watermark(wm_img, cover, r1))
    r2 = dict(cs, svd_route="hybrid")
    out["embed_watermark_hybrid_route_ms"] = timed(lambda: W.embed_watermark(cover, png, True, r2))
    out["extract_watermark_hybrid_route_ms"] = timed(lambda: W.extract_watermark(wm_img, cover, r2))
    # the extract page's inputs are decoded uploads, not embed_watermark's own output image
    b2 = io.BytesIO()
    wm_img.save(b2, format="PNG")
    wm_dec = Image.open(io.BytesIO(b2.getvalue()))
    wm_dec.load()
    out["extract_watermark_decoded_ms"] = timed(lambda: W.extract_watermark(wm_dec, cover, cs))
    # the copying path (np.asarray in, Image.fromarray out), for comparison
    W._zero_copy = False
    out["embed_watermark_copying_path_ms"] = timed(lambda: W.embed_watermark(cover, png, True, cs))
    out["extract_watermark_copying_path_ms"] = timed(lambda: W.extract_watermark(wm_dec, cover, cs))
    W._zero_copy = True
    # where embed_watermark's time goes (its stages, each timed alone)
    from thatsmyface_amd import _lib
    rgb = np.ascontiguousarray(np.asarray(cover.convert("RGB"), dtype=np.uint8))
    wimg = Image.open(io.BytesIO(png))
    nbh, nbw = a.height // a.block, a.width // a.block
    tile = np.ascontiguousarray(np.asarray(W.resize_watermark(wimg, nbh, nbw, True), dtype=np.uint8))
    host_out = np.empty_like(rgb)
    view = W._rgbx_view(cover)
    out4 = np.empty(a.height * a.width * 4, np.uint8)
    L = _lib.load()
    stages = {
        "convert_rgb": lambda: cover.convert("RGB"),
        "asarray": lambda: np.ascontiguousarray(np.asarray(cover, dtype=np.uint8)),
        "png_decode": lambda: Image.open(io.BytesIO(png)).convert("L"),
        "resize_watermark": lambda: W.resize_watermark(wimg, nbh, nbw, True),
        "tmfwm_embed_host": lambda: _lib.check(L.tmfwm_embed(rgb.ctypes.data, 1, a.height, a.width, rgb.size, tile.ctypes.data,
                                                             a.block, 0.1, host_out.ctypes.data, _lib.MEM_HOST, None), "embed"),
        "fromarray": lambda: Image.fromarray(host_out),
        "rgbx_view": lambda: W._rgbx_view(cover),
        "fromarrow": lambda: W._rgb_from_rgbx(out4, a.width, a.height),
    }
    if view is not None:  # PIL holds the cover in one block (images up to ~16 MB)
        stages["tmfwm_embed_px_host"] = lambda: _lib.check(
            L.tmfwm_embed_px(view[0], 4, a.height * a.width * 4, 1, a.height, a.width, tile.ctypes.data, a.block, 0.1,
                             out4.ctypes.data, 4, a.height * a.width * 4, _lib.MEM_HOST, None, 0, None), "px")
    out["embed_stages_ms"] = {k: timed(f) for k, f in stages.items()}
    dev = torch.device("cuda", 0)
    fr = torch.from_numpy(np.asarray(cover)[None].copy()).to(dev)
    tile = batch.synth_tile(a.height // a.block, a.width // a.block, device=dev)
    res = torch.empty_like(fr)

    def dev_embed():
        batch.embed_batch(fr, tile, a.block, 0.1, out=res)
        torch.cuda.synchronize()
    out["device_embed_1frame_ms"] = timed(dev_embed)
    print(json.dumps({"image": f"{a.width}x{a.height} camera-like", "block": a.block, "reps": a.reps, **out}))


if __name__ == "__main__":
    main()
