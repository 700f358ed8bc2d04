#!/usr/bin/env python3
"""App-path throughput: the embed page's per-image loop vs thatsmyface_amd.pipeline.

Both use the GPU drop-in; the difference is only the host stages.  Inputs: N
camera-like synthetic RGB images encoded as PNG (what the page receives), a 29x29
QR-like watermark as PNG bytes, preserve_ratio=True, b=8, alpha=0.1.
  sequential: for each image: decode -> embed_watermark -> PNG encode
              (embed_watermark_page.py:492-558 without its 0.1 s UI sleep)
  pipelined : pipeline.embed_images (decode / encode thread pools, side-stream GPU)
Prints one JSON line (images/s for both, equality of the PNG bytes).
"""
import argparse
import io
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
from PIL import Image  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--images", type=int, default=24)
    p.add_argument("--height", type=int, default=1080)
    p.add_argument("--width", type=int, default=1920)
    p.add_argument("--workers", type=int, default=16)
    a = p.parse_args()
    from lapack_path import photo_cover

    from thatsmyface_amd import pipeline
    from thatsmyface_amd import watermarking as W

    pngs = []
    for i in range(a.images):
        buf = io.BytesIO()
        Image.fromarray(photo_cover(a.height, a.width, i)).save(buf, format="PNG", compress_level=1)
        pngs.append(buf.getvalue())
    wbuf = io.BytesIO()
    Image.fromarray((np.random.default_rng(1).integers(0, 2, (29, 29)) * 255).astype(np.uint8), "L").save(wbuf, format="PNG")
    wm = wbuf.getvalue()
    settings = {"block_size": 8, "alpha": 0.1}
    pipeline.embed_images(pngs[:2], wm, True, settings, workers=a.workers)  # warm-up (library, tile, allocator)
    t0 = time.perf_counter()
    seq = []
    for data in pngs:
        img = Image.open(io.BytesIO(data))
        out = W.embed_watermark(img, wm, preserve_ratio=True, custom_settings=settings)
        buf = io.BytesIO()
        out.save(buf, format="PNG")
        seq.append(buf.getvalue())
    t_seq = time.perf_counter() - t0
    t0 = time.perf_counter()
    res = pipeline.embed_images(pngs, wm, True, settings, workers=a.workers)
    t_pipe = time.perf_counter() - t0
    print(json.dumps({"images": a.images, "size": f"{a.width}x{a.height}", "workers": a.workers,
                      "sequential_img_per_s": round(a.images / t_seq, 2), "pipelined_img_per_s": round(a.images / t_pipe, 2),
                      "speedup": round(t_seq / t_pipe, 2), "png_bytes_identical": all(r.png == s for r, s in zip(res, seq))}))


if __name__ == "__main__":
    main()
