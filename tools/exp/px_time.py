#!/usr/bin/env python3
"""Host-memory latency of one 1080p embed call by pixel layout (tmfwm_embed_px, ABI 8): 3- or
4-byte pixels in and out, the input in PIL's own memory (Image.__arrow_c_array__) or in a numpy
copy, and the route.  Median ms over --reps calls; one JSON line per case."""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
from PIL import Image  # noqa: E402

from thatsmyface_amd import _lib  # noqa: E402
from thatsmyface_amd import watermarking as W  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--height", type=int, default=1080)
    p.add_argument("--width", type=int, default=1920)
    p.add_argument("--block", type=int, default=8)
    p.add_argument("--reps", type=int, default=30)
    a = p.parse_args()
    H, W_, b = a.height, a.width, a.block
    rng = np.random.default_rng(1)
    img = Image.fromarray(rng.integers(0, 256, (H, W_, 3), dtype=np.uint8))
    view = W._rgbx_view(img)
    rgb = np.ascontiguousarray(np.asarray(img))
    rgbx = np.frombuffer(img.tobytes("raw", "RGBX"), np.uint8).copy()
    tile = rng.integers(0, 256, (H // b, W_ // b), dtype=np.uint8)
    out3 = np.empty(H * W_ * 3, np.uint8)
    out4 = np.empty(H * W_ * 4, np.uint8)
    L = _lib.load()

    def timed(fn):
        fn()
        t = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            fn()
            t.append((time.perf_counter() - t0) * 1e3)
        return round(statistics.median(t), 3)

    def px(src, ipx, out, opx, route):
        return lambda: _lib.check(L.tmfwm_embed_px(src, ipx, H * W_ * ipx, 1, H, W_, tile.ctypes.data, b, 0.1, out.ctypes.data, opx,
                                                   H * W_ * opx, _lib.MEM_HOST, None, route, None), "px")

    cases = {
        "rgb->rgb (tmfwm_embed_route)": (rgb.ctypes.data, 3, out3, 3),
        "rgbx(numpy)->rgbx": (rgbx.ctypes.data, 4, out4, 4),
        "rgbx(PIL memory)->rgbx": (view[0] if view else 0, 4, out4, 4),
        "rgb->rgbx": (rgb.ctypes.data, 3, out4, 4),
        "rgbx(numpy)->rgb": (rgbx.ctypes.data, 4, out3, 3),
    }
    for route in (0, 1):
        for name, (src, ipx, out, opx) in cases.items():
            if not src:
                continue
            print(json.dumps({"case": name, "route": ["hybrid", "reference"][route], "frame": f"{W_}x{H}",
                              "pil_address_mod_64": (view[0] % 64) if view else None,
                              "median_ms": timed(px(src, ipx, out, opx, route))}), flush=True)


if __name__ == "__main__":
    main()
