#!/usr/bin/env python3
"""Host-memory batch throughput of the multi-GPU entry points on one box:
tmfwm_embed_multi over --frames synthetic 4K frames in host memory, as 1 and 2 logical shards of
device 0, against the same frames through one tmfwm_embed host call (upload, kernels, download
back to back).  The multi path runs passes through two device slots, so a pass's PCIe traffic
overlaps its neighbour's kernels; the second call of each case reuses the cached slots.
Prints one JSON line per case: seconds and frames/s (best of --reps), and whether the outputs agree."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from thatsmyface_amd import _lib, multi  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--frames", type=int, default=96)
    p.add_argument("--height", type=int, default=2160)
    p.add_argument("--width", type=int, default=3840)
    p.add_argument("--block", type=int, default=8)
    p.add_argument("--reps", type=int, default=3)
    a = p.parse_args()
    H, W, b, n = a.height, a.width, a.block, a.frames
    rng = np.random.default_rng(3)
    frames = rng.integers(0, 256, (n, H, W, 3), dtype=np.uint8)
    tile = rng.integers(0, 256, (H // b, W // b), dtype=np.uint8)
    L = _lib.load()

    def single():
        out = np.empty_like(frames)
        _lib.check(L.tmfwm_embed(frames.ctypes.data, n, H, W, H * W * 3, tile.ctypes.data, b, 0.1, out.ctypes.data,
                                 _lib.MEM_HOST, None), "embed")
        return out

    cases = {"tmfwm_embed (host, one call)": single,
             "tmfwm_embed_multi, 1 shard": lambda: multi.embed_multi(frames, tile, b, 0.1, devices=[0]),
             "tmfwm_embed_multi, 2 logical shards": lambda: multi.embed_multi(frames, tile, b, 0.1, devices=[0, 0])}
    ref = None
    for name, fn in cases.items():
        times = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            out = fn()
            times.append(time.perf_counter() - t0)
        if ref is None:
            ref = out
        best = min(times)
        print(json.dumps({"case": name, "frames": n, "frame": f"{W}x{H}", "block": b, "best_s": round(best, 3),
                          "first_s": round(times[0], 3), "frames_per_s": round(n / best, 1),
                          "host_GB_per_s": round(2 * frames.nbytes / best / 1e9, 2),
                          "equal_to_first_case": bool(np.array_equal(out, ref))}), flush=True)


if __name__ == "__main__":
    main()
