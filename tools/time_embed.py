#!/usr/bin/env python3
"""Time embed/extract of one library build (TMFWM_LIB=path) on synthetic 4K frames.

Used to price kernel variants (e.g. sweep caps built with -DTMF_F32_SWEEPS=...):
prints one JSON line with microseconds per frame.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from thatsmyface_amd import batch  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--frames", type=int, default=128)
    p.add_argument("--block", type=int, default=8)
    p.add_argument("--reps", type=int, default=3)
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    b = a.block
    fr = batch.synth_frames(a.frames, 2160, 3840, device=dev)
    tile = batch.synth_tile(2160 // b, 3840 // b, device=dev)
    out = batch.embed_batch(fr, tile, b, 0.1)
    ext = batch.extract_batch(out, fr, b, 0.1)
    torch.cuda.synchronize()
    res = {}
    for name, fn in (("embed", lambda: batch.embed_batch(fr, tile, b, 0.1, out=out)),
                     ("extract", lambda: batch.extract_batch(out, fr, b, 0.1, out=ext))):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res[name] = round(e0.elapsed_time(e1) * 1000 / a.reps / a.frames, 2)
    print(json.dumps({"lib": os.path.basename(os.environ.get("TMFWM_LIB", "libtmfwm.so")), "block": b, "us_per_frame": res}))


if __name__ == "__main__":
    main()
