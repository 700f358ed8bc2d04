#!/usr/bin/env python3
"""extract at b = 4 on 64 synthetic 4K frames: the work split (list-pass and dgesdd-route blocks)
and the per-launch kernel times (HIP events around one extract_batch call)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from thatsmyface_amd import batch  # noqa: E402

dev = torch.device("cuda", 0)
for b in (4, 6, 8):
    fr = batch.synth_frames(64, 2160, 3840, device=dev)
    tile = batch.synth_tile(2160 // b, 3840 // b, device=dev)
    out = batch.embed_batch(fr, tile, b, 0.1)
    st = {}
    ext = batch.extract_batch(out, fr, b, 0.1, stats=st)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    batch.extract_batch(out, fr, b, 0.1, out=ext)
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"block": b, "blocks": 64 * (2160 // b) * (3840 // b), "extract_stats": st,
                      "extract_us_per_frame": round(e0.elapsed_time(e1) * 1000 / 64, 1)}), flush=True)
