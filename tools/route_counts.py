#!/usr/bin/env python3
"""How many blocks take the dgesdd route (second pass) in embed / extract on the bench's
synthetic frames: python tools/route_counts.py [--frames N] [--block b]."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from thatsmyface_amd import batch  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--frames", type=int, default=64)
p.add_argument("--height", type=int, default=2160)
p.add_argument("--width", type=int, default=3840)
p.add_argument("--block", type=int, default=8)
a = p.parse_args()
dev = torch.device("cuda", 0)
fr = batch.synth_frames(a.frames, a.height, a.width, device=dev)
tile = batch.synth_tile(a.height // a.block, a.width // a.block, device=dev)
for rep in range(2):
    st, xs = {}, {}
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = batch.embed_batch(fr, tile, a.block, 0.1, stats=st)
    t1 = time.perf_counter()
    batch.extract_batch(out, fr, a.block, 0.1, stats=xs)
    t2 = time.perf_counter()
nb = a.frames * (a.height // a.block) * (a.width // a.block)
print(f"frames={a.frames} b={a.block} blocks={nb} embed dgesdd-route blocks={st['lapack_blocks']} "
      f"({st['lapack_blocks'] / nb:.2e}) extract={xs['lapack_blocks']} ({xs['lapack_blocks'] / nb:.2e}) "
      f"embed {1e3 * (t1 - t0):.1f} ms extract {1e3 * (t2 - t1):.1f} ms", flush=True)
