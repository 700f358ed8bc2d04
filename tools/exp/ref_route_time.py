#!/usr/bin/env python3
"""Throughput of the reference route (TMFWM_ROUTE_REFERENCE: the dgesdd route on every block)
for library variants, one child process per variant and round (TMFWM_LIB is read at load):
us per 1080p frame for embed and extract, and a hash of the outputs (variants must agree).
usage: ref_route_time.py --block 8 --frames 16 --rounds 2 name1 name2 ...  (variants/libtmfwm_<name>.so)"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CHILD = r'''
import hashlib, json, os, sys, torch
sys.path.insert(0, os.environ["ROOT"])
from thatsmyface_amd import batch
b, n = int(sys.argv[1]), int(sys.argv[2])
dev = torch.device("cuda", 0)
fr = batch.synth_frames(n, 1080, 1920, device=dev)
tile = batch.synth_tile(1080 // b, 1920 // b, device=dev)
out = batch.embed_batch(fr, tile, b, 0.1, route="reference")
ext = batch.extract_batch(out, fr, b, 0.1, route="reference")
torch.cuda.synchronize()
h = hashlib.sha256(out.cpu().numpy().tobytes() + ext.cpu().numpy().tobytes()).hexdigest()[:16]
res = {}
for name, fn in (("embed", lambda: batch.embed_batch(fr, tile, b, 0.1, out=out, route="reference")),
                 ("extract", lambda: batch.extract_batch(out, fr, b, 0.1, out=ext, route="reference"))):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    res[name] = round(e0.elapsed_time(e1) * 1000 / n, 1)
print(json.dumps({"hash": h, "us_per_1080p_frame": res}))
'''


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--block", type=int, default=8)
    p.add_argument("--frames", type=int, default=16)
    p.add_argument("--rounds", type=int, default=2)
    p.add_argument("names", nargs="+")
    a = p.parse_args()
    for r in range(a.rounds):
        for name in a.names:
            env = dict(os.environ, ROOT=ROOT, TMFWM_LIB=os.path.join(ROOT, "variants", f"libtmfwm_{name}.so"))
            out = subprocess.run([sys.executable, "-c", CHILD, str(a.block), str(a.frames)], env=env, capture_output=True,
                                 text=True, timeout=600)
            line = out.stdout.strip().splitlines()[-1] if out.returncode == 0 and out.stdout.strip() else None
            print(json.dumps({"round": r, "variant": name, "block": a.block,
                              "result": json.loads(line) if line else None,
                              "error": None if line else out.stderr[-800:]}), flush=True)
            if not line:
                raise SystemExit(1)


if __name__ == "__main__":
    main()
