#!/usr/bin/env python3
"""A/B of library variants on one box: for each ab/libtmfwm_<name>.so (built by
tools/build_variant.sh) time embed / extract on synthetic 4K frames and hash the outputs,
alternating the variants over several rounds (boxes and clocks drift; one call, one box).
Usage: python tools/ab_variants.py --block 16 --frames 64 --rounds 3 name1 name2 ...
Each measurement runs in a child process (TMFWM_LIB is read when the library loads)."""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import hashlib, json, os, sys, torch
sys.path.insert(0, os.environ["ROOT"])
from thatsmyface_amd import batch
b, n, kind = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
dev = torch.device("cuda", 0)
if kind == "photo":  # camera-like covers (tools/exp/flag_margin.py), 4 distinct frames repeated
    sys.path.insert(0, os.path.join(os.environ["ROOT"], "tools", "exp"))
    from flag_margin import photo_cover
    ph = torch.stack([torch.from_numpy(photo_cover(2160, 3840, 100 + k)) for k in range(4)]).to(dev)
    fr = ph.repeat((n + 3) // 4, 1, 1, 1)[:n].contiguous()
else:
    fr = batch.synth_frames(n, 2160, 3840, device=dev)
tile = batch.synth_tile(2160 // b, 3840 // b, device=dev)
out = batch.embed_batch(fr, tile, b, 0.1)
ext = batch.extract_batch(out, fr, b, 0.1)
torch.cuda.synchronize()
h = hashlib.sha256(out.cpu().numpy().tobytes() + ext.cpu().numpy().tobytes()).hexdigest()[:16]
res = {}
for name, fn in (("embed", lambda: batch.embed_batch(fr, tile, b, 0.1, out=out)),
                 ("extract", lambda: batch.extract_batch(out, fr, b, 0.1, out=ext))):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(2):
        fn()
    e1.record()
    torch.cuda.synchronize()
    res[name] = round(e0.elapsed_time(e1) * 1000 / 2 / n, 2)
se, sx = {}, {}
batch.embed_batch(fr, tile, b, 0.1, out=out, stats=se)
batch.extract_batch(out, fr, b, 0.1, out=ext, stats=sx)
print(json.dumps({"hash": h, "us_per_frame": res, "lapack_blocks": {"embed": se["lapack_blocks"], "extract": sx["lapack_blocks"]},
                  "list_pass_blocks": se.get("list_pass_blocks")}))
'''


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--block", type=int, default=8)
    p.add_argument("--frames", type=int, default=64)
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--cover", choices=("noise", "photo"), default="noise")
    p.add_argument("names", nargs="+")
    a = p.parse_args()
    res = {n: [] for n in a.names}
    hashes = {}
    for r in range(a.rounds):
        for n in a.names:
            env = dict(os.environ, ROOT=ROOT, TMFWM_LIB=os.path.join(ROOT, "ab", f"libtmfwm_{n}.so"))
            out = subprocess.run([sys.executable, "-c", CHILD, str(a.block), str(a.frames), a.cover], env=env, capture_output=True,
                                 text=True, timeout=300)
            if out.returncode != 0:
                print(json.dumps({"variant": n, "error": out.stderr[-2000:]}), flush=True)
                sys.exit(1)
            line = json.loads(out.stdout.strip().splitlines()[-1])
            hashes.setdefault(n, line["hash"])
            res[n].append(line["us_per_frame"])
            print(json.dumps({"round": r, "variant": n, **line}), flush=True)
    summary = {n: {k: round(min(x[k] for x in v), 2) for k in ("embed", "extract")} for n, v in res.items()}
    print(json.dumps({"block": a.block, "frames": a.frames, "best_us_per_frame": summary, "hashes": hashes,
                      "all_hashes_equal": len(set(hashes.values())) == 1}), flush=True)


if __name__ == "__main__":
    main()
