#!/usr/bin/env python3
"""HBM bytes per kernel launch from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half of the
bytes of a coalesced streaming read -> doubled; WRITE_SIZE taken as is; both in KB.
Usage: python tools/traffic.py <fetch_csv> <write_csv> --frames 64 --height 2160 --width 3840
       --block 8 --out profiles/traffic.json
Writes per-frame bytes and per-launch bytes for the batch sizes bench.py uses.
"""
import argparse
import csv
import json


def kernel_values(path, counter):
    out = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"]
        key = "embed" if "embed_kernel" in name else "extract" if "extract_kernel" in name else None
        if key:
            out.setdefault(key, []).append(float(r["Counter_Value"]))
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("fetch_csv")
    p.add_argument("write_csv")
    p.add_argument("--frames", type=int, default=64)
    p.add_argument("--height", type=int, default=2160)
    p.add_argument("--width", type=int, default=3840)
    p.add_argument("--block", type=int, default=8)
    p.add_argument("--source", default="")
    p.add_argument("--out", default="profiles/traffic.json")
    a = p.parse_args()
    f = kernel_values(a.fetch_csv, "FETCH_SIZE")
    w = kernel_values(a.write_csv, "WRITE_SIZE")
    H, W, b = a.height, a.width, a.block
    nbh, nbw = H // b, W // b
    res = {
        "source": a.source or f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, bench.py --frames {a.frames} --steps 1 --warmup 0",
        "correction": "gfx950: FETCH_SIZE counts 1/2 of the bytes of a coalesced streaming read -> doubled; WRITE_SIZE as is; KB -> x1024",
        "algorithmic_bytes_per_frame": {"embed": 6 * H * W + nbh * nbw, "extract": 6 * H * W + nbh * nbw},
    }
    for k in ("embed", "extract"):
        per_frame = (2 * f[k][-1] + w[k][-1]) * 1024 / a.frames
        res[f"{k}_kernel_hbm_bytes_per_frame"] = round(per_frame)
        res[f"{k}_kernel_hbm_bytes_per_launch"] = {
            f"{n}x{H}x{W}_b{b}": round(per_frame * n) for n in (64, 128, 256, 512, 1024, 4096)}
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({k: v for k, v in res.items() if "per_frame" in k}))


if __name__ == "__main__":
    main()
