#!/usr/bin/env python3
"""Summarise tools/pmc_embed.sh output: per-wave counter values of one kernel.
Usage: python tools/pmc_summary.py <outdir>... [--kernel embed_kernel]"""
import csv
import glob
import os
import sys


def load(d, kernel):
    agg = {}
    for f in glob.glob(os.path.join(d, "p*", "p_counter_collection.csv")):
        rows = list(csv.DictReader(open(f)))
        disp = {}
        for r in rows:
            if kernel in r["Kernel_Name"]:
                disp.setdefault(r["Dispatch_Id"], {})[r["Counter_Name"]] = float(r["Counter_Value"])
        if disp:  # last dispatch of the kernel (the timed one)
            last = disp[max(disp, key=int)]
            agg.update(last)
    return agg


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    kernel = "embed_kernel"
    for a in sys.argv[1:]:
        if a.startswith("--kernel="):
            kernel = a.split("=", 1)[1]
    data = {os.path.basename(d.rstrip("/")): load(d, kernel) for d in args}
    keys = sorted({k for v in data.values() for k in v})
    print(f"{'counter':28s}" + "".join(f"{n[:18]:>20s}" for n in data))
    for k in keys:
        row = f"{k:28s}"
        for v in data.values():
            w = v.get("SQ_WAVES", 1)
            x = v.get(k)
            row += f"{(x / w if k != 'SQ_WAVES' else x) if x is not None else float('nan'):20.1f}"
        print(row)


if __name__ == "__main__":
    main()
