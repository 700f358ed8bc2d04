#!/usr/bin/env python3
"""VALU-issue roofline of the embed / extract kernels from SQ instruction counters.

Inputs: tools/pmc_embed.sh output directories (three rocprofv3 --pmc passes over
tools/time_embed.py) and the issue costs measured by tools/micro/chain_rate.hip on
MI355X (profiles/r01e_valu_chain_rate.log): with enough independent work per SIMD an
f64 FMA issues every ~5.0 cycles and an f32 FMA every ~2.8 cycles (2.4 GHz clock).
Every f64 arithmetic instruction (SQ_INSTS_VALU_{FMA,MUL,ADD,TRANS}_F64) is priced at
the f64 cost, every other VALU instruction at the f32 cost.  The estimate is the time
one SIMD needs to ISSUE its share of the frame's waves; bench.py divides it by the
measured launch time (fraction of the VALU-issue bound).

Usage: python tools/valu.py <pmc_dir> --frames 16 --height 2160 --width 3840 --block 8 --out profiles/valu.json
"""
import argparse
import csv
import glob
import json
import os

F64_CYC, OTHER_CYC, CLOCK_HZ, SIMDS = 5.0, 2.8, 2.4e9, 1024
F64 = ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_TRANS_F64")


def per_wave(d, kernel):
    agg = {}
    for f in glob.glob(os.path.join(d, "p*", "p_counter_collection.csv")):
        disp = {}
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"]:
                disp.setdefault(int(r["Dispatch_Id"]), {})
                c = disp[int(r["Dispatch_Id"])]
                c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        if disp:
            agg.update(disp[max(disp)])  # the timed (last) dispatch
    waves = agg["SQ_WAVES"]
    return {k: v / waves for k, v in agg.items() if k != "SQ_WAVES"}, waves


def main():
    p = argparse.ArgumentParser()
    p.add_argument("pmc_dir")
    p.add_argument("--frames", type=int, default=16)
    p.add_argument("--height", type=int, default=2160)
    p.add_argument("--width", type=int, default=3840)
    p.add_argument("--block", type=int, default=8)
    p.add_argument("--out", default="profiles/valu.json")
    a = p.parse_args()
    out = {"source": f"{a.pmc_dir} (tools/pmc_embed.sh, {a.frames} frames {a.width}x{a.height}, b={a.block})",
           "issue_cost_cycles": {"f64_arith": F64_CYC, "other_valu": OTHER_CYC,
                                 "from": "tools/micro/chain_rate.hip, profiles/r01e_valu_chain_rate.log"},
           "clock_hz": CLOCK_HZ, "simds": SIMDS, "kernels": {}}
    for k in ("embed_kernel", "extract_kernel"):
        pw, waves = per_wave(a.pmc_dir, k)
        f64 = sum(pw.get(c, 0.0) for c in F64)
        valu = pw["SQ_INSTS_VALU"]
        cyc = f64 * F64_CYC + (valu - f64) * OTHER_CYC
        wpf = waves / a.frames
        us = cyc * wpf / SIMDS / CLOCK_HZ * 1e6
        out["kernels"][f"{k}<{a.block}>"] = {
            "valu_instr_per_wave": round(valu, 1), "f64_instr_per_wave": round(f64, 1),
            "waves_per_frame": wpf, "issue_cycles_per_wave": round(cyc, 1),
            "valu_issue_bound_us_per_frame": round(us, 2)}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out["kernels"], indent=1))


if __name__ == "__main__":
    main()
