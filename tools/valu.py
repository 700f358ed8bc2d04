#!/usr/bin/env python3
"""VALU-issue roofline of the embed / extract kernels from rocprofv3 counters.

Input: one tools/pmc_embed.sh output directory (passes p1-p6 over tools/time_embed.py at
one block size, recorded in <dir>/block).  For the timed (last) dispatch of each kernel:

* instruction mix per wave (SQ_INSTS_VALU and its f64 / transcendental classes);
* issue cycles per wave at the SPEC rates of a gfx950 SIMD-32 (MI355X_MICROARCH.md: a
  wave64 VALU instruction issues over 2 cycles; FP64 vector is half rate, 78.6 vs 157.3
  TFLOP/s, so 4 cycles for f64 FMA / MUL / ADD; a transcendental costs twice a plain op
  in the guide's issue-cost row, 4 cycles f32; f64 transcendentals priced at 8 -- that
  class is not in the guide, so the bound is approximate there, ~1 % of embed's mix);
* the effective clock of that dispatch, GRBM_GUI_ACTIVE / 8 XCDs / its duration (guide,
  'DVFS give-back'), and the bound in microseconds per frame at that clock;
* HBM bytes per frame from FETCH_SIZE (x2, gfx950) and WRITE_SIZE (KB).

The bound is a floor: a kernel that issued VALU work back to back on every SIMD at the
spec rate would take that long.  bench.py reports bound / measured (issue fraction).

Usage: python tools/valu.py <pmc_dir> [--height 2160 --width 3840] --build <lib hash> --out profiles/valu.json
Entries for other block sizes already in --out (same build) are kept.
"""
import argparse
import csv
import glob
import json
import os
import re

SIMDS, XCDS = 1024, 8
CYC = {"plain": 2.0, "f64": 4.0, "trans_f32": 4.0, "trans_f64": 8.0}
F64 = ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64")


def last_dispatch(d, kernel, variant=None):
    """counter -> value and (start, end) ns of the last dispatch of `kernel` (e.g.
    "embed_kernel<8>"; variant "false" / "true": the strip / list pass instantiation
    embed_kernel<8, false> / <8, true>), over all passes."""
    base = re.escape(kernel[:-1])  # "embed_kernel<8"
    rx = re.compile(base + (r", true>" if variant == "true" else r"(, false)?>"))
    agg, span = {}, {}
    for f in sorted(glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True)):
        disp = {}
        for r in csv.DictReader(open(f)):
            if rx.search(r["Kernel_Name"]):
                k = int(r["Dispatch_Id"])
                c = disp.setdefault(k, {})
                c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                span[(f, k)] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
        if disp:
            k = max(disp)
            agg.update(disp[k])
            if "GRBM_GUI_ACTIVE" in disp[k]:
                agg["_ns"] = span[(f, k)][1] - span[(f, k)][0]
    return agg


def add_counters(a, b):
    """counters of two dispatches (the strip and list passes of one embed call) summed"""
    return {n: a.get(n, 0.0) + b.get(n, 0.0) for n in set(a) | set(b)}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("pmc_dir")
    p.add_argument("--height", type=int, default=2160)
    p.add_argument("--width", type=int, default=3840)
    p.add_argument("--build", default=None, help="sha256 prefix of the measured libtmfwm.so (bench.py lib_build)")
    p.add_argument("--ids", default="thatsmyface_amd/libtmfwm.kernels.json",
                   help="the measured build's kernel code ids (tools/kernel_ids.py, written by the Makefile)")
    p.add_argument("--out", default="profiles/valu.json")
    a = p.parse_args()
    block, frames = (int(v) for v in open(os.path.join(a.pmc_dir, "block")).read().split())
    ids = json.load(open(a.ids))["kernels"] if os.path.exists(a.ids) else {}
    out = {}
    if os.path.exists(a.out):
        old = json.load(open(a.out))
        if "spec_issue_cycles" in old:
            out = old  # entries are keyed by kernel and carry the code id they measured
    out.update({
        "build_id": a.build,
        "spec_issue_cycles": CYC,
        "model": "issue cycles per wave at the gfx950 spec rates (tools/valu.py docstring); effective clock from "
                 "GRBM_GUI_ACTIVE / 8 / dispatch time; HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE",
    })
    out.setdefault("kernels", {})
    H, W = a.height, a.width
    for k in ("embed_kernel", "extract_kernel"):
        c = last_dispatch(a.pmc_dir, f"{k}<{block}>", "false" if k == "embed_kernel" else None)
        lp = last_dispatch(a.pmc_dir, f"{k}<{block}>", "true") if k == "embed_kernel" else {}

        def mix(cc):
            """per-wave instruction classes and spec-rate issue cycles of one dispatch's counters"""
            w = cc["SQ_WAVES"]
            pw = {n: v / w for n, v in cc.items() if n.startswith("SQ_") and n != "SQ_WAVES"}
            f64 = sum(pw.get(n, 0.0) for n in F64)
            t32, t64 = pw.get("SQ_INSTS_VALU_TRANS_F32", 0.0), pw.get("SQ_INSTS_VALU_TRANS_F64", 0.0)
            plain = pw["SQ_INSTS_VALU"] - f64 - t32 - t64
            cyc = plain * CYC["plain"] + f64 * CYC["f64"] + t32 * CYC["trans_f32"] + t64 * CYC["trans_f64"]
            return pw, f64, t32, t64, cyc

        # per-wave figures: the strip pass (embed) / the kernel (extract); the bound and the time:
        # every dispatch of the call (embed's list pass, DESIGN.md 4, adds its waves' cycles)
        pw, f64, t32, t64, cyc = mix(c)
        valu = pw["SQ_INSTS_VALU"]
        waves = c["SQ_WAVES"]
        wpf = waves / frames
        total_cyc = cyc * waves
        tot = c
        if lp:
            lp_cyc = mix(lp)[4]
            total_cyc += lp_cyc * lp["SQ_WAVES"]
            tot = add_counters(c, lp)
        ns = tot.get("_ns")
        clock = tot["GRBM_GUI_ACTIVE"] / XCDS / (ns * 1e-9) if ns else None
        bound_cyc_frame = total_cyc / frames / SIMDS
        ent = {
            "frames": frames, "height": H, "width": W,
            "valu_instr_per_wave": round(valu, 1), "f64_arith_per_wave": round(f64, 1),
            "trans_f32_per_wave": round(t32, 1), "trans_f64_per_wave": round(t64, 1),
            "salu_per_wave": round(pw.get("SQ_INSTS_SALU", 0.0), 1), "lds_per_wave": round(pw.get("SQ_INSTS_LDS", 0.0), 1),
            "waves_per_frame": wpf,
            "issue_cycles_per_wave": round(cyc, 1),
            "issue_bound_cycles_per_frame": round(bound_cyc_frame),
            "profiled_us_per_frame": round(ns * 1e-3 / frames, 2) if ns else None,
            "clock_MHz": round(clock / 1e6) if clock else None,
            "valu_issue_bound_us_per_frame": round(bound_cyc_frame / clock * 1e6, 2) if clock else None,
            "wait_inst_any_frac": round(pw["SQ_WAIT_INST_ANY"] / pw["SQ_WAVE_CYCLES"], 3) if "SQ_WAVE_CYCLES" in pw else None,
        }
        if ns and clock:
            ent["issue_fraction_profiled"] = round(ent["valu_issue_bound_us_per_frame"] / ent["profiled_us_per_frame"], 3)
        if "FETCH_SIZE" in tot and "WRITE_SIZE" in tot:
            ent["hbm_bytes_per_frame"] = round((2 * tot["FETCH_SIZE"] + tot["WRITE_SIZE"]) * 1024 / frames)
        if lp:
            ent["list_pass"] = {"waves": lp["SQ_WAVES"], "valu_instr": lp["SQ_INSTS_VALU"],
                                "issue_cycles_share": round(1 - cyc * waves / total_cyc, 4),
                                "note": "per-wave figures are the strip pass's; the bound, the time and the "
                                        "HBM bytes include the list pass"}
        ent["code_id"] = ids.get(f"{k}<{block}>")
        ent["build_id"] = a.build
        out["kernels"][f"{k}<{block}>"] = ent
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({n: v for n, v in out["kernels"].items() if n.endswith(f"<{block}>")}, indent=1))


if __name__ == "__main__":
    main()
