#!/usr/bin/env python3
"""Measure the truth tables of v_rsq_f32 / v_rcp_f32 on the GPU (tools/micro/trans_table)
and store them as deltas against a reference every CPU computes the same way:
    rsq: bits(hw(x)) - bits(f32(1.0 / sqrt(f64(x))))     for the 2^24 inputs x in [1, 4)
    rcp: bits(hw(x)) - bits(f32(1.0 / f64(x)))           for the 2^23 inputs x in [1, 2)
(IEEE f64 sqrt and divide, then one rounding to f32: numpy here, C in oracle/tmfwm_oracle.c).
Run on the GPU box: python tools/trans_table.py <outdir>  ->  <outdir>/trans_delta.npz + JSON."""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def references():
    i = np.arange(1 << 24, dtype=np.uint32)
    xr = (((127 + (i >> 23)) << 23) | (i & 0x7FFFFF)).view(np.float32)
    rsq = (1.0 / np.sqrt(xr.astype(np.float64))).astype(np.float32)
    j = np.arange(1 << 23, dtype=np.uint32)
    xc = ((127 << 23) | j).view(np.float32)
    rcp = (1.0 / xc.astype(np.float64)).astype(np.float32)
    return rsq, rcp


def main():
    out = sys.argv[1]
    os.makedirs(out, exist_ok=True)
    exe = os.path.join(ROOT, "tools", "micro", "trans_table")
    with tempfile.TemporaryDirectory() as d:
        r = subprocess.run([exe, d], capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            raise SystemExit(f"trans_table failed ({r.returncode}): {r.stderr}")
        stats = json.loads(r.stdout)
        hw_rsq = np.fromfile(os.path.join(d, "rsq.bin"), dtype=np.uint32)
        hw_rcp = np.fromfile(os.path.join(d, "rcp.bin"), dtype=np.uint32)
    ref_rsq, ref_rcp = references()
    d_rsq = hw_rsq.astype(np.int64) - ref_rsq.view(np.uint32).astype(np.int64)
    d_rcp = hw_rcp.astype(np.int64) - ref_rcp.view(np.uint32).astype(np.int64)
    for name, dd in (("rsq", d_rsq), ("rcp", d_rcp)):
        vals, cnt = np.unique(dd, return_counts=True)
        stats[f"{name}_delta_ulps"] = {str(int(v)): int(c) for v, c in zip(vals, cnt)}
    assert np.abs(d_rsq).max() < 128 and np.abs(d_rcp).max() < 128
    np.savez_compressed(os.path.join(out, "trans_delta.npz"), rsq=d_rsq.astype(np.int8), rcp=d_rcp.astype(np.int8))
    stats["npz_bytes"] = os.path.getsize(os.path.join(out, "trans_delta.npz"))
    print(json.dumps(stats))


if __name__ == "__main__":
    main()
