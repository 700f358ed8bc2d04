"""Round 6: what the Newton finish's scaled acceptance test costs in sweeps.
Per-block f64 sweep counts of the oracle's Jacobi route with the round-5 test (|F| <= 2^-27
alone, orc_set_newton_scaled(0)) and with the scaled test (the contract, 1), on 1088 x 1920
frames of noise, camera-like and QR-module covers (tests/k_corpus.py) at b = 4, 8, 12, 16, and
the outlier block's Jacobi-vs-LAPACK ratio under both.  "wmax": the mean over 64/L-block waves of
the wave's slowest block (the device runs a wave until its slowest block is done).
usage: newton_sweeps.py > profiles/r06/newton_scaled_sweeps.log"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import k_corpus as kc  # noqa: E402

L = kc.O.lib()
MODES = (0, 1)
for on in MODES:
    L.orc_set_newton_scaled(on)
    D = np.load(os.path.join(ROOT, "tests", "golden", "k_newton_outlier_b8.npy"))[None]
    c, ru, rv, rs = kc.ratios(D)
    print("scaled", on, "outlier block u %.1f v %.1f" % (ru[0], rv[0]))
for b in (8, 16, 4, 12):
    for kind in ("noise", "photo", "qr"):
        D = kc.pixel_class(kind, b, 7, H=1088, W=1920)
        res = []
        for on in MODES:
            L.orc_set_newton_scaled(on)
            sw = kc.O.svd_blocks(D)[3]
            f64 = sw & 255
            lanes = {4: 1, 6: 2, 8: 2, 10: 4, 12: 4, 14: 8, 16: 8}[b]
            bpw = 64 // lanes
            n = len(f64) // bpw * bpw
            wv = f64[:n].reshape(-1, bpw).max(1)
            res.append("m%d %.3f wmax %.3f" % (on, f64.mean(), wv.mean()))
        print(b, kind, " | ".join(res), flush=True)
L.orc_set_newton_scaled(1)
