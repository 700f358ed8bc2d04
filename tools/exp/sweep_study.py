#!/usr/bin/env python3
"""How many f32 Jacobi sweeps should phase 1 of the hybrid route's SVD run?

The oracle is compiled with JAC32_MAX_SWEEPS = 2..5 (gcc, into a temporary directory; the same
source the tests use) and run on the DCT blocks of covers (the bench's uniform noise and
camera-like).  Per block it reports the f32 sweeps, the f64 sweeps and whether the Newton finish
ended the loop; per wave of embed_kernel<b> (64 / L consecutive blocks of a block row) it models
what the device runs: the f32 sweeps until no block of the wave rotates (capped), and the f64
sweeps until at most kDeferMax blocks of the wave are unfinished (b = 8: those go to the list
pass).  With per-sweep cycle costs from the phase stamps (profiles/r04/r04c/stamps_b8.log) it
predicts the SVD phases' cycles per wave.  It also counts the blocks whose f32 factors differ
from the shipped setting's (4), i.e. how far the contract would move.

usage: sweep_study.py --block 8 --height 1080 --width 1920 --frames 2"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from oracle import oracle as O  # noqa: E402
from lapack_path import _blocks, photo_cover  # noqa: E402

L_OF = {4: 1, 6: 2, 8: 2, 10: 4, 12: 4, 14: 8, 16: 8}
DEFER = {8: 4}


def build(n, d):
    path = os.path.join(d, f"orc_s{n}.so")
    src = [os.path.join(ROOT, "oracle", f) for f in ("tmfwm_oracle.c", "tmfwm_lapack.c")]
    subprocess.run(["gcc", "-O2", "-fPIC", "-fopenmp", "-ffp-contract=off", "-fno-fast-math", "-std=c11",
                    f"-DJAC32_MAX_SWEEPS={n}", "-shared", "-o", path] + src + ["-lm"], check=True)
    lib = ctypes.CDLL(path)
    lib.orc_svd_blocks.restype = ctypes.c_int
    O.lib()  # loads the hardware rsq table (O._rsq_delta), which every copy of the oracle needs
    lib.orc_set_rsq_table.restype = None
    lib.orc_set_rsq_table.argtypes = [ctypes.c_void_p]
    lib.orc_set_rsq_table(O._rsq_delta.ctypes.data)
    return lib


def svd(lib, D):
    b = D.shape[-1]
    nb = D.shape[0]
    U = np.empty_like(D)
    Vt = np.empty_like(D)
    S = np.empty((nb, b), np.float32)
    sw = np.empty(nb, np.int32)
    f = ctypes.c_void_p
    lib.orc_svd_blocks(f(D.ctypes.data), ctypes.c_int64(nb), b, f(U.ctypes.data), f(S.ctypes.data), f(Vt.ctypes.data),
                       f(sw.ctypes.data))
    return U, S, Vt, sw


def waves(sw, nbw, b):
    """per wave: (f32 sweeps run, f64 sweeps run) under the device's rules"""
    bpw = 64 // L_OF[b]
    s64 = sw & 0xFF
    s32 = (sw >> 8) & 0xFF
    nwt = (sw >> 16) & 1
    # sweeps after which the block is finished: a Newton finish ends it after sweep s64; a
    # converged block's last counted sweep is the one without rotation (nothing left to do after
    # the previous one, but the wave still runs that sweep to see it)
    fin = s64
    out = []
    nbh = len(sw) // nbw
    for r in range(nbh):
        row = slice(r * nbw, (r + 1) * nbw)
        for w0 in range(0, nbw, bpw):
            f = fin[row][w0:w0 + bpw]
            k32 = int(s32[row][w0:w0 + bpw].max())
            d = DEFER.get(b, 0)
            srt = np.sort(f)[::-1]
            k64 = int(srt[d]) if d and len(srt) > d else int(srt[0])
            out.append((k32, max(k64, 1), int(nwt[row][w0:w0 + bpw].min())))
    return np.array(out)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--block", type=int, default=8)
    p.add_argument("--height", type=int, default=1080)
    p.add_argument("--width", type=int, default=1920)
    p.add_argument("--frames", type=int, default=2)
    p.add_argument("--sweeps", default="2,3,4,5")
    a = p.parse_args()
    b, H, W = a.block, a.height, a.width
    d = tempfile.mkdtemp()
    libs = {n: build(n, d) for n in map(int, a.sweeps.split(","))}
    for kind in ("noise", "photo"):
        Ds = []
        for f in range(a.frames):
            cov = (O.synth_bytes(0x5EED0001, f, 1, H * W * 3).reshape(H, W, 3) if kind == "noise" else photo_cover(H, W, 500 + f))
            Ds.append(O.dct2d_blocks(_blocks(O.rgb_to_ycbcr(cov)[..., 0], b)))
        D = np.ascontiguousarray(np.concatenate(Ds))
        base = None
        res = {}
        for n, lib in libs.items():
            U, S, Vt, sw = svd(lib, D)
            wv = np.concatenate([waves(sw[i * len(D) // a.frames:(i + 1) * len(D) // a.frames], W // b, b) for i in range(a.frames)])
            res[n] = dict(U=U, S=S, Vt=Vt, sw=sw, wv=wv)
            if n == 4:
                base = res[n]
        for n, r in res.items():
            diff = ~(np.all(r["U"] == base["U"], axis=(1, 2)) & np.all(r["S"] == base["S"], axis=1) & np.all(r["Vt"] == base["Vt"], axis=(1, 2)))
            s64 = r["sw"] & 0xFF
            wv = r["wv"]
            print(json.dumps({"kind": kind, "block": b, "f32_sweeps_max": n, "blocks": int(len(D)),
                              "block_f64_sweeps_hist": {int(k): int(v) for k, v in zip(*np.unique(s64, return_counts=True))},
                              "block_newton_frac": round(float(((r["sw"] >> 16) & 1).mean()), 4),
                              "wave_f32_sweeps_mean": round(float(wv[:, 0].mean()), 3),
                              "wave_f64_sweeps_mean": round(float(wv[:, 1].mean()), 3),
                              "wave_f64_sweeps_hist": {int(k): int(v) for k, v in zip(*np.unique(wv[:, 1], return_counts=True))},
                              "blocks_factors_differ_from_4": int(diff.sum())}), flush=True)


if __name__ == "__main__":
    main()
