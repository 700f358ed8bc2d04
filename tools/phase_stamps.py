#!/usr/bin/env python3
"""Phase profile of embed_kernel<b>: per-wave s_memtime cycles per kernel phase.

Needs the opt-in build `make -C thatsmyface_amd/csrc stamps` (libtmfwm_stamps.so,
compiled with -DTMF_STAMPS).  Phases: 0 load+luma+DCT, 1 f32 Jacobi, 2 Bjorck+D*V,
3 f64 Jacobi, 4 sigma/U/sort/blend/reconstruct, 5 IDCT, 6 colour+store.
Usage: python tools/phase_stamps.py [--frames 64] [--block 8]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["TMFWM_LIB"] = os.environ.get("TMF_STAMPS_LIB") or os.path.join(ROOT, "thatsmyface_amd", "libtmfwm_stamps.so")

import torch  # noqa: E402

from thatsmyface_amd import _lib, batch  # noqa: E402

NAMES = ["load+luma+dct", "f32 jacobi", "bjorck+DV", "f64 jacobi", "post+reconstruct", "idct", "colour+store"]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--frames", type=int, default=64)
    p.add_argument("--block", type=int, default=8)
    p.add_argument("--height", type=int, default=2160)
    p.add_argument("--width", type=int, default=3840)
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    b = a.block
    frames = batch.synth_frames(a.frames, a.height, a.width, device=dev)
    tile = batch.synth_tile(a.height // b, a.width // b, device=dev)
    L = _lib.load()
    # embed_kernel<8> lives in its own TU (tmfwm_embed8.hip) with its own copy of the stamps
    rd = L.tmfwm_debug_stamps_e8 if b == 8 and hasattr(L, "tmfwm_debug_stamps_e8") else L.tmfwm_debug_stamps
    rd.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = (ctypes.c_ulonglong * 16)()
    out = batch.embed_batch(frames, tile, b, 0.1)
    torch.cuda.synchronize()
    rd(buf, 1)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    batch.embed_batch(frames, tile, b, 0.1, out=out)
    ev1.record()
    torch.cuda.synchronize()
    rd(buf, 1)
    bpw = {4: 64, 8: 32, 16: 8}[b]
    nbw, nbh = a.width // b, a.height // b
    gx = nbh * ((nbw + bpw - 1) // bpw)
    waves = a.frames * ((gx + 63) // 64)  # the kernel samples blockIdx.x % 64 == 0
    tot = sum(buf[:7])
    res = {n: round(buf[i] / waves) for i, n in enumerate(NAMES)}
    print(json.dumps({"block": b, "frames": a.frames, "waves": waves, "ms": ev0.elapsed_time(ev1),
                      "cycles_per_wave": res, "total_per_wave": round(tot / waves),
                      "share": {n: round(buf[i] / tot, 3) for i, n in enumerate(NAMES)}}))


if __name__ == "__main__":
    main()
