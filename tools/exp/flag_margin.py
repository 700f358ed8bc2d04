"""Margin of the hybrid route's conditioning flag: over whole 4K frames of
noise and camera-like covers, per block: flagged?, IDCT output bits differ between the
Jacobi and dgesdd routes?, output bytes differ?, and the block's amplification
sigma_1 / m (m = min over triplets reaching the output of min(sigma_k, gap_k); flagged iff
sigma_1 / m > 2^20).  Prints counts and the largest amplification of any block whose bits
diverge.  usage: flag_margin.py B FRAMES_PER_KIND [H W]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import oracle as O  # noqa: E402
from lapack_path import _blocks, photo_cover  # noqa: E402


def amplification(sig):
    """sigma_1 / m per block (orc_svd_flag's quantity); inf for m == 0, 0 for zero blocks."""
    s1 = sig.max(axis=1)
    keep = sig.astype(np.float32) != 0
    d = np.abs(sig[:, :, None] - sig[:, None, :])
    b = sig.shape[1]
    d[:, np.arange(b), np.arange(b)] = np.inf
    g = np.minimum(sig, d.min(axis=2))
    g = np.where(keep, g, np.inf)
    m = np.minimum(g.min(axis=1), s1)
    with np.errstate(divide="ignore", invalid="ignore"):
        a = np.where(s1 == 0, 0.0, s1 / m)
    return a


def flags_of(sig):
    """orc_svd_flag over blocks, vectorised: m * 2^20 < sigma_1 (zero blocks never)."""
    s1 = sig.max(axis=1)
    a = amplification(sig)
    return (s1 > 0) & (a > 2.0**20)


def frame_stats(cov, tile, b, alpha=0.1):
    H, W = cov.shape[:2]
    D = O.dct2d_blocks(_blocks(O.rgb_to_ycbcr(cov)[..., 0], b))
    U64, sig, V64 = O.svd_blocks_f64(D)  # the Jacobi route before rounding (orc_svd_block rounds these)
    J = (U64.astype(np.float32), sig.astype(np.float32), np.ascontiguousarray(np.swapaxes(V64, 1, 2)).astype(np.float32))
    Lp = O.lp_svd_blocks(D)
    t = tile.reshape(-1)
    Yj, Yl = (O.dct2d_blocks(O.blend_reconstruct_blocks(*f, t, alpha), inverse=True) for f in (J, Lp))
    ydiff = ~np.all((Yj.view(np.uint32) == Yl.view(np.uint32)).reshape(len(D), -1), axis=1)
    amp = amplification(sig)
    flags = flags_of(sig)
    ej = O.embed_frame(cov, tile, b, alpha, route="jacobi")
    el = O.embed_frame(cov, tile, b, alpha, route="lapack")
    nbh, nbw = H // b, W // b
    bd = (ej != el)[: nbh * b, : nbw * b].reshape(nbh, b, nbw, b, 3).any(axis=(1, 3, 4)).reshape(-1)
    return len(D), flags, ydiff, bd, amp


def main():
    b, n = int(sys.argv[1]), int(sys.argv[2])
    H, W = (int(x) for x in sys.argv[3:5]) if len(sys.argv) > 4 else (2160, 3840)
    tot = {}
    for kind in ("noise", "photo"):
        for f in range(n):
            t0 = time.time()
            if kind == "noise":
                cov = O.synth_bytes(0x5EED0001, f, 1, H * W * 3).reshape(H, W, 3)
            else:
                cov = photo_cover(H, W, 100 + f)
            tile = O.synth_bytes(0x5EED0002, f, 1, (H // b) * (W // b)).reshape(H // b, W // b)
            nb, flags, yd, bd, amp = frame_stats(cov, tile, b)
            t = tot.setdefault(kind, {"blocks": 0, "flagged": 0, "ydiff_unflagged": 0, "bytediff_unflagged": 0,
                                      "ydiff_flagged": 0, "max_amp_ydiff_unflagged": 0.0, "max_amp_unflagged": 0.0})
            t["blocks"] += nb
            t["flagged"] += int(flags.sum())
            t["ydiff_unflagged"] += int((yd & ~flags).sum())
            t["bytediff_unflagged"] += int((bd & ~flags).sum())
            t["ydiff_flagged"] += int((yd & flags).sum())
            if (yd & ~flags).any():
                t["max_amp_ydiff_unflagged"] = max(t["max_amp_ydiff_unflagged"], float(amp[yd & ~flags].max()))
            t["max_amp_unflagged"] = max(t["max_amp_unflagged"], float(amp[~flags].max()))
            print(kind, f, f"{time.time() - t0:.1f}s", t, flush=True)
    print({"b": b, **tot})


if __name__ == "__main__":
    main()
