"""Study driver for the byte-level certificate (tools/exp/cert_byte.cpp).

Per frame (the bench's noise covers or camera-like covers; the bench's noise watermark):
  * the Jacobi route's f64 factors (oracle svd_blocks_f64) and the cover's Cb / Cr;
  * cert_blocks() at K = 0 must give the Jacobi route's own bytes (checks the interval code);
  * at each K: blocks whose bytes the certificate cannot decide ("fail"), and the soundness
    check: every certified block's bytes equal the dgesdd route's (np.linalg.svd's arithmetic).
usage: cert_byte.py B FRAMES_PER_KIND [H W] [K ...]"""
import ctypes
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import oracle as O  # noqa: E402
from lapack_path import _blocks, photo_cover  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
SO = "/tmp/cert_byte.so"


def lib():
    src = os.path.join(HERE, "cert_byte.cpp")
    if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(src):
        subprocess.run(["g++", "-O2", "-fopenmp", "-ffp-contract=off", "-fno-fast-math", "-std=c++17", "-shared", "-fPIC",
                        "-I", os.path.join(ROOT, "thatsmyface_amd", "csrc"), src, "-o", SO], check=True)
    L = ctypes.CDLL(SO)
    L.cert_blocks.restype = ctypes.c_int
    return L


def p(a):
    assert a.flags["C_CONTIGUOUS"]
    return ctypes.c_void_p(a.ctypes.data)


def cert(L, Uj, sj, Vj, w, alpha, cb, cr, K):
    nb, b = sj.shape
    flag = np.zeros(nb, np.uint8)
    byts = np.zeros((nb, b, b, 3), np.uint8)
    st = np.zeros(3, np.int64)
    rc = L.cert_blocks(ctypes.c_int64(nb), b, p(Uj), p(sj), p(Vj), p(w), ctypes.c_double(alpha), p(cb), p(cr),
                       ctypes.c_double(K), p(flag), p(byts), p(st))
    assert rc == 0
    return flag.astype(bool), byts, st


def block_bytes(rgb, b):
    H, W = rgb.shape[:2]
    nbh, nbw = H // b, W // b
    return np.ascontiguousarray(rgb[: nbh * b, : nbw * b].reshape(nbh, b, nbw, b, 3).transpose(0, 2, 1, 3, 4).reshape(-1, b, b, 3))


def study(L, cov, tile, b, alpha, Ks):
    ycc = O.rgb_to_ycbcr(cov)
    D = O.dct2d_blocks(_blocks(ycc[..., 0], b))
    Uj, sj, Vj = O.svd_blocks_f64(D)
    cb = _blocks(ycc[..., 1], b)
    cr = _blocks(ycc[..., 2], b)
    w = np.ascontiguousarray(tile.reshape(-1), np.uint8)
    jac = block_bytes(O.embed_frame(cov, tile, b, alpha, route="jacobi"), b)
    ref = block_bytes(O.embed_frame(cov, tile, b, alpha, route="lapack"), b)
    # the hybrid route's conditioning flag (orc_svd_flag)
    m = np.abs(sj[:, :, None] - sj[:, None, :])
    m[:, np.arange(b), np.arange(b)] = np.inf
    m = np.minimum(sj, m.min(axis=2))
    keep = sj.astype(np.float32) != 0
    s1 = sj.max(axis=1)
    mm = np.where(keep, m, np.inf).min(axis=1)
    flag20 = (s1 > 0) & (mm * 2.0**20 < s1)
    f0, b0, _ = cert(L, Uj, sj, Vj, w, alpha, cb, cr, 0.0)
    assert not f0.any(), "K = 0 must certify every block"
    diff_j = ~np.all((jac == ref).reshape(len(D), -1), axis=1)
    res = {"blocks": len(D), "flag20": int(flag20.sum()), "k0_equals_jacobi": bool(np.array_equal(b0, jac)),
           "jacobi_bytes_differ_unflagged": int((diff_j & ~flag20).sum())}
    for K in Ks:
        t0 = time.time()
        f, byts, st = cert(L, Uj, sj, Vj, w, alpha, cb, cr, K)
        ok = ~f & ~flag20
        unsound = int((~np.all((byts == ref).reshape(len(D), -1), axis=1) & ok).sum())
        res[f"K{K:g}"] = {"fail": int((f & ~flag20).sum()), "fail_pct": round(100.0 * (f & ~flag20).mean(), 4),
                          "unsound": unsound, "missed_jacobi_diff": int((diff_j & ~flag20 & ~f).sum()),
                          "M_unc_per_block": round(st[0] / len(D), 3), "Y_unc_per_block": round(st[1] / len(D), 3), "elem_unc_blocks_pct": round(100.0 * st[2] / len(D), 2),
                          "s": round(time.time() - t0, 2)}
    return res


def main():
    b, n = int(sys.argv[1]), int(sys.argv[2])
    H, W = (int(x) for x in sys.argv[3:5]) if len(sys.argv) > 4 else (2160, 3840)
    Ks = [float(k) for k in sys.argv[5:]] or [128.0, 256.0]
    alpha = float(os.environ.get("ALPHA", "0.1"))
    L = lib()
    for kind in os.environ.get("KINDS", "noise,photo").split(","):
        for f in range(n):
            t0 = time.time()
            if kind == "noise":
                cov = O.synth_bytes(0x5EED0001, f, 1, H * W * 3).reshape(H, W, 3)
            elif kind == "photo":
                cov = photo_cover(H, W, 100 + f)
            else:
                from golden.gen_golden import cover
                cov = cover(kind, H, W, 11 + f)
                if cov.ndim == 2:
                    cov = np.stack([cov] * 3, -1)
            if os.environ.get("WM") == "qr":
                from golden.gen_golden import wmark
                tile = wmark("qr", H // b, W // b, 3 + f)
            else:
                tile = O.synth_bytes(0x5EED0002, 0, 1, (H // b) * (W // b)).reshape(H // b, W // b)
            r = study(L, cov, tile, b, alpha, Ks)
            print(kind, f, f"{time.time() - t0:.1f}s", r, flush=True)


if __name__ == "__main__":
    main()
