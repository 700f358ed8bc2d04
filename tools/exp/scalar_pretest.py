"""VERDICT r05 item 2, first step: how many blocks would a scalar |dY| pre-test on the point path
leave undecided?  

The point path reconstructs with the Jacobi route's f32 factors (U32, S'32, Vt32: the round-4
kernel).  LAPACK's f32 factors lie inside the certificate's intervals (K = 256), so per element
  dU = max |ends - U32|, dB = max over S' / V corners |f32(S' v) - B32|.
Bounds on |Y_L - Y_J| per pixel, in increasing rigour:
  first-order  dM = sum_k dU |B| + |U| dB + dU dB          (no rounding terms: optimistic),
               dY = |C| dM |C|^T
  rigorous     dM += n_ij ulp(P_ij) (one RN flip per fmaf step from the first perturbed one on,
               P_ij = sum_k |U||B| bounds every partial), dY += 2 gamma_2b (|C| |M| |C|^T) (the
               IDCT's rounding on both routes' inputs, pocketfft's two passes)
and the pre-test decides a pixel iff every channel gives the same byte at Y - dY and Y + dY
(each channel is monotone in Y; the f64 model of the inverse colour stands in for the f32 one).
Reports, over the certified blocks (non-zero, not flat, unflagged): blocks whose intervals are all
points (dY = 0, decided outright), and blocks the pre-test leaves undecided -- per pixel with each
bound, and with one scalar per block (max dY).  usage: scalar_pretest.py B [FRAMES] [H W]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import oracle as O  # noqa: E402
from lapack_path import _blocks, photo_cover  # noqa: E402

f32 = np.float32
KS = 2.0 ** -45  # kCertScale
U24 = 2.0 ** -24


def dct_matrix(b):
    """Orthonormal DCT-II matrix: Y = C^T M C for the 2-D IDCT (values only, for |C|)."""
    n = np.arange(b)
    C = np.cos(np.pi * (2 * n[None, :] + 1) * n[:, None] / (2 * b)) * np.sqrt(2.0 / b)
    C[0] /= np.sqrt(2.0)
    return C


def ulp(x):
    x = np.maximum(np.abs(x), 2.0 ** -126)
    return 2.0 ** (np.floor(np.log2(x)) - 23)


def study(cov, tile, b, alpha):
    ycc = O.rgb_to_ycbcr(cov)
    D = O.dct2d_blocks(_blocks(ycc[..., 0], b))
    n = len(D)
    Uj, sj, Vj = O.svd_blocks_f64(D)
    s1 = sj.max(axis=1)
    d = np.abs(sj[:, :, None] - sj[:, None, :])
    d[:, np.arange(b), np.arange(b)] = np.inf
    g = np.minimum(sj, d.min(axis=2))
    out = sj.astype(f32) != 0
    m = np.minimum(np.where(out, g, np.inf).min(axis=1), s1)
    flag = m * 2.0 ** 20 < s1
    flat = ~np.any(D.reshape(n, -1)[:, 1:] != 0, axis=1)
    cert = (s1 > 0) & ~flat & ~flag
    tE = KS * s1
    with np.errstate(divide="ignore", invalid="ignore"):
        E = np.where(out & cert[:, None], (tE[:, None] / g).astype(f32).astype(np.float64), 0.0)  # per triplet
    U32 = Uj.astype(f32)
    Ul, Uh = (Uj - E[:, None, :]).astype(f32), (Uj + E[:, None, :]).astype(f32)
    dU = np.maximum(np.abs(Ul.astype(float) - U32), np.abs(Uh.astype(float) - U32))
    dU = np.where(out[:, None, :], dU, 2.0)  # non-output triplets: any f32 entry
    Vt = np.swapaxes(Vj, 1, 2)
    Vt32 = Vt.astype(f32)
    Vl, Vh = (Vt - E[:, :, None]).astype(f32), (Vt + E[:, :, None]).astype(f32)
    w = tile.reshape(-1).astype(np.float64)
    cw = alpha * (w / 255.0)
    S32 = sj.astype(f32)
    Sl = np.maximum(sj - tE[:, None] * cert[:, None], 0).astype(f32)
    Sh = (sj + tE[:, None] * cert[:, None]).astype(f32)
    Sp, Spl, Sph = S32.copy(), Sl.copy(), Sh.copy()
    for a in (Sp, Spl, Sph):
        a[:, 0] = (a[:, 0].astype(np.float64) + cw).astype(f32)
    B32 = (Sp[:, :, None] * Vt32)  # f32 products, one rounding each
    cs = [(s[:, :, None] * v).astype(f32) for s in (Spl, Sph) for v in (Vl, Vh)]
    dB = np.max([np.abs(c.astype(float) - B32) for c in cs], axis=0)
    dB = np.where(out[:, :, None], dB, np.abs(Sph[:, :, None]).astype(float) + np.abs(B32))
    point = (dU.reshape(n, -1).max(axis=1) == 0) & (dB.reshape(n, -1).max(axis=1) == 0)
    # point path's M and Y (the oracle's exact fmaf chain and pocketfft IDCT)
    M = O.blend_reconstruct_blocks(U32, S32, Vt32, tile.reshape(-1).astype(np.uint8), alpha)
    Y = O.dct2d_blocks(M, inverse=True).astype(np.float64)
    aU, aB = np.abs(U32).astype(float), np.abs(B32).astype(float)
    dM1 = np.einsum("nik,nkj->nij", dU, aB) + np.einsum("nik,nkj->nij", aU, dB) + np.einsum("nik,nkj->nij", dU, dB)
    P = np.einsum("nik,nkj->nij", aU + dU, aB + dB)
    # steps from the first perturbed one: k0_ij = min k with dU_ik > 0 or dB_kj > 0
    pert = (dU[:, :, :, None] > 0) | (dB[:, None, :, :] > 0)  # n, i, k, j
    anyp = pert.any(axis=2)
    k0 = np.where(anyp, pert.argmax(axis=2), b)
    dM2 = dM1 + (b - k0) * ulp(P)
    C = np.abs(dct_matrix(b))
    idct_abs = lambda X: np.einsum("pi,nij,jq->npq", C.T, X, C)
    dY1 = idct_abs(dM1)
    gam = 2 * b * U24 / (1 - 2 * b * U24)
    dY2 = idct_abs(dM2) + 2 * gam * idct_abs(np.abs(M).astype(float) + dM2)
    dY2 = np.where(point[:, None, None], 0.0, dY2)
    dY1 = np.where(point[:, None, None], 0.0, dY1)
    # inverse colour (f64 model of watermarking.py:55-70) per pixel and channel
    cb = _blocks(ycc[..., 1], b).astype(np.float64) - 0.5
    cr = _blocks(ycc[..., 2], b).astype(np.float64) - 0.5
    v = np.stack([Y + 1.403 * cr, Y - 0.344 * cb - 0.714 * cr, Y + 1.773 * cb], -1)

    def undecided(dY):
        # bytes at both ends of [Y - dY, Y + dY] (every channel is monotone in Y with slope 1);
        # the device would evaluate the ends exactly for the pixels a 2^-14 pre-filter flags
        lo, hi = v - dY[..., None], v + dY[..., None]
        byte = lambda x: np.floor(255.0 * np.clip(x, 0, 1))
        bad = byte(lo) != byte(hi)
        return bad.reshape(n, -1).any(axis=1)

    res = {"blocks": n, "certified": int(cert.sum()), "point_blocks": int((point & cert).sum())}
    for name, dY in (("first_order_pixel", dY1), ("rigorous_pixel", dY2)):
        res[name] = int((undecided(dY) & cert).sum())
    blk = lambda dY: np.broadcast_to(dY.reshape(n, -1).max(axis=1)[:, None, None], dY.shape)
    res["first_order_block_scalar"] = int((undecided(blk(dY1)) & cert).sum())
    res["rigorous_block_scalar"] = int((undecided(blk(dY2)) & cert).sum())
    wide = cert & ~point
    res["median_dY_wide_rigorous"] = float(np.median(dY2.reshape(n, -1).max(axis=1)[wide])) if wide.any() else 0.0
    res["median_dY_wide_first_order"] = float(np.median(dY1.reshape(n, -1).max(axis=1)[wide])) if wide.any() else 0.0
    c = max(res["certified"], 1)
    res["pct"] = {k: round(100.0 * res[k] / c, 3) for k in ("point_blocks", "first_order_pixel", "rigorous_pixel",
                                                           "first_order_block_scalar", "rigorous_block_scalar")}
    return res


def main():
    b = int(sys.argv[1])
    nf = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    H, W = (int(x) for x in sys.argv[3:5]) if len(sys.argv) > 4 else (1080, 1920)
    for kind in ("noise", "photo"):
        for f in range(nf):
            t0 = time.time()
            cov = O.synth_bytes(0x5EED0001, f, 1, H * W * 3).reshape(H, W, 3) if kind == "noise" else photo_cover(H, W, 100 + f)
            tile = O.synth_bytes(0x5EED0002, 0, 1, (H // b) * (W // b)).reshape(H // b, W // b)
            r = study(cov, tile, b, 0.1)
            print(json.dumps({"b": b, "kind": kind, "frame": f, "s": round(time.time() - t0, 1), **r}), flush=True)


if __name__ == "__main__":
    main()
