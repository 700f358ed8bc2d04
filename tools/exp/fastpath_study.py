"""Certified rank-1 embed ("fast path", SURVEY 7 H2 / VERDICT r03 item 4): how many blocks can
skip the full SVD with a rigorous proof that their output bytes are the reference's?

The reference (watermarking.py:192-216) computes per block M_ref = fl(U32 @ fl(S'32 * Vt32))
from LAPACK's factors rounded to f32, then Y_ref = IDCT_fl(M_ref) and the bytes.  Because only
S[0] changes, M_ref = D + c u1 v1^T + (rounding terms), c = alpha * w / 255.  The fast path
computes M_fast = f32(D + c u1 v1^T) from the top singular pair alone, Y_fast = IDCT_fl(M_fast),
and a per-pixel bound eps_Y >= |Y_ref - Y_fast|:

  dM_ij <= 1.01 [(b+5) u (G_ij + c P_ij) + 2u (s1 + c) P_ij] + eps_A + 2 c eps_uv
    u = 2^-24; G_ij = sqrt(|D_i,:| |D_:,j|) bounds sum_t |U_it| s_t |V_jt| (Cauchy-Schwarz twice,
    rows of U and V are unit vectors); P_ij = |u1_i| |v1_j|; eps_A = K_A 2^-53 s1 (LAPACK's
    residual |U S V^T - D|, K_A = 1024); eps_uv bounds the top pair's disagreement (K 2^-53 s1/gap1);
    the (b+5) u counts the b fmaf roundings of the chain, 4 factor roundings and the f32(M_fast);
  eps_Y = kappa |C| (dM + 2 gamma_L (|M_fast| + dM)) |C|^T   (linear part + both IDCT roundings;
    |C| the exact ortho DCT-III matrix, kappa = 2, L = 16 as the pocketfft depth allowance).
A channel byte is certain when the colour inverse (monotone in Y, slope 1) gives the same byte
for every Y in [Y_fast - eps_Y, Y_fast + eps_Y] (f32 rounding slack included); a block is
certified when all its bytes are.  Reported: certified fraction, and that every certified
block's bytes equal the dgesdd route's (np.linalg.svd's arithmetic).
usage: fastpath_study.py B FRAMES_PER_KIND [H W]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from oracle import oracle as O  # noqa: E402
from lapack_path import _blocks, _unblocks, photo_cover  # noqa: E402
from cert_study import lp_f64  # noqa: E402

U32 = 2.0**-24
EPS = 2.0**-53


def dct_matrix(b):
    """exact orthonormal DCT-II matrix C (Y = C X C^T); its transpose is the DCT-III."""
    k = np.arange(b)[:, None]
    n = np.arange(b)[None, :]
    C = np.cos(np.pi * (2 * n + 1) * k / (2 * b)) * np.sqrt(2.0 / b)
    C[0] /= np.sqrt(2.0)
    return C


def byte_of(t):
    """u8_from_unit of an f64 colour value already rounded to f32"""
    return np.floor(np.clip(t.astype(np.float32), 0, 1) * np.float32(255)).astype(np.int64)


def certify(cov, tile, b, alpha=0.1, K_A=1024.0, K_uv=1024.0, kappa=2.0, L=16, route_check=True):
    H, W = cov.shape[:2]
    nbh, nbw = H // b, W // b
    ycc = O.rgb_to_ycbcr(cov)
    D = O.dct2d_blocks(_blocks(ycc[..., 0], b))
    Ul, sl, Vtl = lp_f64(D)
    n = len(D)
    s1 = sl[:, 0]
    u1 = Ul[:, :, 0]
    v1 = Vtl[:, 0, :]
    c = alpha * (tile.reshape(-1).astype(np.float64) / 255.0)
    D64 = D.astype(np.float64)
    Mf = (D64 + c[:, None, None] * u1[:, :, None] * v1[:, None, :]).astype(np.float32)
    Yf = O.dct2d_blocks(Mf, inverse=True)
    # bound
    r = np.sqrt((D64**2).sum(axis=2)) * (1 + 1e-12)
    cn = np.sqrt((D64**2).sum(axis=1)) * (1 + 1e-12)
    G = np.sqrt(r[:, :, None] * cn[:, None, :])
    P = np.abs(u1)[:, :, None] * np.abs(v1)[:, None, :]
    F = (D64**2).sum(axis=(1, 2))
    s2 = np.sqrt(np.maximum(F - s1**2, 0))
    gap = np.maximum(s1 - s2, 1e-300)
    eps_uv = K_uv * EPS * s1 / gap
    dM = 1.01 * ((b + 5) * U32 * (G + c[:, None, None] * P) + 2 * U32 * (s1 + c)[:, None, None] * P) \
        + (K_A * EPS * s1)[:, None, None] + (2 * c * eps_uv)[:, None, None]
    gL = L * U32 / (1 - L * U32)
    X = dM + 2 * gL * (np.abs(Mf.astype(np.float64)) + dM)
    C = np.abs(dct_matrix(b))
    epsY = kappa * np.einsum("ai,nij,bj->nab", C.T, X, C.T)  # DCT-III = C^T
    # per pixel / channel certainty
    Yp = _unblocks(Yf, nbh, nbw, b).astype(np.float64)
    Ep = _unblocks(epsY, nbh, nbw, b)
    cbp = (ycc[: nbh * b, : nbw * b, 1] - np.float32(0.5)).astype(np.float64)
    crp = (ycc[: nbh * b, : nbw * b, 2] - np.float32(0.5)).astype(np.float64)
    ok = np.ones(Yp.shape, bool)
    for a_cr, a_cb in ((1.403, 0.0), (-0.714, -0.344), (0.0, 1.773)):
        base = a_cr * crp + a_cb * cbp
        t = Yp + base
        slack = Ep * (1 + 1e-9) + 2 * U32 * np.abs(t) + 1e-12
        lo, hi = t - slack, t + slack
        plo = np.where(lo >= 1, 255.0, np.clip(lo, 0, 1) * 255.0 * (1 - 2**-21) - 1e-9)
        phi = np.where(hi <= 0, 0.0, np.clip(hi, 0, 1) * 255.0 * (1 + 2**-21) + 1e-9)
        ok &= (np.floor(np.maximum(plo, 0)) == np.floor(np.minimum(phi, 255.0)))
    cert = ok.reshape(nbh, b, nbw, b).all(axis=(1, 3)).reshape(-1)
    res = {"blocks": n, "certified": int(cert.sum()), "frac_exact_path": 1 - float(cert.mean()),
           "epsY_median_bytes": float(np.median(epsY) * 255)}
    if route_check:
        # certified blocks' bytes must be the dgesdd route's
        out_fast = ycc.copy()
        out_fast[: nbh * b, : nbw * b, 0] = _unblocks(Yf, nbh, nbw, b)
        fast = O.ycbcr_to_rgb(out_fast)
        ref = O.embed_frame(cov, tile, b, alpha, route="lapack")
        bd = (fast != ref)[: nbh * b, : nbw * b].reshape(nbh, b, nbw, b, 3).any(axis=(1, 3, 4)).reshape(-1)
        res["certified_blocks_differing_from_lapack"] = int((bd & cert).sum())
        res["uncertified_blocks_differing"] = int((bd & ~cert).sum())
    return res


def main():
    b, nfr = int(sys.argv[1]), int(sys.argv[2])
    H, W = (int(x) for x in sys.argv[3:5]) if len(sys.argv) > 4 else (2160, 3840)
    for kind in ("noise", "photo"):
        for f in range(nfr):
            t0 = time.time()
            cov = O.synth_bytes(0x5EED0001, f, 1, H * W * 3).reshape(H, W, 3) if kind == "noise" else photo_cover(H, W, 100 + f)
            tile = O.synth_bytes(0x5EED0002, f, 1, (H // b) * (W // b)).reshape(H // b, W // b)
            print(kind, f, f"{time.time() - t0:.1f}s", certify(cov, tile, b), flush=True)


if __name__ == "__main__":
    main()
