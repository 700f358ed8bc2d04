"""Calibration study for the f32-rounding certificate of the hybrid route.

Per block of whole frames (noise and camera-like covers), with the Jacobi route's f64
factors (oracle svd_blocks_f64) and the dgesdd route's (orc_lp_svd_blocks_f64):
  * the per-triplet factor disagreement in units of eps_k = 2^-53 sigma_1 / m_k
    (m_k = min(sigma_k, gap_k)) for U and V columns, and of 2^-53 sigma_1 for sigma_k;
  * for a bound constant K: the fraction of blocks with an uncertain f32 rounding
    (some factor element x with f32(x - E) != f32(x + E)), and whether every block whose
    f32 factors differ between the routes is among them.
usage: cert_study.py B FRAMES_PER_KIND [H W]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import oracle as O  # noqa: E402
from lapack_path import _blocks, photo_cover  # noqa: E402

EPS = 2.0**-53


def lp_f64(D):
    import ctypes
    D = np.ascontiguousarray(D, np.float32)
    nb, b = D.shape[0], D.shape[-1]
    U = np.empty(D.shape, np.float64)
    Vt = np.empty(D.shape, np.float64)
    S = np.empty((nb, b), np.float64)
    f64p = ctypes.POINTER(ctypes.c_double)
    f32p = ctypes.POINTER(ctypes.c_float)
    fn = O.lib().orc_lp_svd_blocks_f64
    fn.restype = ctypes.c_int
    rc = fn(D.ctypes.data_as(f32p), ctypes.c_int64(nb), b, U.ctypes.data_as(f64p), S.ctypes.data_as(f64p),
            Vt.ctypes.data_as(f64p), O.default_threads())
    assert rc == 0
    return U, S, Vt


def gaps(sig):
    """m_k = min(sigma_k, min_{j != k} |sigma_k - sigma_j|), s1, keep (f32(sigma) != 0)."""
    b = sig.shape[1]
    d = np.abs(sig[:, :, None] - sig[:, None, :])
    d[:, np.arange(b), np.arange(b)] = np.inf
    m = np.minimum(sig, d.min(axis=2))
    return m, sig.max(axis=1), sig.astype(np.float32) != 0


def frame(cov, b):
    D = O.dct2d_blocks(_blocks(O.rgb_to_ycbcr(cov)[..., 0], b))
    Uj, sj, Vj = O.svd_blocks_f64(D)
    Ul, sl, Vtl = lp_f64(D)
    Vl = np.swapaxes(Vtl, 1, 2)
    return D, (Uj, sj, Vj), (Ul, sl, Vl)


def study(cov, b, Ks):
    D, (Uj, sj, Vj), (Ul, sl, Vl) = frame(cov, b)
    m, s1, keep = gaps(sj)
    nz = s1 > 0
    amp = np.where(keep, s1[:, None] / np.where(m > 0, m, np.inf), 0.0).max(axis=1)
    flag20 = nz & (amp > 2.0**20)
    # sign alignment per triplet
    sgn = np.sign(np.einsum("nrk,nrk->nk", Uj, Ul))
    sgn[sgn == 0] = 1
    du = np.abs(Uj - Ul * sgn[:, None, :]).max(axis=1)
    dv = np.abs(Vj - Vl * sgn[:, None, :]).max(axis=1)
    ds = np.abs(sj - sl)
    with np.errstate(divide="ignore", invalid="ignore"):
        ek = EPS * s1[:, None] / m
        ru = np.where(keep, du / ek, 0.0)
        rv = np.where(keep, dv / ek, 0.0)
        rs = np.where(keep, ds / (EPS * s1[:, None]), 0.0)
    ok = nz & ~flag20
    # f32 factors differ (the event the certificate must catch)
    f32diff = ((Uj.astype(np.float32) != (Ul * sgn[:, None, :]).astype(np.float32)) & keep[:, None, :]).any(axis=(1, 2)) | \
              ((Vj.astype(np.float32) != (Vl * sgn[:, None, :]).astype(np.float32)) & keep[:, None, :]).any(axis=(1, 2)) | \
              ((sj.astype(np.float32) != sl.astype(np.float32)) & keep).any(axis=1)
    res = {"blocks": len(D), "flag20": int(flag20.sum()), "f32diff_unflagged": int((f32diff & ok).sum()),
           "ru_max": float(ru[ok].max()), "rv_max": float(rv[ok].max()), "rs_max": float(rs[ok].max()),
           "ru_q999": float(np.quantile(ru[ok].max(axis=1), 0.999)), "rv_q999": float(np.quantile(rv[ok].max(axis=1), 0.999))}
    for K in Ks:
        E = np.where(keep, K * ek, 0.0)  # per triplet
        Es = np.where(keep, K * EPS * s1[:, None], 0.0)
        unc_u = ((Uj - E[:, None, :]).astype(np.float32) != (Uj + E[:, None, :]).astype(np.float32)) & keep[:, None, :]
        unc_v = ((Vj - E[:, None, :]).astype(np.float32) != (Vj + E[:, None, :]).astype(np.float32)) & keep[:, None, :]
        unc_s = ((sj - Es).astype(np.float32) != (sj + Es).astype(np.float32)) & keep
        unc = unc_u.any(axis=(1, 2)) | unc_v.any(axis=(1, 2)) | unc_s.any(axis=1)
        res[f"K{K}"] = {"uncertain": int((unc & ok).sum()), "missed": int((f32diff & ok & ~unc).sum()),
                        "unc_u_elems": int(unc_u[ok].sum()), "unc_v_elems": int(unc_v[ok].sum()), "unc_s": int(unc_s[ok].sum())}
    return res


def level2(Uj, sj, Vj, w, alpha, K):
    """Reconstruction-level certificate: per chain step of M = U @ (S' Vt) (fmaf chain over t),
    do all factor values within the bound give the same f32 rounding?  Returns per-block fail."""
    n, b = sj.shape
    m, s1, keep = gaps(sj)
    with np.errstate(divide="ignore", invalid="ignore"):
        Ek = np.where(keep & (m > 0), K * EPS * s1[:, None] / m, np.inf)
    Es = (K * EPS * s1)[:, None]
    f32 = np.float32
    def iv(x, e):
        lo = np.clip(x - e, -1, 1).astype(f32)
        hi = np.clip(x + e, -1, 1).astype(f32)
        return lo, hi
    U32 = Uj.astype(f32)
    Ulo, Uhi = iv(Uj, Ek[:, None, :])
    Vt = np.swapaxes(Vj, 1, 2)
    Vt32 = Vt.astype(f32)
    Vlo, Vhi = iv(Vt, Ek[:, :, None])
    S32 = sj.astype(f32)
    Slo = np.maximum(sj - Es, 0).astype(f32)
    Shi = (sj + Es).astype(f32)
    c = alpha * (w.astype(np.float64) / 255.0)
    Sp, Splo, Sphi = S32.copy(), Slo.copy(), Shi.copy()
    Sp[:, 0] = (S32[:, 0].astype(np.float64) + c).astype(f32)
    Splo[:, 0] = (Slo[:, 0].astype(np.float64) + c).astype(f32)
    Sphi[:, 0] = (Shi[:, 0].astype(np.float64) + c).astype(f32)
    B = (Sp[:, :, None] * Vt32)  # f32 * f32 -> f32 (numpy rounds once)
    d = np.float64
    cs = [Splo[:, :, None].astype(d) * Vlo.astype(d), Splo[:, :, None].astype(d) * Vhi.astype(d),
          Sphi[:, :, None].astype(d) * Vlo.astype(d), Sphi[:, :, None].astype(d) * Vhi.astype(d)]
    Blo = np.minimum.reduce(cs).astype(f32)
    Bhi = np.maximum.reduce(cs).astype(f32)
    acc = np.zeros((n, b, b), f32)
    fail = np.zeros(n, bool)
    unc_steps = 0
    if os.environ.get("IVL"):
        # interval propagation: [alo, ahi] = every f32 value the chain can hold after step t
        alo = np.zeros((n, b, b), d)
        ahi = np.zeros((n, b, b), d)
        for t in range(b):
            ul, uh = (a[:, :, t][:, :, None].astype(d) for a in (Ulo, Uhi))
            bl, bh = (a[:, t, :][:, None, :].astype(d) for a in (Blo, Bhi))
            unc_steps += int(((ul != uh) | (bl != bh)).sum())
            cs = [ul * bl, ul * bh, uh * bl, uh * bh]
            lo = np.minimum.reduce(cs) + alo
            hi = np.maximum.reduce(cs) + ahi
            lo = lo - np.abs(lo) * 2.0**-52
            hi = hi + np.abs(hi) * 2.0**-52
            alo = lo.astype(f32).astype(d)
            ahi = hi.astype(f32).astype(d)
        fail = (alo != ahi).any(axis=(1, 2))
        return fail, unc_steps
    for t in range(b):
        u, ul, uh = (a[:, :, t][:, :, None].astype(d) for a in (U32, Ulo, Uhi))
        bt, bl, bh = (a[:, t, :][:, None, :].astype(d) for a in (B, Blo, Bhi))
        pert = (ul != uh) | (bl != bh)
        cs = [ul * bl, ul * bh, uh * bl, uh * bh]
        a64 = acc.astype(d)
        lo = np.minimum.reduce(cs) + a64
        hi = np.maximum.reduce(cs) + a64
        lo = lo - np.abs(lo) * 2.0**-52
        hi = hi + np.abs(hi) * 2.0**-52
        ok = lo.astype(f32) == hi.astype(f32)
        fail |= (pert & ~ok).any(axis=(1, 2))
        unc_steps += int(pert.sum())
        acc = (u * bt + a64).astype(f32)
    return fail, unc_steps


def study2(cov, tile, b, Ks, alpha=0.1):
    D, (Uj, sj, Vj), (Ul, sl, Vl) = frame(cov, b)
    m, s1, keep = gaps(sj)
    nz = s1 > 0
    amp = np.where(keep, s1[:, None] / np.where(m > 0, m, np.inf), 0.0).max(axis=1)
    flag20 = nz & (amp > 2.0**20)
    w = tile.reshape(-1)
    J = (Uj.astype(np.float32), sj.astype(np.float32), np.ascontiguousarray(np.swapaxes(Vj, 1, 2)).astype(np.float32))
    L = (Ul.astype(np.float32), sl.astype(np.float32), np.ascontiguousarray(np.swapaxes(Vl, 1, 2)).astype(np.float32))
    Yj, Yl = (O.dct2d_blocks(O.blend_reconstruct_blocks(*f, w, alpha), inverse=True) for f in (J, L))
    ydiff = ~np.all((Yj.view(np.uint32) == Yl.view(np.uint32)).reshape(len(D), -1), axis=1)
    res = {"blocks": len(D), "flag20": int(flag20.sum()), "nonkeep_blocks": int((~keep & nz[:, None]).any(axis=1).sum()),
           "ydiff_unflagged20": int((ydiff & ~flag20).sum())}
    for K in Ks:
        fail, us = level2(Uj, sj, Vj, w, alpha, K)
        res[f"K{K}"] = {"fail": int((fail & ~flag20).sum()), "missed": int((ydiff & ~flag20 & ~fail).sum()), "pert_steps_per_block": us / len(D)}
    return res


def main():
    b, n = int(sys.argv[1]), int(sys.argv[2])
    H, W = (int(x) for x in sys.argv[3:5]) if len(sys.argv) > 4 else (2160, 3840)
    Ks = (4, 16, 64, 256)
    for kind in ("noise", "photo"):
        for f in range(n):
            t0 = time.time()
            cov = O.synth_bytes(0x5EED0001, f, 1, H * W * 3).reshape(H, W, 3) if kind == "noise" else photo_cover(H, W, 100 + f)
            if os.environ.get("L2"):
                tile = O.synth_bytes(0x5EED0002, f, 1, (H // b) * (W // b)).reshape(H // b, W // b)
                r = study2(cov, tile, b, Ks)
            else:
                r = study(cov, b, Ks)
            print(kind, f, f"{time.time() - t0:.1f}s", r, flush=True)


if __name__ == "__main__":
    main()
