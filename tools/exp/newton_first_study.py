#!/usr/bin/env python3
"""Could the hybrid route's f64 phase start with Newton steps instead of a Jacobi sweep?
(DESIGN.md 4, round-5 lever study; CPU only, numpy.)

Today, after phase 1 (f32 one-sided Jacobi, 4 sweeps) and two Bjorck steps, phase 3 runs f64
sweeps until a first-order Newton step F_ij = G_ij / (G_jj - G_ii) (G = A^T A) is small enough
(|F| <= 2^-27) to finish.  On noise covers at b = 8 that is one sweep + the step for nearly every
block.  The alternative studied here replaces the sweep by a second-order step from the f32
start: V <- V (I + F + F^2 / 2), A <- A (I + F + F^2 / 2) in f64 (orthogonal to O(F^4)), then the
usual first-order finish.  It is valid for a block when its first |F| is small; the device would
need every block of a wave but kDeferMax of them to qualify.

This script restates phase 1 in numpy (f32 rotations in the circle-method order, the contract's
rotation formula, 1/sqrt in f32 -- not the hardware rsq table, so its f32 factors are close to,
not bit-equal with, the oracle's), then reports per block the largest first |F|, the fraction of
blocks (and of 32-block waves, b = 8) that a threshold admits, and for the admitted blocks the
two-step result's error against np.linalg.svd (LAPACK), next to the shipped route's
(oracle orc_svd_blocks_f64) -- both in units of 2^-53 sigma_1 / m_k as DESIGN.md 3.5 measures.

usage: newton_first_study.py --block 8 --height 1080 --width 1920"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from oracle import oracle as O  # noqa: E402
from lapack_path import _blocks, photo_cover  # noqa: E402


def circle_pairs(b):
    idx = lambda s, k: 0 if k == 0 else 1 + ((k - 1 + s) % (b - 1))  # noqa: E731
    rounds = []
    for s in range(b - 1):
        rounds.append([tuple(sorted((idx(s, p), idx(s, b - 1 - p)))) for p in range(b // 2)])
    return rounds


def phase1(D, sweeps=4):
    """f32 one-sided Jacobi on D (nb, b, b) -> V32 (nb, b, b); columns rotated as the contract does."""
    A = D.astype(np.float32).copy()
    nb, b, _ = A.shape
    V = np.broadcast_to(np.eye(b, dtype=np.float32), A.shape).copy()
    F = np.einsum("nij,nij->n", A, A)
    c2 = np.float32(2.0 ** -45) * F
    tol2 = np.float32(2.0 ** -40)
    c2a = np.float32(2.0 ** -48) * F * F
    one = np.float32(1)
    for _ in range(sweeps):
        nrm = np.einsum("nij,nij->nj", A, A)
        for rnd in circle_pairs(b):
            for i, j in rnd:
                a, bb = nrm[:, i], nrm[:, j]
                g = np.einsum("ni,ni->n", A[:, :, i], A[:, :, j])
                g2 = g * g
                rot = ~((g2 <= c2 * (a + bb)) | (g2 <= (tol2 * a) * bb) | (g2 <= c2a))
                d = bb - a
                gg = g + g
                x = d * d + gg * gg
                r = x / np.sqrt(x)
                w = np.abs(d) + r
                q = one / np.sqrt((r + r) * w)
                sg = np.where(d < 0, np.float32(-1), one)
                c = np.where(rot, w * q, one).astype(np.float32)
                s = np.where(rot, (gg * sg) * q, np.float32(0)).astype(np.float32)
                tg = np.where(rot, (((gg * gg) * r) * (q * q)) * sg, np.float32(0)).astype(np.float32)
                for M in (A, V):
                    xi, yj = M[:, :, i].copy(), M[:, :, j].copy()
                    M[:, :, i] = -s[:, None] * yj + c[:, None] * xi
                    M[:, :, j] = s[:, None] * xi + c[:, None] * yj
                nrm[:, i] = a - tg
                nrm[:, j] = bb + tg
    return V


def bjorck(V):
    I = np.eye(V.shape[-1])
    N = 1.5 * I - 0.5 * np.einsum("nki,nkj->nij", V, V)
    return V @ N


def first_f(A):
    G = np.einsum("nki,nkj->nij", A, A)
    dg = np.einsum("nii->ni", G)
    den = dg[:, None, :] - dg[:, :, None]
    with np.errstate(divide="ignore", invalid="ignore"):
        F = np.where(np.triu(np.ones(G.shape[1:], bool), 1), G / den, 0.0)
    F = F - np.swapaxes(F, 1, 2)
    return F


def errors(U, sig, V, Ul, sl, Vl):
    """per block: max over k of |factor diff| / (2^-53 sigma_1 / m_k) (sign-aligned columns)"""
    b = sig.shape[1]
    order = np.argsort(-sig, axis=1)
    sig = np.take_along_axis(sig, order, 1)
    U = np.take_along_axis(U, order[:, None, :], 2)
    V = np.take_along_axis(V, order[:, None, :], 2)
    sgn = np.sign(np.einsum("nik,nik->nk", U, Ul))
    sgn[sgn == 0] = 1
    U, V = U * sgn[:, None, :], V * sgn[:, None, :]
    gaps = np.abs(sl[:, :, None] - sl[:, None, :]) + np.eye(b)[None] * 1e300
    m = np.minimum(sl, gaps.min(axis=2))
    unit = 2.0 ** -53 * sl[:, :1] / np.maximum(m, 1e-300)
    eu = (np.abs(U - Ul).max(axis=1) / unit).max(axis=1)
    ev = (np.abs(V - Vl).max(axis=1) / unit).max(axis=1)
    return eu, ev


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--block", type=int, default=8)
    p.add_argument("--height", type=int, default=1080)
    p.add_argument("--width", type=int, default=1920)
    a = p.parse_args()
    b, H, W = a.block, a.height, a.width
    for kind in ("noise", "photo"):
        cov = O.synth_bytes(0x5EED0001, 0, 1, H * W * 3).reshape(H, W, 3) if kind == "noise" else photo_cover(H, W, 500)
        D = O.dct2d_blocks(_blocks(O.rgb_to_ycbcr(cov)[..., 0], b)).astype(np.float32)
        D = D[np.abs(D).reshape(len(D), -1).max(axis=1) > 0]
        V0 = bjorck(bjorck(phase1(D).astype(np.float64)))
        A0 = D.astype(np.float64) @ V0
        F1 = first_f(A0)
        fmax = np.nan_to_num(np.abs(F1).reshape(len(F1), -1).max(axis=1), nan=np.inf)
        # two steps: second order from the f32 start, then the contract's first-order finish
        M = F1 + 0.5 * (F1 @ F1)
        I = np.eye(b)
        V1, A1 = V0 @ (I + M), A0 @ (I + M)
        F2 = first_f(A1)
        f2max = np.nan_to_num(np.abs(F2).reshape(len(F2), -1).max(axis=1), nan=np.inf)
        F2f = F2.astype(np.float32).astype(np.float64)
        V2 = V1 + (V1.astype(np.float32).astype(np.float64) @ F2f)
        A2 = A1 + (A1.astype(np.float32).astype(np.float64) @ F2f)
        sig2 = np.sqrt(np.einsum("nki,nki->ni", A2, A2))
        U2 = A2 / sig2[:, None, :]
        Ul, sl, Vlt = np.linalg.svd(D.astype(np.float64))
        Vl = np.swapaxes(Vlt, 1, 2)
        Uo, so, Vo = O.svd_blocks_f64(D)
        eu2, ev2 = errors(U2, sig2, V2, Ul, sl, Vl)
        euo, evo = errors(Uo, so, Vo, Ul, sl, Vl)
        orth = np.abs(np.einsum("nki,nkj->nij", V2, V2) - I).reshape(len(V2), -1).max(axis=1)
        res = {"kind": kind, "block": b, "blocks": int(len(D))}
        for t in (2.0 ** -20, 2.0 ** -16, 2.0 ** -12, 2.0 ** -10):
            ok = (fmax <= t) & (f2max <= 2.0 ** -27)
            row = {"blocks_admitted": round(float(ok.mean()), 4)}
            if b == 8:
                nw = len(ok) // 32
                bad = (~ok[: nw * 32]).reshape(nw, 32).sum(axis=1)
                row["waves_with_<=4_rejected"] = round(float((bad <= 4).mean()), 4)
            if ok.any():
                row["two_step_err_U_V_p99_max"] = [round(float(np.percentile(eu2[ok], 99)), 2), round(float(eu2[ok].max()), 1),
                                                   round(float(np.percentile(ev2[ok], 99)), 2), round(float(ev2[ok].max()), 1)]
                row["two_step_orthogonality_max"] = float(orth[ok].max())
            res[f"tau=2^{int(np.log2(t))}"] = row
        res["first_F_max_percentiles_50_90_99"] = [float(np.percentile(fmax, q)) for q in (50, 90, 99)]
        res["shipped_route_err_U_V_p99_max"] = [round(float(np.percentile(euo, 99)), 2), round(float(euo.max()), 1),
                                               round(float(np.percentile(evo, 99)), 2), round(float(evo.max()), 1)]
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
