"""The rank-1 pre-pass's two LAPACK constants at scale (csrc/tmfwm_rank1.hip header).

The pre-pass bounds |M_ref - M_fast| assuming
  (1) LAPACK's residual |(U S V^T)_ij - D_ij| <= 8192 units of 2^-53 sigma_1 (gamma' = 2^-40 s1), and
  (2) LAPACK's top singular pair within 1024 units of 2^-53 sigma_1 / (sigma_1 - sigma_2).
(1) is measured here directly: np.linalg.svd's f64 factors (the restated dgesdd route, pinned bit
for bit against numpy) multiplied back in extended precision (np.longdouble, 64-bit mantissa, so
the product's own error is ~2^-11 of a unit).  (2) is bounded by the K study's direct
Jacobi-vs-dgesdd difference (every output triplet, the top one included; profiles/r06/k_study/)
plus the Jacobi route's own error (<= 30 units against a long-double refinement, round 4's
route_errors study); here the top triplet's share of that difference is reported on its own.
Every block with sigma_1 > 0 counts for (1); (2) is over blocks with sigma_1 > sigma_2.
Same seeded cover classes as the K study (tests/k_corpus.py).
usage: lapack_bounds.py B BLOCKS_PER_CLASS [CLASS ...]  -> profiles/r06/lapack_bounds_b{B}.json
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import k_corpus as kc  # noqa: E402

RESID_UNITS = kc.RESID_UNITS
PAIR_UNITS = kc.PAIR_UNITS


def main():
    b, target = int(sys.argv[1]), int(sys.argv[2])
    only = sys.argv[3:]
    res = {}
    for kind in only or (kc.PIXEL_KINDS + kc.DCT_KINDS):
        t0 = time.time()
        seed, nblk, rmax, pmax, rq, pq = 2000, 0, 0.0, 0.0, [], []
        while nblk < target:
            D = kc.corpus(kind, b, seed, n=50000) if kind in kc.DCT_KINDS else \
                kc.pixel_class(kind, b, seed, H=1088, W=1920)
            U, S, V = kc.lapack_f64(D)
            r = kc.residual_units(D, U, S, V)
            ok, p = kc.top_pair_units(D, S, U, V)
            rmax, pmax = max(rmax, float(r.max())), max(pmax, float(p[ok].max(initial=0.0)))
            rq.append(r.astype(np.float32)); pq.append(p[ok].astype(np.float32))
            nblk += len(D)
            seed += 1
        ra, pa = np.concatenate(rq), np.concatenate(pq)
        res[kind] = {"blocks": nblk, "resid_max": rmax, "resid_q9999": float(np.quantile(ra, 0.9999)),
                     "top_pair_max": pmax, "top_pair_q9999": float(np.quantile(pa, 0.9999)) if len(pa) else 0.0,
                     "seconds": round(time.time() - t0, 1)}
        print(b, kind, json.dumps(res[kind]), flush=True)
    summary = {"b": b, "resid_bound_units": RESID_UNITS, "pair_bound_units": PAIR_UNITS,
               "blocks_total": sum(r["blocks"] for r in res.values()),
               "resid_max": max(r["resid_max"] for r in res.values()),
               "top_pair_max": max(r["top_pair_max"] for r in res.values()), "classes": res}
    print(json.dumps({k: v for k, v in summary.items() if k != "classes"}), flush=True)
    if not only:
        out = os.path.join(ROOT, "profiles", "r06", f"lapack_bounds_b{b}.json")
        with open(out, "w") as f:
            json.dump(summary, f, indent=1)


if __name__ == "__main__":
    main()
