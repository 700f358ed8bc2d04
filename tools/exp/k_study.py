"""The certificate's bound K at scale: the direct
Jacobi-vs-dgesdd factor difference over >= TARGET certified blocks per block size, per cover class
(tests/k_corpus.py), in units of 2^-53 s1 / g_k (U, V) and 2^-53 s1 (sigma).  Prints per-class max
and q99.99, writes profiles/r06/k_study/k_study_b{B}.json and the worst blocks of every class to
tests/golden/k_corpus_worst_b{B}.npz (the CPU test re-checks them).
usage: k_study.py B TARGET_PER_CLASS [--r05] [CLASS ...]
  --r05: the round-5 contract (the Newton finish's absolute |F| <= 2^-27 test alone; no files
  are written but the log), for the before / after comparison."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import k_corpus as kc  # noqa: E402

KEEP = 64


def main():
    b, target = int(sys.argv[1]), int(sys.argv[2])
    r05 = "--r05" in sys.argv[3:]
    only = [a for a in sys.argv[3:] if not a.startswith("--")]
    if r05:
        kc.O.lib().orc_set_newton_scaled(0)
    res, worst = {}, {}
    for kind in only or (kc.PIXEL_KINDS + kc.DCT_KINDS):
        t0 = time.time()
        seed, nblk, ncert = 1000, 0, 0
        rs_all, ru_all, rv_all = [], [], []
        wD, wr = np.zeros((0, b, b), np.float32), np.zeros(0)
        while ncert < target:
            D = kc.corpus(kind, b, seed, n=50000) if kind in kc.DCT_KINDS else \
                kc.pixel_class(kind, b, seed, H=1088, W=1920)
            cert, ru, rv, rs = kc.ratios(D)
            nblk += len(D)
            ncert += int(cert.sum())
            ru_all.append(ru[cert].astype(np.float32)); rv_all.append(rv[cert].astype(np.float32))
            rs_all.append(rs[cert].astype(np.float32))
            score = np.maximum(np.maximum(ru, rv), rs)
            score[~cert] = -1
            top = np.argsort(score)[-KEEP:]
            wD = np.concatenate([wD, D[top]]); wr = np.concatenate([wr, score[top]])
            keep = np.argsort(wr)[-KEEP:]
            wD, wr = wD[keep], wr[keep]
            seed += 1
        ru_a, rv_a, rs_a = (np.concatenate(x) for x in (ru_all, rv_all, rs_all))
        q = lambda a: float(np.quantile(a, 0.9999))
        r = {"blocks": nblk, "certified": ncert, "seeds": [1000, seed - 1],
             "u_max": float(ru_a.max()), "u_q9999": q(ru_a), "v_max": float(rv_a.max()), "v_q9999": q(rv_a),
             "s_max": float(rs_a.max()), "s_q9999": q(rs_a), "seconds": round(time.time() - t0, 1)}
        res[kind] = r
        worst[kind] = wD
        print(b, kind, json.dumps(r), flush=True)
    tot = sum(r["certified"] for r in res.values())
    allmax = max(max(r["u_max"], r["v_max"], r["s_max"]) for r in res.values())
    summary = {"b": b, "K": kc.K_CERT, "certified_total": tot, "max_units": allmax,
               "margin_vs_K": kc.K_CERT / allmax, "classes": res}
    print(json.dumps({k: v for k, v in summary.items() if k != "classes"}), flush=True)
    if r05 or only:
        return
    with open(os.path.join(ROOT, "profiles", "r06", "k_study", f"k_study_b{b}.json"), "w") as f:
        json.dump(summary, f, indent=1)
    np.savez_compressed(os.path.join(ROOT, "tests", "golden", f"k_corpus_worst_b{b}.npz"),
                        **{k: v for k, v in worst.items()})


if __name__ == "__main__":
    main()
