"""Study: phase 3 with the Newton finish (the contract) against the plain f64
Jacobi to convergence (orc_set_newton_finish(0)), both against the dgesdd route
(np.linalg.svd's arithmetic).  Per cover class: flagged blocks, unflagged blocks whose
IDCT output bits differ from the dgesdd route's, and the per-wave maxima (32 blocks of
a block row at b = 8) of sweeps and Newton steps -- the wave runs its slowest block.
usage: refine_study.py B H W kinds seeds"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import oracle as O  # noqa: E402
from golden.gen_golden import cover, wmark  # noqa: E402
from lapack_path import _blocks, photo_cover  # noqa: E402

b = int(sys.argv[1]) if len(sys.argv) > 1 else 8
H, W = (int(x) for x in (sys.argv[2:4] if len(sys.argv) > 3 else (544, 960)))
kinds = sys.argv[4].split(",") if len(sys.argv) > 4 else ["noise", "photo", "smooth", "blocky", "qr", "diagonal"]
seeds = [int(x) for x in sys.argv[5].split(",")] if len(sys.argv) > 5 else [11, 12]
L = O.lib()
bpw = 64 // (1 if b == 4 else 2 if b <= 8 else 4 if b <= 12 else 8)
tot = {}
for kind in kinds:
    for seed in seeds:
        cov = photo_cover(H, W, seed) if kind == "photo" else cover(kind, H, W, seed)
        D = O.dct2d_blocks(_blocks(O.rgb_to_ycbcr(cov)[..., 0], b))
        tile = wmark("qr", H // b, W // b, 3).reshape(-1)
        Lp = O.lp_svd_blocks(D)
        Yl = O.dct2d_blocks(O.blend_reconstruct_blocks(*Lp, tile, 0.1), inverse=True)
        row = []
        for nf in (0, 1):
            L.orc_set_newton_finish(nf)
            U, S, Vt, sw = O.svd_blocks(D)
            _, sig, _ = O.svd_blocks_f64(D)
            flags = np.array([O.svd_flag(s) for s in sig])
            Yj = O.dct2d_blocks(O.blend_reconstruct_blocks(U, S, Vt, tile, 0.1), inverse=True)
            diff = ~np.all((Yj.view(np.uint32) == Yl.view(np.uint32)).reshape(len(D), -1), axis=1)
            nbw = W // b
            sweeps, newton = (sw & 0xFF).reshape(H // b, nbw), ((sw >> 16) & 0xFF).reshape(H // b, nbw)
            wmax = lambda a: np.concatenate([a[:, k:k + bpw].max(axis=1) for k in range(0, nbw, bpw)])  # noqa: E731
            t = tot.setdefault((kind, nf), [0, 0, 0])
            t[0] += len(D); t[1] += int(flags.sum()); t[2] += int((diff & ~flags).sum())
            row.append(f"newton_finish={nf}: flag {flags.mean()*100:.3f}% diffY_unflagged {int((diff & ~flags).sum())} "
                       f"wave-max sweeps {np.bincount(wmax(sweeps))} newton {np.bincount(wmax(newton))}")
        L.orc_set_newton_finish(1)
        print(f"b={b} {kind} seed {seed} ({len(D)} blocks)\n   " + "\n   ".join(row), flush=True)
print("totals (blocks, flagged, unflagged Y-bit diffs):", tot)
