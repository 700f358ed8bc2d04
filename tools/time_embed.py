#!/usr/bin/env python3
"""Time embed/extract of one library build (TMFWM_LIB=path) on synthetic 4K frames.

Used to price kernel variants (e.g. sweep caps built with -DTMF_F32_SWEEPS=...):
prints one JSON line with microseconds per frame.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from thatsmyface_amd import batch  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--frames", type=int, default=128)
    p.add_argument("--block", type=int, default=8)
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--kind", choices=["noise", "photo"], default="noise", help="covers: the bench's noise or camera-like")
    p.add_argument("--wm", choices=["noise", "qr"], default="noise", help="watermark tile: uniform bytes or binary (QR)")
    p.add_argument("--route", choices=["hybrid", "reference", "rank1", "rank1_reference"], default="hybrid")
    p.add_argument("--hash", action="store_true", help="sha256 of the embed output and the extracted tiles (A/B identity)")
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    b = a.block
    sys.path.insert(0, os.path.join(ROOT, "tools", "exp"))
    from route_diff_gpu import photo_covers, qr_tile

    fr = photo_covers(a.frames, 2160, 3840, 5, dev) if a.kind == "photo" else batch.synth_frames(a.frames, 2160, 3840, device=dev)
    tile = qr_tile(2160 // b, 3840 // b, 1, dev) if a.wm == "qr" else batch.synth_tile(2160 // b, 3840 // b, device=dev)
    st = {}
    rt = a.route
    out = batch.embed_batch(fr, tile, b, 0.1, stats=st, route=rt)
    ext = batch.extract_batch(out, fr, b, 0.1, route=rt)
    torch.cuda.synchronize()
    res = {}
    for name, fn in (("embed", lambda: batch.embed_batch(fr, tile, b, 0.1, out=out, route=rt)),
                     ("extract", lambda: batch.extract_batch(out, fr, b, 0.1, out=ext, route=rt))):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res[name] = round(e0.elapsed_time(e1) * 1000 / a.reps / a.frames, 2)
    line = {"lib": os.path.basename(os.environ.get("TMFWM_LIB", "libtmfwm.so")), "block": b, "kind": a.kind, "wm": a.wm,
            "route": rt, "frames": a.frames, "dgesdd_route_blocks": st.get("lapack_blocks"), "us_per_frame": res}
    if a.hash:
        import hashlib
        line["sha256"] = {"embed": hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16],
                          "extract": hashlib.sha256(ext.cpu().numpy().tobytes()).hexdigest()[:16]}
    print(json.dumps(line))


if __name__ == "__main__":
    main()
