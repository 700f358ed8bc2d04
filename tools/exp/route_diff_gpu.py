#!/usr/bin/env python3
"""The hybrid route's bytes against the reference route's, at scale, on the GPU.

The reference route (TMFWM_ROUTE_REFERENCE) runs the dgesdd route on every block: np.linalg.svd's
arithmetic by construction, pinned bit for bit against the oracle and numpy.  The hybrid route
sends only conditioning-flagged blocks there and keeps the Jacobi route's f32-rounded factors for
the rest, so its exactness is statistical (the CPU flag-margin studies count IDCT-bit divergences
at ~1e-4 of blocks at b = 16 on camera-like covers, with ~1e-4 expected byte flips each).  This
script counts the bytes themselves, over far more blocks than the CPU oracle can reach: for each
batch of synthetic covers (uniform noise as the bench uses, and camera-like covers: a blurred
noise field + gradients + grain, the recipe of tests/lapack_path.photo_cover drawn with torch's
generator on the device) it runs both routes' embed and extract and reports the differing bytes,
the blocks that hold them, and the blocks the hybrid route sent to the dgesdd route.

usage: route_diff_gpu.py --block 16 --kind photo --frames 512 --batch 32 [--height 2160 --width 3840]
Prints one JSON line per batch and a total line."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from thatsmyface_amd import batch  # noqa: E402


def photo_covers(n, H, W, seed, dev):
    """Camera-like covers (tests/lapack_path.photo_cover's recipe, torch's generator)."""
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    f = torch.randn((n, H // 16 + 2, W // 16 + 2, 3), generator=g, device=dev)
    f = f.repeat_interleave(16, 1).repeat_interleave(16, 2)[:, :H, :W]
    for ax in (1, 2):
        for _ in range(2):
            f = (torch.roll(f, 5, ax) + torch.roll(f, -5, ax) + f) / 3.0
    y = torch.linspace(0, 1, H, device=dev).view(1, H, 1, 1)
    x = torch.linspace(0, 1, W, device=dev).view(1, 1, W, 1)
    img = 128 + 45 * f + 60 * (x - 0.5) + 30 * (y - 0.5)
    img = img + 2.0 * torch.randn(img.shape, generator=g, device=dev)
    return img.clamp_(0, 255).to(torch.uint8)


def qr_tile(nbh, nbw, seed, dev):
    """Binary 0 / 255 watermark tile (a resized QR code's modules at one pixel per block)."""
    g = torch.Generator(device=dev)
    g.manual_seed(seed + 99)
    return torch.randint(0, 2, (nbh, nbw), generator=g, device=dev, dtype=torch.uint8) * 255


def blocks_differing(a, c, b):
    """Blocks of (n, H, W, 3) frames holding at least one differing byte."""
    n, H, W, _ = a.shape
    d = (a != c).any(dim=3)[:, : H // b * b, : W // b * b]
    return int(d.view(n, H // b, b, W // b, b).any(dim=4).any(dim=2).sum())


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--block", type=int, default=16)
    p.add_argument("--alpha", type=float, default=0.1)
    p.add_argument("--kind", choices=["noise", "photo"], default="photo")
    p.add_argument("--frames", type=int, default=256)
    p.add_argument("--batch", type=int, default=32)
    p.add_argument("--height", type=int, default=2160)
    p.add_argument("--width", type=int, default=3840)
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--wm", choices=["noise", "qr"], default="noise",
                   help="watermark tile: uniform bytes (the bench's) or binary 0 / 255 (a QR code, the app's)")
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    H, W, b = a.height, a.width, a.block
    tile = qr_tile(H // b, W // b, a.seed, dev) if a.wm == "qr" else batch.synth_tile(H // b, W // b, device=dev)
    tot = dict(frames=0, blocks=0, dgesdd_route_blocks=0, embed_bytes_differing=0, embed_blocks_differing=0,
               extract_bytes_differing=0, extract_same_input_bytes_differing=0)
    t_start = time.time()
    for i, f0 in enumerate(range(0, a.frames, a.batch)):
        n = min(a.batch, a.frames - f0)
        if a.kind == "photo":
            fr = photo_covers(n, H, W, a.seed * 1000003 + i, dev)
        else:
            fr = batch.synth_frames(n, H, W, seed=batch.SEED_COVER + a.seed, frame0=f0, device=dev)
        st = {}
        oh = batch.embed_batch(fr, tile, b, a.alpha, stats=st, route="hybrid")
        orf = batch.embed_batch(fr, tile, b, a.alpha, route="reference")
        xh = batch.extract_batch(oh, fr, b, a.alpha, route="hybrid")
        xr = batch.extract_batch(orf, fr, b, a.alpha, route="reference")
        xs = batch.extract_batch(orf, fr, b, a.alpha, route="hybrid")
        torch.cuda.synchronize()
        row = dict(batch=i, frames=n, blocks=n * (H // b) * (W // b), dgesdd_route_blocks=int(st.get("lapack_blocks") or 0),
                   embed_bytes_differing=int((oh != orf).sum()), embed_blocks_differing=blocks_differing(oh, orf, b),
                   extract_bytes_differing=int((xh != xr).sum()),
                   extract_same_input_bytes_differing=int((xs != xr).sum()))
        for k in tot:
            tot[k] += row[k]
        print(json.dumps(row), flush=True)
        del fr, oh, orf, xh, xr, xs
    tot.update(block=b, kind=a.kind, wm=a.wm, frame=f"{W}x{H}", alpha=a.alpha, seconds=round(time.time() - t_start, 1))
    print(json.dumps({"total": tot}), flush=True)


if __name__ == "__main__":
    main()
