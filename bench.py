#!/usr/bin/env python3
"""Benchmark: Mpixels/s of the embed+extract round trip on a batch of 4K RGB frames.

BASELINE.json metric "Mpixels/s embed+extract, 4K RGB batch, 1/2/4/8 MI355X; % HBM
roofline", workload configs[2]: 4096 synthetic 3840x2160 RGB frames per GPU, b=8,
alpha=0.1, embed then extract (watermarking.py:135 and :224 per frame).

One step = (rank 0 broadcasts the watermark tile over RCCL when N > 1) + one embed
launch over the whole batch + one extract launch over the whole batch.  Frames are
generated in HBM before timing (SURVEY 8(d) generator); nothing crosses PCIe in the
timed region.  N > 1: one process per GPU (torch.distributed.run), weak scaling
(every rank processes its own `--frames` frames), no data-path collective besides
the tile broadcast; value = all ranks' pixels / max-over-ranks time.

Prints ONE JSON line on rank 0.  `roofline` is the embed kernel (the dominant one):
algorithmic bytes per launch / its mean launch time from HIP events on the launch
stream.  `cpu_baseline` times the oracle (oracle/, a C port of the reference's
arithmetic) on a bounded sample on this host's cores.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--frames", type=int, default=4096, help="frames per GPU (configs[2]: 4096)")
    p.add_argument("--height", type=int, default=2160)
    p.add_argument("--width", type=int, default=3840)
    p.add_argument("--block", type=int, default=8)
    p.add_argument("--alpha", type=float, default=0.1)
    p.add_argument("--cpu-frames", type=int, default=48,
                   help="frames in the CPU-baseline sample, ~10 s of oracle work on 16 cores (0 = skip)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                   help="process-group backend for N > 1 (nccl = RCCL over xGMI; gloo only to rehearse "
                        "several ranks on one GPU)")
    return p.parse_args()


def cpu_baseline(host_frames, host_tile, block, alpha):
    """Oracle (C restatement, OpenMP over block rows) on a bounded sample, this host's cores."""
    from oracle import oracle as O

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or O.default_threads()
    threads = max(1, min(threads, O.default_threads()))
    O.lib()
    n, h, w = host_frames.shape[:3]
    t0 = time.perf_counter()
    emb = O.embed_batch(host_frames, host_tile, block, alpha, threads)
    O.extract_batch(emb, host_frames, block, alpha, threads)
    dt = time.perf_counter() - t0
    return {
        "value": n * h * w / dt / 1e6,
        "unit": "Mpixels/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{n} synthetic {w}x{h} frames (the batch's first {n}), embed+extract round trip, "
                  f"oracle/tmfwm_oracle.c with {threads} OpenMP threads, {dt:.2f} s",
    }


def measured_copy_peak(torch, dev, nbytes=4 << 30, reps=5):
    """Device-to-device copy rate (read + write bytes / time) of a 4 GiB buffer: the
    measured stream-copy peak SURVEY 8(d) asks to quote beside the 8 TB/s spec."""
    src = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    dst = torch.empty_like(src)
    dst.copy_(src)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        dst.copy_(src)
    e1.record()
    e1.synchronize()
    gbs = 2 * nbytes * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9
    del src, dst
    torch.cuda.empty_cache()
    return round(gbs, 1)


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one GPU per rank; more ranks than GPUs only in a gloo rehearsal (ranks share a GPU)
    gpu = local % max(1, torch.cuda.device_count()) if args.backend == "gloo" else local
    dev = torch.device("cuda", gpu)
    torch.cuda.set_device(dev)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    from thatsmyface_amd import batch
    from thatsmyface_amd.dist import ShardedRoundTrip, max_over_ranks, shard_range

    F, H, W, b, alpha = args.frames, args.height, args.width, args.block, args.alpha
    nbh, nbw = H // b, W // b
    start, stop = shard_range(F * world, rank, world)  # weak scaling: F frames per GPU
    frames = batch.synth_frames(stop - start, H, W, seed=batch.SEED_COVER, frame0=start, device=dev)
    wm = batch.synth_tile(nbh, nbw, device=dev) if rank == 0 else torch.zeros((nbh, nbw), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()

    stream = torch.cuda.current_stream()
    marks = {}

    def hook(phase):
        e = torch.cuda.Event(enable_timing=True)
        e.record(stream)
        marks.setdefault(phase, []).append(e)

    rt = ShardedRoundTrip(
        embed_fn=lambda f, t, bb, a, o: batch.embed_batch(f, t, bb, a, out=o),
        extract_fn=lambda w_, o_, bb, a, out: batch.extract_batch(w_, o_, bb, a, out=out),
        frames=frames, tile=wm, block=b, alpha=alpha,
    )

    for _ in range(args.warmup):
        rt.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    rt.hooks.append(hook)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        rt.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = max_over_ranks(time.perf_counter() - t0, dev)
    ev = list(zip(marks["broadcast"], marks["embed"], marks["extract"]))

    embed_ms = sum(a.elapsed_time(m) for a, m, _ in ev) / len(ev)
    extract_ms = sum(m.elapsed_time(z) for _, m, z in ev) / len(ev)
    px_step = F * H * W * world
    value = px_step * args.steps / elapsed / 1e6

    embed_bytes = F * (6 * H * W + nbh * nbw)  # read 3HW + nh*nw, write 3HW per frame
    extract_bytes = F * (6 * H * W + nbh * nbw)  # read 6HW, write nh*nw per frame
    achieved = embed_bytes / (embed_ms * 1e-3) / 1e9

    traffic = None
    tp = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tp):
        try:
            with open(tp) as f:
                tj = json.load(f)
            key = f"{F}x{H}x{W}_b{b}"
            if key in tj.get("embed_kernel_hbm_bytes_per_launch", {}):
                traffic = tj["embed_kernel_hbm_bytes_per_launch"][key]
        except (OSError, ValueError):
            traffic = None

    # VALU-issue bound per frame (tools/valu.py: PMC instruction mix x measured issue costs)
    valu = {}
    vp = os.path.join(ROOT, "profiles", "valu.json")
    if os.path.exists(vp) and H == 2160 and W == 3840:
        try:
            with open(vp) as f:
                vk = json.load(f).get("kernels", {})
            for name, ms in ((f"embed_kernel<{b}>", embed_ms), (f"extract_kernel<{b}>", extract_ms)):
                if name in vk:
                    bound = vk[name]["valu_issue_bound_us_per_frame"]
                    got = ms * 1e3 / F
                    valu[name] = {"bound_us_per_frame": bound, "us_per_frame": round(got, 2), "frac": round(bound / got, 3)}
        except (OSError, ValueError, KeyError):
            valu = {}

    copy_gbs = measured_copy_peak(torch, dev) if rank == 0 else None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.cpu_frames > 0:
        k = min(args.cpu_frames, F)
        cpu = cpu_baseline(frames[:k].cpu().numpy(), wm.cpu().numpy(), b, alpha)

    if rank == 0:
        line = {
            "metric": "Mpixels/s embed+extract, 4K RGB batch",
            "value": round(value, 3),
            "unit": "Mpixels/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64+f32 (u8 I/O)",
            "data": "synthetic (splitmix64 uniform u8 covers + tile, generated in HBM)",
            "config": {
                "workload": f"{F} x {W}x{H} RGB frames per GPU, embed+extract round trip (configs[2])",
                "frames_per_gpu": F,
                "height": H,
                "width": W,
                "block": b,
                "alpha": alpha,
                "parallelism": f"frame shards x{world}, {'RCCL' if args.backend == 'nccl' else 'gloo'} tile broadcast",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": f"embed_kernel<{b}>",
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5),
                "traffic": traffic,
                "algorithmic_bytes_per_launch": embed_bytes,
                "launch_ms": round(embed_ms, 3),
                "copy_peak_measured_GBs": copy_gbs,
                "binding_bound": "VALU issue (DESIGN.md section 4), not HBM",
                "valu_issue": valu.get(f"embed_kernel<{b}>"),
            },
            "kernels_ms": {"embed": round(embed_ms, 3), "extract": round(extract_ms, 3),
                           "extract_GBs": round(extract_bytes / (extract_ms * 1e-3) / 1e9, 2),
                           "extract_valu_issue": valu.get(f"extract_kernel<{b}>")},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
