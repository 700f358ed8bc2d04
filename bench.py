#!/usr/bin/env python3
"""Benchmark: Mpixels/s of the embed+extract round trip on a batch of RGB frames.

BASELINE.json metric "Mpixels/s embed+extract, 4K RGB batch, 1/2/4/8 MI355X; % HBM
roofline".  Default workload = configs[2]: 4096 synthetic 3840x2160 RGB frames per GPU,
b=8, alpha=0.1, embed then extract (watermarking.py:135 and :224 per frame).  At
--gpus 8 the same per-GPU batch is configs[3] (32,768 frames over 8 GPUs).

One step = (rank 0 broadcasts the watermark tile over RCCL when N > 1) + one embed
launch over the rank's whole shard + one extract launch over it.  Frames are generated
in HBM before timing (SURVEY 8(d) generator); nothing crosses PCIe in the timed region.

N > 1: one process per GPU.  Under torch.distributed.run (RANK/WORLD_SIZE in the env)
this process is one rank; started as `bench.py --gpus N` without them, it launches N
ranks itself (a child `python -m torch.distributed.run`, started before this process
touches a GPU) and exits with their status.  Weak scaling: every rank processes its own
`--frames` frames, a contiguous range of the global batch (thatsmyface_amd.dist);
value = all ranks' pixels / max-over-ranks time.  Ranks must sit on distinct GPUs
(checked by PCI id) unless `--backend gloo` rehearses several ranks on one GPU.

Prints ONE JSON line on rank 0.  `roofline` is the embed kernel (the dominant one):
algorithmic bytes per launch / its mean launch time from HIP events on the launch
stream.  `cpu_baseline` times the oracle (oracle/, a C port of the reference's
arithmetic) on a bounded sample on this host's cores; the same sample's oracle outputs
are compared with the timed batch's GPU outputs (`parity_sample`), and a mismatch
makes the run fail.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time
from types import SimpleNamespace

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
BASELINE_METRIC = "Mpixels/s embed+extract, 4K RGB batch, 1/2/4/8 MI355X; % HBM roofline"


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--frames", type=int, default=4096, help="frames per GPU (configs[2]/[3]: 4096)")
    p.add_argument("--height", type=int, default=2160)
    p.add_argument("--width", type=int, default=3840)
    p.add_argument("--block", type=int, default=8)
    p.add_argument("--alpha", type=float, default=0.1)
    p.add_argument("--cpu-frames", type=int, default=48,
                   help="frames in the CPU-baseline / parity sample, ~10-20 s of oracle work on 16 cores (0 = skip)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--structured-crops", type=int, default=16,
                   help="block-aligned 960x544 crops timed with the reference's cost model (oracle/structured.py), "
                        "one per host core; 0 = skip")
    p.add_argument("--lapack-frames", type=int, default=8,
                   help="frames of the parity sample also checked against the reference's own SVD arithmetic "
                        "(the oracle's dgesdd route, ~1 s per 4K frame per 16 cores; 0 = skip)")
    p.add_argument("--exact-frames", type=int, default=-1,
                   help="hybrid route only: frames of each rank's batch re-run on the GPU's reference route (the "
                        "dgesdd route for every block, exact by construction) after the timed region, timed and "
                        "compared byte for byte with the timed run's output; -1 = every frame (default), 0 = skip; "
                        "a differing byte fails the run (exit status 3)")
    p.add_argument("--pg-timeout", type=float, default=600.0,
                   help="seconds a rank may wait in a collective before the run fails (N > 1)")
    p.add_argument("--route", default="hybrid", choices=["hybrid", "reference", "rank1", "rank1_reference"],
                   help="SVD route (DESIGN.md 3.5): hybrid = Jacobi + byte certificate (the throughput route); "
                        "reference = the dgesdd route for every block (np.linalg.svd's arithmetic by construction); "
                        "rank1 = the hybrid route behind the rank-1 pre-pass (b = 8 / 16, photo mode, DESIGN.md 5); "
                        "rank1_reference = the reference route behind it")
    p.add_argument("--covers", default="noise", choices=["noise", "photo"],
                   help="synthetic covers: uniform bytes (configs[1]-[4], the default) or camera-like frames")
    p.add_argument("--wm", default="noise", choices=["noise", "qr"],
                   help="synthetic watermark tile: uniform bytes (the default) or a binary QR-style tile")
    p.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                   help="process-group backend for N > 1 (nccl = RCCL over xGMI; gloo only to rehearse "
                        "several ranks on one GPU)")
    return p.parse_args(argv)


def workload_name(F, H, W, b, alpha, world):
    """Which BASELINE.json config a run is (configs[0] is the CPU-only plumbing case)."""
    if (H, W) == (2160, 3840) and F == 4096 and b == 8 and world == 8:
        return "configs[3]: 32768-frame 4K batch over 8 GPUs"
    if (H, W) == (2160, 3840) and F == 4096 and b == 8 and world == 1:
        return "configs[2]: 4096 x 4K frames, embed+extract round trip, 1 GPU"
    if (H, W) == (2160, 3840) and b == 16:
        return f"configs[4]-style: {F} x 4K frames per GPU, b=16, alpha={alpha}"
    if (H, W) == (1080, 1920) and b == 8 and F == 256 and world == 1:
        return "configs[1]: 256 x 1080p frames, 1 GPU"
    return f"custom: {F} x {W}x{H} frames per GPU x {world}, b={b}, alpha={alpha}"


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def visible_gpu_count():
    """GPUs this process could open, counted WITHOUT initialising HIP (no torch.cuda call:
    a HIP runtime initialised in this process must not precede the fork+exec of the
    ranks).  KFD topology nodes with SIMDs whose render node exists in /dev/dri (a
    container only gets the render nodes of its GPUs), narrowed by the *_VISIBLE_DEVICES
    masks.  None when the topology is unreadable (then the ranks check for themselves)."""
    import glob

    if not os.path.isdir("/sys/class/kfd"):
        return 0  # no amdgpu KFD driver: no GPU at all
    base = "/sys/class/kfd/kfd/topology/nodes"
    nodes = glob.glob(os.path.join(base, "*", "properties"))
    if not nodes:
        return None
    n = 0
    for path in nodes:
        try:
            with open(path) as f:
                props = dict(line.split()[:2] for line in f if len(line.split()) >= 2)
        except OSError:
            continue
        if int(props.get("simd_count", "0")) <= 0:
            continue
        minor = props.get("drm_render_minor")
        if minor is not None and not os.path.exists(f"/dev/dri/renderD{minor}"):
            continue
        n += 1
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip() != ""]))
    return n


def spawn_ranks(args, argv, script=None) -> int:
    """Launch args.gpus ranks of this script under torch.distributed.run and return their
    exit status.  This process makes no GPU call at all (it does not even import torch):
    the GPU count comes from sysfs (visible_gpu_count), and the ranks are children, never
    an exec of this process.  torch.distributed.run ends every rank as soon as one fails,
    and each rank's process group carries a timeout (--pg-timeout), so a failing or stuck
    rank ends the run with a non-zero status instead of leaving the others in a collective."""
    if args.backend == "nccl":
        ndev = visible_gpu_count()
        if ndev is not None and ndev < args.gpus:
            print(f"bench.py: --gpus {args.gpus} needs {args.gpus} visible GPUs, this box has {ndev} "
                  "(use --backend gloo to rehearse several ranks on one GPU)", file=sys.stderr, flush=True)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", script or os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def gpu_kernels(route="hybrid", covers="noise", wm="noise"):
    """The product path: libtmfwm.so's HIP kernels (thatsmyface_amd.batch).  covers / wm: the
    synthetic inputs (noise bytes, the default; or camera-like frames and a binary QR-style tile)."""
    from thatsmyface_amd import batch

    if covers == "photo":
        synth = lambda n, h, w, frame0, dev: batch.synth_photo_frames(n, h, w, seed=batch.SEED_COVER, frame0=frame0, device=dev)  # noqa: E731
    else:
        synth = lambda n, h, w, frame0, dev: batch.synth_frames(n, h, w, seed=batch.SEED_COVER, frame0=frame0, device=dev)  # noqa: E731
    return SimpleNamespace(
        synth_frames=synth,
        synth_tile=(lambda nbh, nbw, dev: batch.synth_qr_tile(nbh, nbw, device=dev)) if wm == "qr" else
                   (lambda nbh, nbw, dev: batch.synth_tile(nbh, nbw, device=dev)),
        embed=lambda f, t, b, a, o: batch.embed_batch(f, t, b, a, out=o, route=route),
        extract=lambda w_, o_, b, a, out: batch.extract_batch(w_, o_, b, a, out=out, route=route),
        embed_stats=lambda f, t, b, a, o: (lambda st: (batch.embed_batch(f, t, b, a, out=o, stats=st, route=route), st)[1])({}),
        embed_list_pass=lambda b: batch.embed_list_pass(b) and route != "reference",
        route=route,
        exact_embed=lambda f, t, b, a, o: batch.embed_batch(f, t, b, a, out=o, route="reference"),
        exact_extract=lambda w_, o_, b, a, out: batch.extract_batch(w_, o_, b, a, out=out, route="reference"),
    )


def exact_route_check(K, frames, tile, out, tiles, block, alpha, n, on_gpu, chunk=64):
    """The timed (hybrid-route) output against the reference route's, both on the GPU
    (DESIGN.md 3.5), over the first n frames of this rank's batch (n < 0: every frame), in
    chunks of `chunk` frames after the timed region.  The reference route runs the dgesdd route
    on every block -- np.linalg.svd's arithmetic by construction -- so this compares every timed
    byte with the reference's arithmetic (watermarking.py:135 embed, :224 extract of the GPU's
    own watermarked frames).  Also times the reference route (embed + extract per chunk)."""
    import torch

    total = frames.shape[0]
    n = total if n < 0 else min(n, total)
    if n <= 0 or not hasattr(K, "exact_embed"):
        return None
    c = min(chunk, n)
    eo, et = torch.empty_like(frames[:c]), torch.empty_like(tiles[:c])
    K.exact_embed(frames[:c], tile, block, alpha, eo)  # warm: first call sizes the pools
    sync = torch.cuda.synchronize if on_gpu else (lambda: None)
    sync()
    diff_e = diff_x = frames_e = frames_x = 0
    dt = 0.0
    for s in range(0, n, c):
        e = min(n, s + c)
        f, m = frames[s:e], e - s
        t0 = time.perf_counter()
        K.exact_embed(f, tile, block, alpha, eo[:m])
        K.exact_extract(eo[:m], f, block, alpha, et[:m])
        sync()
        dt += time.perf_counter() - t0
        de = (eo[:m] != out[s:e]).reshape(m, -1).sum(dim=1)
        dx = (et[:m] != tiles[s:e]).reshape(m, -1).sum(dim=1)
        diff_e += int(de.sum())
        diff_x += int(dx.sum())
        frames_e += int((de != 0).sum())
        frames_x += int((dx != 0).sum())
    H, W = frames.shape[1], frames.shape[2]
    return {"frames": n, "of_frames": total, "blocks": n * (H // block) * (W // block),
            "embed_bytes_differing": diff_e, "extract_bytes_differing": diff_x,
            "frames_differing": max(frames_e, frames_x),
            "reference_route_Mpx_per_s": round(n * H * W / dt / 1e6, 1) if dt > 0 else None,
            "what": "every timed (hybrid-route) output byte of these frames vs the GPU reference route (dgesdd "
                    f"route on every block), {c}-frame chunks after the timed region; reference-route rate = "
                    "embed + extract of those frames"}


def oracle_check(host_frames, host_tile, out, tiles, block, alpha, threads):
    """Oracle (C restatement, OpenMP) on k frames: (seconds, embed mismatches, extract mismatches).
    The checker and the CPU baseline are the same computation, timed once."""
    import numpy as np

    from oracle import oracle as O

    O.lib()
    t0 = time.perf_counter()
    emb = O.embed_batch(host_frames, host_tile, block, alpha, threads)
    ext = O.extract_batch(emb, host_frames, block, alpha, threads)
    dt = time.perf_counter() - t0
    bad_e = int(sum(not np.array_equal(emb[i], out[i]) for i in range(len(emb))))
    bad_x = int(sum(not np.array_equal(ext[i], tiles[i]) for i in range(len(ext))))
    return dt, bad_e, bad_x


def lapack_check(host_frames, host_tile, out, tiles, block, alpha, threads):
    """The reference's own SVD arithmetic on k frames: every block through the oracle's
    dgesdd route (np.linalg.svd restated, pinned bit for bit against numpy).  Extract is
    run on the GPU's watermarked frames, the input the GPU's extract consumed.
    Returns (frames, embed mismatches, extract mismatches)."""
    import numpy as np

    from oracle import oracle as O

    bad_e = bad_x = 0
    for i in range(len(host_frames)):
        emb = O.embed_frame(host_frames[i], host_tile, block, alpha, threads, route="lapack")
        ext = O.extract_frame(out[i], host_frames[i], block, alpha, threads, route="lapack")
        bad_e += int(not np.array_equal(emb, out[i]))
        bad_x += int(not np.array_equal(ext, tiles[i]))
    return len(host_frames), bad_e, bad_x


def oracle_threads(world: int) -> int:
    from oracle import oracle as O

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or O.default_threads()
    threads = max(1, min(threads, O.default_threads()))
    return max(1, threads // max(1, world)) if world > 1 else threads


def measured_copy_peak(torch, dev, nbytes=4 << 30, reps=5):
    """Device-to-device copy rate (read + write bytes / time) of a 4 GiB buffer by torch's
    uint8 copy_ -- a lower bound of the copy peak SURVEY 8(d) asks to quote beside the 8 TB/s
    spec (the guide's dwordx4 stream copy measured 6.29 TB/s)."""
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


def _device_id(torch, dev):
    if dev.type != "cuda":
        return f"cpu:{socket.gethostname()}"
    p = torch.cuda.get_device_properties(dev)
    return f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x} {p.uuid}"


def _profile_json(name):
    path = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def kernel_code_ids():
    """kernel -> code id of the loaded build (libtmfwm.kernels.json next to the library)."""
    from thatsmyface_amd import _lib

    path = os.path.splitext(_lib.LIB_PATH)[0] + ".kernels.json"
    try:
        with open(path) as f:
            return json.load(f).get("kernels", {})
    except (OSError, ValueError):
        return {}


def lib_build_id():
    """sha256 prefix of the loaded libtmfwm.so: profiles/*.json record the build they measured."""
    import hashlib

    from thatsmyface_amd import _lib

    try:
        with open(_lib.LIB_PATH, "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()[:16]
    except OSError:
        return None


def run(args, kernels=None, device=None):
    """One rank of the benchmark.  `kernels` / `device` default to the HIP path on this
    rank's GPU; the CPU test of the multi-rank code substitutes its own (tests/)."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from thatsmyface_amd.dist import ShardedRoundTrip, max_over_ranks, shard_range

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if device is None:
        ndev = torch.cuda.device_count()
        if ndev == 0:
            raise SystemExit("bench.py: no GPU visible (the product path has no CPU fallback)")
        if args.backend == "nccl" and local >= ndev:
            raise SystemExit(f"bench.py: local rank {local} has no GPU of its own ({ndev} visible)")
        gpu = local % ndev  # gloo rehearsal: ranks may share a GPU
        device = torch.device("cuda", gpu)
        torch.cuda.set_device(device)
    dev = device
    on_gpu = dev.type == "cuda"
    if world > 1:
        import datetime

        timeout = datetime.timedelta(seconds=args.pg_timeout)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev, timeout=timeout)
        else:
            dist.init_process_group("gloo", timeout=timeout)
    K = kernels or gpu_kernels(getattr(args, "route", "hybrid"), getattr(args, "covers", "noise"), getattr(args, "wm", "noise"))
    sync = torch.cuda.synchronize if on_gpu else (lambda: None)

    # distinct physical devices across ranks
    ids = [_device_id(torch, dev)]
    if world > 1:
        ids = [None] * world
        dist.all_gather_object(ids, _device_id(torch, dev))
    n_phys = len(set(ids))
    if on_gpu and args.backend == "nccl" and n_phys != world:
        raise SystemExit(f"bench.py: {world} ranks share {n_phys} GPUs ({ids}); RCCL needs one GPU per rank")

    F, H, W, b, alpha = args.frames, args.height, args.width, args.block, args.alpha
    nbh, nbw = H // b, W // b
    start, stop = shard_range(F * world, rank, world)  # weak scaling: F frames per GPU
    frames = K.synth_frames(stop - start, H, W, start, dev)
    wm = K.synth_tile(nbh, nbw, dev) if rank == 0 else torch.zeros((nbh, nbw), dtype=torch.uint8, device=dev)
    sync()

    marks = {}
    if on_gpu:
        stream = torch.cuda.current_stream()

        def hook(phase):
            e = torch.cuda.Event(enable_timing=True)
            e.record(stream)
            marks.setdefault(phase, []).append(e)
    else:
        def hook(phase):
            marks.setdefault(phase, []).append(time.perf_counter())

    rt = ShardedRoundTrip(embed_fn=K.embed, extract_fn=K.extract, frames=frames, tile=wm, block=b, alpha=alpha)

    # the timing hooks run in the warmup steps too, so the timed steps pay no first-use cost
    # (the first event records of a process take milliseconds on the host)
    rt.hooks.append(hook)
    for _ in range(args.warmup):
        rt.step()
    # how one embed call over this rank's whole batch splits its work (untimed; the same bytes
    # are rewritten, and every embed launch of the run has the same size, so a kernel trace's
    # averages are the timed launches'): blocks the strip pass left to the list pass, blocks
    # on the dgesdd route
    work = None
    if hasattr(K, "embed_stats") and stop > start:
        st = K.embed_stats(frames, wm, b, alpha, rt.out)
        work = {"frames": stop - start, "blocks": (stop - start) * nbh * nbw,
                "list_pass_blocks": st.get("list_pass_blocks"), "dgesdd_route_blocks": st.get("lapack_blocks")}
    sync()
    if world > 1:
        dist.barrier()
    sync()
    marks.clear()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        rt.step()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    elapsed = max_over_ranks(time.perf_counter() - t0, dev)
    ev = list(zip(marks["broadcast"], marks["embed"], marks["extract"]))
    if on_gpu:
        embed_ms = sum(a.elapsed_time(m) for a, m, _ in ev) / len(ev)
        extract_ms = sum(m.elapsed_time(z) for _, m, z in ev) / len(ev)
    else:
        embed_ms = sum(m - a for a, m, _ in ev) / len(ev) * 1e3
        extract_ms = sum(z - m for _, m, z in ev) / len(ev) * 1e3
    # every rank's mean launch times (the line's roofline is rank 0's; N > 1 adds the spread)
    launch_ranks = [(embed_ms, extract_ms)]
    if world > 1:
        launch_ranks = [None] * world
        dist.all_gather_object(launch_ranks, (embed_ms, extract_ms))
    px_step = F * H * W * world
    value = px_step * args.steps / elapsed / 1e6

    # SURVEY 8(d) algorithmic bytes per frame
    embed_read, embed_write = 3 * H * W + nbh * nbw, 3 * H * W
    embed_bytes = F * (embed_read + embed_write)
    extract_bytes = F * (6 * H * W + nbh * nbw)
    achieved = embed_bytes / (embed_ms * 1e-3) / 1e9
    achieved_read = F * embed_read / (embed_ms * 1e-3) / 1e9

    # every rank compares its timed output with the reference route (all of it by default)
    exact = None
    if getattr(K, "route", "hybrid") != "reference" and args.exact_frames != 0:
        exact = exact_route_check(K, frames, wm, rt.out, rt.tiles, b, alpha, args.exact_frames, on_gpu)
        if world > 1:
            cdev = dev if args.backend == "nccl" else "cpu"
            mine = exact or {}
            v = torch.tensor([mine.get(k, 0) for k in ("frames", "of_frames", "blocks", "embed_bytes_differing",
                                                       "extract_bytes_differing", "frames_differing")],
                             dtype=torch.int64, device=cdev)
            dist.all_reduce(v)
            rates = [None] * world
            dist.all_gather_object(rates, mine.get("reference_route_Mpx_per_s"))
            if exact is not None:
                exact = dict(exact, **dict(zip(("frames", "of_frames", "blocks", "embed_bytes_differing",
                                                "extract_bytes_differing", "frames_differing"), (int(x) for x in v.cpu()))),
                             reference_route_Mpx_per_s=rates[0], ranks=world,
                             reference_route_Mpx_per_s_over_ranks=rates)

    # parity of the timed batch against the oracle.  N = 1: rank 0 checks the CPU-baseline
    # sample (the batch's first --cpu-frames frames); N > 1: every rank checks its share of
    # --cpu-frames, spread evenly over its shard.  The first --lapack-frames of the sample
    # (N > 1: their share per rank) are also checked against the oracle's dgesdd route,
    # i.e. np.linalg.svd's own arithmetic (tmfwm_lapack.c), not the device contract's
    # conditioning flag, which the default (hybrid) route shares with the GPU.
    cpu, parity = None, None
    n_local = stop - start
    # N = 1: rank 0 times the sample on all host cores; N > 1: every rank checks its share at
    # the same time on cores / world, and the baseline is the host's: all ranks' checked pixels
    # over the slowest rank's time, on the cores all ranks used
    want_cpu = rank == 0 and not args.no_cpu_baseline and args.cpu_frames > 0 and n_local > 0
    checked = bad_e = bad_x = 0
    dt, threads = None, 0
    lp_checked = lp_bad_e = lp_bad_x = 0
    if (want_cpu and world == 1) or (world > 1 and n_local > 0 and args.cpu_frames > 0):
        if world == 1:
            idx = list(range(min(args.cpu_frames, n_local)))
        else:
            k = min(n_local, max(1, -(-args.cpu_frames // world)))
            idx = sorted({int(round(x)) for x in np.linspace(0, n_local - 1, k)})
        threads = oracle_threads(world)
        host = frames[idx].cpu().numpy()
        host_tile = wm.cpu().numpy()
        gout, gtiles = rt.out[idx].cpu().numpy(), rt.tiles[idx].cpu().numpy()
        dt, bad_e, bad_x = oracle_check(host, host_tile, gout, gtiles, b, alpha, threads)
        checked = len(idx)
        n_lp = min(checked, args.lapack_frames if world == 1 else -(-args.lapack_frames // world))
        lp_checked, lp_bad_e, lp_bad_x = lapack_check(host[:n_lp], host_tile, gout[:n_lp], gtiles[:n_lp], b, alpha, threads)
        if want_cpu and world == 1:
            cpu = {
                "value": round(checked * H * W / dt / 1e6, 3),
                "unit": "Mpixels/s",
                "cores": threads,
                "kind": "port",
                "sample": f"{checked} synthetic {W}x{H} frames (the batch's first {checked}), embed+extract round trip, "
                          f"oracle/tmfwm_oracle.c with {threads} OpenMP threads, {dt:.2f} s",
            }
    if world > 1 and args.cpu_frames > 0:  # the host's baseline: every rank's share, checked concurrently
        shares = [None] * world
        dist.all_gather_object(shares, (checked, dt, threads))
        done = [(c, t, th) for c, t, th in shares if c and t]
        if want_cpu and done:
            px, slow_dt, cores = sum(c for c, _, _ in done) * H * W, max(t for _, t, _ in done), sum(th for _, _, th in done)
            cpu = {
                "value": round(px / slow_dt / 1e6, 3),
                "unit": "Mpixels/s",
                "cores": cores,
                "kind": "port",
                "sample": f"{sum(c for c, _, _ in done)} synthetic {W}x{H} frames (the parity sample, spread over the "
                          f"{world} ranks' shards and checked concurrently, {cores // max(1, len(done))} OpenMP threads per "
                          f"rank), embed+extract round trip, oracle/tmfwm_oracle.c; all ranks' pixels / the slowest "
                          f"rank's {slow_dt:.2f} s",
                "per_rank_s": [round(t, 2) for _, t, _ in done],
            }
    if world > 1:  # every rank joins, checked or not
        cdev = dev if args.backend == "nccl" else "cpu"
        counts = torch.tensor([checked, bad_e, bad_x, lp_checked, lp_bad_e, lp_bad_x], dtype=torch.int64, device=cdev)
        dist.all_reduce(counts)
        checked, bad_e, bad_x, lp_checked, lp_bad_e, lp_bad_x = (int(v) for v in counts.cpu())
    if checked:
        parity = {"frames": checked, "embed_mismatch": bad_e, "extract_mismatch": bad_x,
                  "summary": f"{checked - max(bad_e, bad_x)}/{checked} frames bit-exact vs oracle"}
    lapack_sample = None
    if lp_checked:
        ok = lp_checked - max(lp_bad_e, lp_bad_x)
        lapack_sample = {"frames": lp_checked, "embed_mismatch": lp_bad_e, "extract_mismatch": lp_bad_x,
                         "route": "oracle dgesdd route for every block (np.linalg.svd's arithmetic, tmfwm_lapack.c)",
                         "summary": f"{ok}/{lp_checked}"}

    # the reference's own cost model: per-pixel np.dot colour loops and
    # per-block scipy / LAPACK calls (oracle/structured.py) on block-aligned crops of the
    # batch's first frames, one single-threaded process per host core; each crop's bytes are
    # compared with the same region of the GPU's output (equal where this host's OpenBLAS
    # core is the reference's SkylakeX)
    structured = None
    if want_cpu and world == 1 and args.structured_crops > 0:
        from oracle import structured as ST

        ch, cw = min(H, 68 * b), min(W, 120 * b)
        k = min(args.structured_crops, n_local)
        idx = list(range(k))
        covers = list(frames[idx, :ch, :cw].cpu().numpy())
        tiles = [wm[: ch // b, : cw // b].cpu().numpy()] * k
        res, wall = ST.run_pool(covers, tiles, b, alpha, oracle_threads(1))
        gout = rt.out[idx, :ch, :cw].cpu().numpy()
        gext = rt.tiles[idx, : ch // b, : cw // b].cpu().numpy()
        same = sum(int(np.array_equal(r[1], gout[i]) and np.array_equal(r[2], gext[i])) for i, r in enumerate(res))
        structured = {
            "value": round(k * ch * cw / wall / 1e6, 4),
            "unit": "Mpixels/s",
            "cores": oracle_threads(1),
            "kind": "reference cost model (oracle/structured.py: the reference's per-pixel np.dot and per-block "
                    "scipy.fftpack / np.linalg.svd loops, one single-threaded process per core)",
            "sample": f"{k} crops of {cw}x{ch} from the batch's first {k} frames, embed+extract, {wall:.2f} s wall",
            "per_crop_s": round(sum(r[0] for r in res) / k, 2),
            "crops_bit_exact_vs_gpu": f"{same}/{k}",
        }
    copy_gbs = measured_copy_peak(torch, dev) if rank == 0 and on_gpu else None
    build = lib_build_id() if on_gpu else None

    # Counter-derived figures (tools/pmc_embed.sh -> tools/valu.py -> profiles/valu.json) are
    # used only for the device code they measured: each entry carries its kernel's code id (a
    # hash of the kernel's own machine code and descriptors, tools/kernel_ids.py ->
    # libtmfwm.kernels.json, written when the library is linked), so a rebuild that leaves the
    # kernel's code unchanged keeps its profile.
    ids = kernel_code_ids() if on_gpu else {}
    vj = _profile_json("valu.json")

    def profiled(name):
        k = (vj or {}).get("kernels", {}).get(name)
        if k and k.get("code_id") and k.get("code_id") == ids.get(name) and (k.get("height"), k.get("width")) == (H, W):
            return k
        return None

    # HBM bytes of the embed launch: counted FETCH / WRITE bytes per frame x frames
    # (hybrid route only: the other routes launch other kernels)
    route = getattr(K, "route", "hybrid")
    traffic = None
    ek = profiled(f"embed_kernel<{b}>") if route == "hybrid" else None
    if ek and ek.get("hbm_bytes_per_frame"):
        traffic = int(ek["hbm_bytes_per_frame"] * F)

    # VALU-issue roofline: the spec-rate issue cycles per frame over this run's cycles per
    # frame at the clock the counter pass measured (GRBM_GUI_ACTIVE), i.e. the fraction of
    # peak VALU issue
    valu = {}
    for name, ms in ((f"embed_kernel<{b}>", embed_ms), (f"extract_kernel<{b}>", extract_ms)):
        k = profiled(name) if route == "hybrid" or name.startswith("extract") and route != "reference" else None
        if k and k.get("clock_MHz"):
            got = ms * 1e3 / F
            frac = k["issue_bound_cycles_per_frame"] / (got * k["clock_MHz"])
            valu[name] = {"valu_instr_per_wave": k["valu_instr_per_wave"], "f64_per_wave": k["f64_arith_per_wave"],
                          "bound_us_per_frame_at_clock": k["valu_issue_bound_us_per_frame"],
                          "clock_MHz": k["clock_MHz"], "us_per_frame": round(got, 2), "issue_fraction": round(frac, 3),
                          "code_id": k["code_id"]}

    if rank == 0:
        is4k = (H, W) == (2160, 3840)
        line = {
            "metric": BASELINE_METRIC if is4k else f"Mpixels/s embed+extract, {W}x{H} RGB batch",
            "value": round(value, 3),
            "unit": "Mpixels/s",
            "n_gpus": n_phys if on_gpu else 0,
            "n_ranks": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64+f32 (u8 I/O)",
            "data": ("synthetic (splitmix64 uniform u8 covers + tile, generated in HBM)"
                     if getattr(args, "covers", "noise") == "noise" and getattr(args, "wm", "noise") == "noise" else
                     f"synthetic ({getattr(args, 'covers', 'noise')} covers, {getattr(args, 'wm', 'noise')} tile, generated in HBM)"),
            "config": {
                "workload": workload_name(F, H, W, b, alpha, world) + (
                    "" if getattr(args, "covers", "noise") == "noise" and getattr(args, "wm", "noise") == "noise" else
                    f" [{getattr(args, 'covers', 'noise')} covers, {getattr(args, 'wm', 'noise')} watermark]"),
                "frames_per_gpu": F,
                "frames_total": F * world,
                "height": H,
                "width": W,
                "block": b,
                "alpha": alpha,
                "svd_route": getattr(args, "route", "hybrid"),
                "parallelism": ("single GPU" if world == 1 else
                                f"frame shards x{world}, {'RCCL' if args.backend == 'nccl' else 'gloo'} tile broadcast"),
            },
            "roofline": {
                "bound": "hbm",
                "kernel": {"reference": f"embed_fixup_kernel<{b}>"}.get(route, f"embed_rank1_kernel<{b}>" if route.startswith("rank1") else f"embed_kernel<{b}>"),
                "launch": {
                    "hybrid": (f"one tmfwm_embed call: embed_kernel<{b}> strip pass"
                               + (" + list pass" if getattr(K, "embed_list_pass", lambda _b: False)(b) else "")
                               + f" + embed_fixup_kernel<{b}> (dgesdd route)"),
                    "reference": f"one tmfwm_embed_route call, TMFWM_ROUTE_REFERENCE: embed_fixup_kernel<{b}> (dgesdd route) on every block",
                    "rank1": (f"one tmfwm_embed_route call, TMFWM_ROUTE_RANK1: embed_rank1_kernel<{b}> (rank-1 pre-pass) + "
                              f"embed_kernel<{b}> list pass (hybrid route) + embed_fixup_kernel<{b}> (dgesdd route)"),
                    "rank1_reference": (f"one tmfwm_embed_route call, TMFWM_ROUTE_RANK1_REFERENCE: embed_rank1_kernel<{b}> "
                                        f"(rank-1 pre-pass) + embed_fixup_kernel<{b}> (dgesdd route) on the blocks it leaves"),
                }[route],
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5),
                "traffic": traffic,
                "read_achieved": round(achieved_read, 2),
                "read_frac": round(achieved_read / HBM_PEAK_GBS, 5),
                "algorithmic_bytes_per_launch": embed_bytes,
                "launch_ms": round(embed_ms, 3),
                "launch_ms_over_ranks": {"max": round(max(e for e, _ in launch_ranks), 3),
                                         "min": round(min(e for e, _ in launch_ranks), 3), "ranks": world},
                # a torch uint8 copy_ (its own elementwise kernel), not a dwordx4 stream copy: the
                # guide's measured stream-copy peak is quoted beside it (MI355X_MICROARCH.md)
                "torch_copy_measured_GBs": copy_gbs,
                "stream_copy_peak_guide_GBs": 6290.0,
                "binding_bound": "VALU issue (DESIGN.md section 4), not HBM",
                "valu_issue": valu.get(f"embed_kernel<{b}>"),
            },
            "kernels_ms": {"embed": round(embed_ms, 3), "extract": round(extract_ms, 3),
                           "extract_over_ranks": {"max": round(max(x for _, x in launch_ranks), 3),
                                                  "min": round(min(x for _, x in launch_ranks), 3)},
                           "extract_GBs": round(extract_bytes / (extract_ms * 1e-3) / 1e9, 2),
                           "extract_valu_issue": valu.get(f"extract_kernel<{b}>")},
            "embed_work_sample": work,
            "parity_sample": parity,
            "lapack_route_sample": lapack_sample["summary"] if lapack_sample else None,
            "lapack_route_detail": lapack_sample,
            "exact_route_check": exact,
            "cpu_baseline": cpu,
            "cpu_baseline_reference_model": structured,
            "lib_build": build,
            "kernel_code_ids": {k: ids.get(k) for k in (f"embed_kernel<{b}>", f"extract_kernel<{b}>")} if on_gpu else None,
        }
        if world > 1 and args.backend == "gloo":
            line["rehearsal"] = f"gloo: {world} ranks on {n_phys} device(s); not a multi-GPU measurement"
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if parity and (parity["embed_mismatch"] or parity["extract_mismatch"]):
        print(f"bench.py: parity FAILED on rank {rank}: {parity}", file=sys.stderr, flush=True)
        return 3
    if lapack_sample and (lapack_sample["embed_mismatch"] or lapack_sample["extract_mismatch"]):
        print(f"bench.py: parity vs the dgesdd route FAILED on rank {rank}: {lapack_sample}", file=sys.stderr, flush=True)
        return 3
    if exact and (exact["embed_bytes_differing"] or exact["extract_bytes_differing"]):
        print(f"bench.py: the timed output differs from the GPU reference route on rank {rank}: {exact}",
              file=sys.stderr, flush=True)
        return 3
    return 0


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(args, argv)
    return run(args)


if __name__ == "__main__":
    sys.exit(main())
