"""bench.py's launcher and multi-rank path on the CPU.

* `bench.py --gpus 2` without a GPU per rank must fail loudly, not measure one GPU.
* `bench.spawn_ranks` at world size 2 (gloo) runs bench.run() in two ranks
  (tests/bench_rank_cpu.py supplies oracle kernels on CPU tensors); the union of the
  shards equals a serial oracle run, rank 1 received rank 0's tile, and rank 0 prints
  one JSON line with both ranks' pixels and a parity sample from both ranks.
"""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from oracle import oracle as O  # noqa: E402


def test_gpus_without_gpus_fails_loudly():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--frames", "1"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "--gpus 2 needs 2 visible GPUs" in r.stderr


def test_spawn_parent_makes_no_gpu_call():
    """configs[3]: the launching process counts GPUs from sysfs and never imports torch
    (a HIP runtime initialised before the fork+exec of the ranks is refused on the pool)."""
    code = ("import sys; sys.path.insert(0, %r); import bench; n = bench.visible_gpu_count(); "
            "assert 'torch' not in sys.modules, 'torch imported'; print(n)") % ROOT
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() in ("None",) or int(r.stdout) >= 0
    src = open(os.path.join(ROOT, "bench.py")).read()
    body = src[src.index("def spawn_ranks("):src.index("def gpu_kernels(")]
    code_only = body.split('"""')[2]
    assert "import torch" not in code_only and "torch.cuda" not in code_only, "spawn_ranks must not touch torch"


def test_workload_names():
    assert bench.workload_name(4096, 2160, 3840, 8, 0.1, 1).startswith("configs[2]")
    assert bench.workload_name(4096, 2160, 3840, 8, 0.1, 8).startswith("configs[3]")
    assert bench.workload_name(256, 1080, 1920, 8, 0.1, 1).startswith("configs[1]")
    assert bench.workload_name(512, 2160, 3840, 16, 0.2, 1).startswith("configs[4]")
    assert bench.workload_name(3, 64, 96, 8, 0.1, 2).startswith("custom")


def test_bench_two_ranks_gloo(tmp_path, capfd):
    F, H, W, B, A = 3, 48, 80, 8, 0.1
    argv = ["--gpus", "2", "--backend", "gloo", "--frames", str(F), "--height", str(H), "--width", str(W),
            "--steps", "1", "--warmup", "0", "--block", str(B), "--alpha", str(A)]
    os.environ["TMF_BENCH_DUMP"] = str(tmp_path)
    try:
        rc = bench.spawn_ranks(bench.parse(argv), argv, script=os.path.join(ROOT, "tests", "bench_rank_cpu.py"))
    finally:
        del os.environ["TMF_BENCH_DUMP"]
    out = capfd.readouterr().out
    assert rc == 0, out
    lines = [json.loads(x) for x in out.splitlines() if x.startswith("{")]
    assert len(lines) == 1, out
    line = lines[0]
    assert line["n_ranks"] == 2 and line["config"]["frames_total"] == 2 * F
    assert line["parity_sample"]["frames"] == 2 * F and line["parity_sample"]["embed_mismatch"] == 0
    assert line["lapack_route_sample"] == f"{2 * F}/{2 * F}"
    assert "rehearsal" in line and line["value"] > 0

    frames = O.synth_bytes(0x5EED0001, 0, 2 * F, H * W * 3).reshape(2 * F, H, W, 3)
    tile = O.synth_bytes(0x5EED0002, 0, 1, (H // B) * (W // B)).reshape(H // B, W // B)
    ref = O.embed_batch(frames, tile, B, A, 1)
    refx = O.extract_batch(ref, frames, B, A, 1)
    got, gotx = np.zeros_like(ref), np.zeros_like(refx)
    for r in range(2):
        z = np.load(tmp_path / f"r{r}.npz")
        assert np.array_equal(z["tile"], tile), f"rank {r} tile broadcast"
        s = int(z["frame0"])
        got[s:s + len(z["out"])] = z["out"]
        gotx[s:s + len(z["tiles"])] = z["tiles"]
    assert np.array_equal(got, ref)
    assert np.array_equal(gotx, refx)


def _spawn(argv, tmp_path, fail=None, timeout=600):
    env = dict(os.environ, TMF_BENCH_DUMP=str(tmp_path))
    env.pop("WORLD_SIZE", None)
    if fail:
        env["TMF_BENCH_FAIL"] = fail
    code = ("import sys; sys.path.insert(0, %r); import bench; "
            "sys.exit(bench.spawn_ranks(bench.parse(sys.argv[1:]), sys.argv[1:], script=%r))"
            % (ROOT, os.path.join(ROOT, "tests", "bench_rank_cpu.py")))
    return subprocess.run([sys.executable, "-c", code] + argv, env=env, capture_output=True, text=True, timeout=timeout)


def test_bench_eight_ranks_gloo(tmp_path):
    """configs[3]'s launch path at world size 8 (gloo, oracle kernels on CPU tensors):
    the union of the 8 shards equals a serial oracle run, every rank holds rank 0's tile,
    and every rank's parity share (frames spread over its shard) is reported."""
    F, H, W, B, A = 2, 32, 48, 8, 0.1
    argv = ["--gpus", "8", "--backend", "gloo", "--frames", str(F), "--height", str(H), "--width", str(W),
            "--steps", "1", "--warmup", "1", "--block", str(B), "--alpha", str(A), "--cpu-frames", "16",
            "--lapack-frames", "8"]
    r = _spawn(argv, tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_ranks"] == 8 and line["config"]["frames_total"] == 8 * F
    assert line["parity_sample"]["frames"] == 16 and line["parity_sample"]["embed_mismatch"] == 0
    assert line["lapack_route_sample"] == "8/8"
    # self-contained N > 1 line: the host's CPU baseline -- every rank's share
    # checked concurrently, all ranks' pixels over the slowest rank's time -- and the spread of the
    # ranks' mean launch times; every frame of every shard checked against the reference route
    cb = line["cpu_baseline"]
    assert cb and cb["kind"] == "port" and cb["value"] > 0 and cb["cores"] >= 8 and len(cb["per_rank_s"]) == 8
    ex = line["exact_route_check"]
    assert ex["ranks"] == 8 and ex["frames"] == ex["of_frames"] == 8 * F and ex["embed_bytes_differing"] == 0
    lm = line["roofline"]["launch_ms_over_ranks"]
    assert lm["ranks"] == 8 and 0 < lm["min"] <= line["roofline"]["launch_ms"] <= lm["max"]
    xm = line["kernels_ms"]["extract_over_ranks"]
    assert 0 < xm["min"] <= line["kernels_ms"]["extract"] <= xm["max"]
    frames = O.synth_bytes(0x5EED0001, 0, 8 * F, H * W * 3).reshape(8 * F, H, W, 3)
    tile = O.synth_bytes(0x5EED0002, 0, 1, (H // B) * (W // B)).reshape(H // B, W // B)
    ref = O.embed_batch(frames, tile, B, A, 1)
    got = np.zeros_like(ref)
    for rk in range(8):
        z = np.load(tmp_path / f"r{rk}.npz")
        assert np.array_equal(z["tile"], tile), f"rank {rk} tile broadcast"
        s = int(z["frame0"])
        got[s:s + len(z["out"])] = z["out"]
    assert np.array_equal(got, ref)


import pytest  # noqa: E402


@pytest.mark.parametrize("mode", ["raise", "parity", "hang"])
def test_bench_eight_ranks_failure_ends_run(tmp_path, mode):
    """A rank that raises, fails parity or hangs makes the 8-rank run end with a non-zero
    status, with no rank left waiting in a collective (the hang ends through --pg-timeout)."""
    F, H, W = 1, 16, 32
    argv = ["--gpus", "8", "--backend", "gloo", "--frames", str(F), "--height", str(H), "--width", str(W),
            "--steps", "1", "--warmup", "1", "--cpu-frames", "8", "--lapack-frames", "0", "--pg-timeout", "20"]
    import time

    t0 = time.time()
    r = _spawn(argv, tmp_path, fail=f"5:{mode}", timeout=300)
    assert r.returncode != 0, r.stdout[-2000:]
    assert time.time() - t0 < 240
    if mode == "parity":
        assert "parity FAILED" in r.stderr


def test_bench_one_rank_cpu_baselines(tmp_path, capfd):
    """N = 1: the oracle CPU baseline + parity sample and the reference-cost-model baseline
    (oracle/structured.py on block-aligned crops) both run and report; with oracle kernels
    standing in for the GPU the crops must be bit-exact on this host's OpenBLAS core."""
    import subprocess
    import sys

    F, H, W, B = 2, 48, 80, 8
    env = dict(os.environ, TMF_BENCH_DUMP=str(tmp_path))
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "bench_rank_cpu.py"), "--frames", str(F), "--height",
                          str(H), "--width", str(W), "--steps", "1", "--warmup", "0", "--cpu-frames", "2",
                          "--structured-crops", "2"], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    line = json.loads([x for x in out.stdout.splitlines() if x.startswith("{")][-1])
    assert line["parity_sample"]["frames"] == 2 and line["parity_sample"]["embed_mismatch"] == 0
    assert line["cpu_baseline"]["kind"] == "port" and line["cpu_baseline"]["value"] > 0
    ex = line["exact_route_check"]  # every frame of the batch by default
    assert ex["frames"] == 2 and ex["of_frames"] == 2 and ex["blocks"] == 2 * (H // B) * (W // B)
    assert ex["embed_bytes_differing"] == 0 and ex["extract_bytes_differing"] == 0 and ex["reference_route_Mpx_per_s"] > 0
    rm = line["cpu_baseline_reference_model"]
    assert rm["value"] > 0 and rm["crops_bit_exact_vs_gpu"].endswith("/2")
    from test_oracle_lapack import _CORE

    if _CORE == "SkylakeX":
        assert rm["crops_bit_exact_vs_gpu"] == "2/2"
