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
    assert line["parity_sample"]["frames"] == 2 and line["parity_sample"]["embed_mismatch"] == 0
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
    rm = line["cpu_baseline_reference_model"]
    assert rm["value"] > 0 and rm["crops_bit_exact_vs_gpu"].endswith("/2")
    from test_oracle_lapack import _CORE

    if _CORE == "SkylakeX":
        assert rm["crops_bit_exact_vs_gpu"] == "2/2"
