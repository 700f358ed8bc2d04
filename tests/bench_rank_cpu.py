"""One rank of bench.py on the CPU (gloo), for tests/test_bench_cli.py.

bench.py's own multi-rank code (spawn_ranks -> torch.distributed.run -> run(): shard
ranges, tile broadcast, barriers, max-over-ranks timing, parity all-reduce, the JSON
line) runs unchanged; only the per-rank kernels are the oracle's, on CPU tensors,
because this container has no GPU.  Each rank saves its shard's outputs to
$TMF_BENCH_DUMP so the test can compare the union with a serial oracle run.

TMF_BENCH_FAIL="<rank>:<mode>" injects a failure into one rank's timed embed: "raise"
(an exception), "parity" (one corrupted output byte) or "hang" (the rank never returns;
the others must end through the process-group timeout).
"""
import os
import sys
from types import SimpleNamespace

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from oracle import oracle as O  # noqa: E402

SEED_COVER, SEED_WM = 0x5EED0001, 0x5EED0002


def main():
    args = bench.parse(sys.argv[1:])
    rank = int(os.environ.get("RANK", "0"))
    dump = os.environ["TMF_BENCH_DUMP"]
    state = {}

    def synth_frames(n, h, w, frame0, dev):
        state["frame0"] = frame0
        return torch.from_numpy(O.synth_bytes(SEED_COVER, frame0, n, h * w * 3).reshape(n, h, w, 3))

    fail_rank, _, fail_mode = os.environ.get("TMF_BENCH_FAIL", "-1:").partition(":")
    calls = [0]

    def embed(f, t, b, a, o):
        o.copy_(torch.from_numpy(O.embed_batch(f.numpy(), t.numpy(), b, a, 1)))
        state["tile"] = t.numpy().copy()
        calls[0] += 1
        if rank == int(fail_rank) and calls[0] > args.warmup:
            if fail_mode == "raise":
                raise RuntimeError(f"injected failure on rank {rank}")
            if fail_mode == "parity":
                o.view(-1)[0] ^= 1
            if fail_mode == "hang":
                import time

                time.sleep(3600)

    def extract(w, o, b, a, out):
        out.copy_(torch.from_numpy(O.extract_batch(w.numpy(), o.numpy(), b, a, 1)))
        np.savez(os.path.join(dump, f"r{rank}.npz"), out=w.numpy(), tiles=out.numpy(), tile=state["tile"],
                 frame0=state["frame0"])

    K = SimpleNamespace(
        synth_frames=synth_frames,
        synth_tile=lambda nbh, nbw, dev: torch.from_numpy(O.synth_bytes(SEED_WM, 0, 1, nbh * nbw).reshape(nbh, nbw)),
        embed=embed,
        extract=extract,
        # the GPU's reference route stands in as the oracle's dgesdd route
        exact_embed=lambda f, t, b, a, o: o.copy_(torch.from_numpy(np.stack(
            [O.embed_frame(x, t.numpy(), b, a, 1, route="lapack") for x in f.numpy()]))),
        exact_extract=lambda w, o, b, a, out: out.copy_(torch.from_numpy(np.stack(
            [O.extract_frame(x, y, b, a, 1, route="lapack") for x, y in zip(w.numpy(), o.numpy())]))),
    )
    return bench.run(args, kernels=K, device=torch.device("cpu"))


if __name__ == "__main__":
    sys.exit(main())
