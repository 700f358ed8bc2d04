"""Multi-GPU driver: one process per GPU, frames sharded, watermark tile broadcast.

Frames are independent (watermarking.py:183-210 iterates independent blocks; no
halo), so a batch splits into contiguous frame ranges, one per rank, with no
data-path collective.  The only exchange is the watermark tile: rank 0 holds it
(the app resizes it with PIL on the host, watermarking.py:177) and broadcasts it
to every rank -- RCCL over xGMI when the backend is "nccl" (ROCm), gloo on CPU.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable

import torch
import torch.distributed as dist


def world() -> tuple[int, int]:
    """(rank, world_size); (0, 1) without an initialised process group."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard_range(n: int, rank: int, world_size: int) -> tuple[int, int]:
    """Contiguous [start, stop) of n frames for `rank`; sizes differ by at most one."""
    if world_size <= 0 or not 0 <= rank < world_size:
        raise ValueError(f"rank {rank} / world {world_size}")
    base, rem = divmod(n, world_size)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def broadcast_tile(tile: torch.Tensor, src: int = 0) -> torch.Tensor:
    """Make every rank's `tile` equal to rank `src`'s (in place)."""
    _, ws = world()
    if ws > 1:
        if tile.is_cuda and dist.get_backend() == "gloo":  # gloo rehearsal: stage through the host
            host = tile.cpu()
            dist.broadcast(host, src=src)
            tile.copy_(host)
        else:
            dist.broadcast(tile, src=src)
    return tile


def max_over_ranks(x: float, device: torch.device | str = "cpu") -> float:
    _, ws = world()
    if ws == 1:
        return x
    if dist.get_backend() == "gloo":
        device = "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


@dataclass
class ShardedRoundTrip:
    """One step of the sharded path: tile broadcast, embed of the local frames,
    extract of the local frames against their covers.

    embed_fn(frames, tile, block, alpha, out) and extract_fn(wframes, oframes,
    block, alpha, out) are the per-rank kernels (thatsmyface_amd.batch on GPUs).
    """

    embed_fn: Callable
    extract_fn: Callable
    frames: torch.Tensor          # (n_local, H, W, 3) uint8
    tile: torch.Tensor            # (H/b, W/b) uint8, valid on rank 0
    block: int = 8
    alpha: float = 0.1
    out: torch.Tensor | None = None
    tiles: torch.Tensor | None = None
    hooks: list = field(default_factory=list)

    def __post_init__(self):
        n, h, w, _ = self.frames.shape
        if self.out is None:
            self.out = torch.empty_like(self.frames)
        if self.tiles is None:
            self.tiles = torch.empty((n, h // self.block, w // self.block), dtype=torch.uint8, device=self.frames.device)

    def step(self) -> None:
        broadcast_tile(self.tile, src=0)
        for h in self.hooks:
            h("broadcast")
        self.embed_fn(self.frames, self.tile, self.block, self.alpha, self.out)
        for h in self.hooks:
            h("embed")
        self.extract_fn(self.out, self.frames, self.block, self.alpha, self.tiles)
        for h in self.hooks:
            h("extract")
