"""Multi-GPU batch API over host memory, without torch.distributed.

One process drives several MI355X devices through the C ABI's tmfwm_embed_multi /
tmfwm_extract_multi (include/tmfwm.h): contiguous frame shards (dist.shard_range's
split), one host thread + HIP stream per shard, the watermark tile broadcast with RCCL.
This is the path for a non-torch caller (a C/C++ service, or Python that only has numpy
frames, e.g. the app's per-image loop embed_watermark_page.py:492-558 batched); the
torchrun path (one process per GPU) is thatsmyface_amd.dist / bench.py.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .constants import SUPPORTED_BLOCK_SIZES


def _frames(a: np.ndarray, name: str) -> np.ndarray:
    if a.dtype != np.uint8 or a.ndim != 4 or a.shape[-1] != 3:
        raise ValueError(f"{name} must be (N, H, W, 3) uint8, got {a.shape} {a.dtype}")
    return np.ascontiguousarray(a)


def _device_list(devices):
    if devices is None:
        return None, 0
    devs = (ctypes.c_int32 * len(devices))(*[int(d) for d in devices])
    return devs, len(devices)


def embed_multi(frames: np.ndarray, wm_tile: np.ndarray, block: int = 8, alpha: float = 0.1, devices=None,
                stats: dict | None = None, route: str = "hybrid") -> np.ndarray:
    """Embed one tile into every frame, frames sharded over `devices` (default: every
    visible GPU; repeat a device for logical shards).  stats receives "lapack_blocks";
    route as batch.embed_batch ("hybrid", "reference", "rank1" or "rank1_reference")."""
    frames = _frames(frames, "frames")
    n, h, w, _ = frames.shape
    if block not in SUPPORTED_BLOCK_SIZES:
        raise NotImplementedError(f"block {block}")
    tile = np.ascontiguousarray(wm_tile, dtype=np.uint8)
    if tile.shape != (h // block, w // block):
        raise ValueError(f"wm_tile must be ({h // block}, {w // block}), got {tile.shape}")
    out = np.empty_like(frames)
    devs, k = _device_list(devices)
    cnt = ctypes.c_int64(0)
    L = _lib.load()
    _lib.check(L.tmfwm_embed_multi_route(frames.ctypes.data, n, h, w, h * w * 3, tile.ctypes.data, block, float(alpha),
                                         out.ctypes.data, devs, k, _lib.route_code(route), ctypes.addressof(cnt)), "embed_multi")
    if stats is not None:
        stats["lapack_blocks"] = int(cnt.value)
    return out


def extract_multi(wframes: np.ndarray, oframes: np.ndarray, block: int = 8, alpha: float = 0.1, devices=None,
                  stats: dict | None = None, route: str = "hybrid") -> np.ndarray:
    """Extract every frame pair's tile, pairs sharded over `devices`."""
    wframes = _frames(wframes, "wframes")
    oframes = _frames(oframes, "oframes")
    if wframes.shape != oframes.shape:
        raise ValueError("watermarked / original batch shapes differ")
    n, h, w, _ = wframes.shape
    if block not in SUPPORTED_BLOCK_SIZES:
        raise NotImplementedError(f"block {block}")
    out = np.empty((n, h // block, w // block), np.uint8)
    devs, k = _device_list(devices)
    cnt = ctypes.c_int64(0)
    L = _lib.load()
    _lib.check(L.tmfwm_extract_multi_route(wframes.ctypes.data, oframes.ctypes.data, n, h, w, h * w * 3, block, float(alpha),
                                           out.ctypes.data, devs, k, _lib.route_code(route), ctypes.addressof(cnt)),
               "extract_multi")
    if stats is not None:
        stats["lapack_blocks"] = int(cnt.value)
    return out


def release_cached_buffers() -> int:
    """Frees the device staging buffers the multi-GPU calls keep between calls (tmfwm_release_cached_buffers)."""
    return int(_lib.load().tmfwm_release_cached_buffers())
