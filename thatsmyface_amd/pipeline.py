"""Batched app pipeline for the embed page.

The reference page embeds uploaded images one at a time
(internal_pages/embed_watermark_page.py:492-558): PIL decode, ``embed_watermark``,
PNG encode into session state, then ``time.sleep(0.1)``.  Once the watermark
arithmetic runs on the GPU, the per-image decode / encode on one host thread is
what is left.  This module overlaps the three stages:

* decode (thread pool): ``Image.open(...).convert("RGB")`` -> uint8 array;
* device (one ordered stage): pinned host buffer -> async H2D on a side stream ->
  ``embed_batch`` (one launch) -> async D2H into pinned memory; the watermark tile
  for each image size is prepared once on the device (``tmfwm_prepare_tile``);
* encode (thread pool): waits for the copy, PNG-encodes (zlib releases the GIL).

Results come back in input order and are byte-identical to
``embed_watermark(img, watermark_data, preserve_ratio)`` followed by
``img.save(format="PNG")`` per image.  The device stage is a parameter so the
pipeline logic is testable on CPU (tests/test_pipeline.py).
"""
from __future__ import annotations

import io
import os
from concurrent.futures import Future, ThreadPoolExecutor
from dataclasses import dataclass
from typing import Callable, Iterable, Sequence

import numpy as np
from PIL import Image

from .constants import ALPHA, BLOCK_SIZE, SVD_ROUTE


@dataclass
class Embedded:
    """One pipeline result: the watermarked RGB pixels and their PNG encoding."""

    pixels: np.ndarray
    png: bytes

    def image(self) -> Image.Image:
        return Image.fromarray(self.pixels, "RGB")


def _decode(src) -> np.ndarray:
    img = src if isinstance(src, Image.Image) else Image.open(io.BytesIO(src) if isinstance(src, (bytes, bytearray)) else src)
    return np.ascontiguousarray(np.asarray(img.convert("RGB"), dtype=np.uint8))


def _encode(pixels: np.ndarray, wait: Callable[[], None] | None) -> Embedded:
    if wait is not None:
        wait()
    buf = io.BytesIO()
    Image.fromarray(pixels, "RGB").save(buf, format="PNG")  # embed_watermark_page.py:533-535
    return Embedded(pixels, buf.getvalue())


class GpuStage:
    """Device stage: per image, pinned staging + side-stream H2D / embed / D2H.

    Returns (pixels, wait) where ``wait()`` blocks until the D2H copy landed.  The
    tile for an image size is prepared on the device once and reused."""

    def __init__(self, watermark_data, block: int, alpha: float, preserve_ratio: bool, device=None, route: str = SVD_ROUTE):
        import torch

        from . import batch

        self.torch, self.batch = torch, batch
        self.block, self.alpha, self.preserve_ratio = int(block), float(alpha), bool(preserve_ratio)
        self.route = route  # the drop-in's SVD route (constants.SVD_ROUTE, custom_settings["svd_route"])
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        wm = watermark_data if isinstance(watermark_data, Image.Image) else Image.open(io.BytesIO(watermark_data))
        grey = np.array(wm.convert("L"), dtype=np.uint8, copy=True)  # watermarking.py:98-103
        self.wm_grey = torch.from_numpy(grey).to(self.device)
        self.stream = torch.cuda.Stream(device=self.device)
        self.tiles: dict[tuple[int, int], object] = {}

    def _tile(self, nbh: int, nbw: int):
        key = (nbh, nbw)
        if key not in self.tiles:
            with self.torch.cuda.stream(self.stream):
                self.tiles[key] = self.batch.prepare_tile(self.wm_grey, nbh, nbw, self.preserve_ratio, stream=self.stream)
        return self.tiles[key]

    def __call__(self, rgb: np.ndarray):
        torch = self.torch
        h, w = rgb.shape[:2]
        nbh, nbw = h // self.block, w // self.block
        if nbh == 0 or nbw == 0:
            raise ValueError("height and width must be > 0")  # PIL's resize raises in the reference
        host_in = torch.empty((1, h, w, 3), dtype=torch.uint8, pin_memory=True)
        host_in.numpy()[0] = rgb
        host_out = torch.empty((1, h, w, 3), dtype=torch.uint8, pin_memory=True)
        tile = self._tile(nbh, nbw)
        with torch.cuda.stream(self.stream):
            dev_in = host_in.to(self.device, non_blocking=True)
            dev_out = self.batch.embed_batch(dev_in, tile, self.block, self.alpha, stream=self.stream, route=self.route)
            host_out.copy_(dev_out, non_blocking=True)
            done = torch.cuda.Event()
            done.record(self.stream)
        # keep the device buffers alive until the copy has landed
        keep = (dev_in, dev_out, host_in)

        def wait(_e=done, _k=keep):
            _e.synchronize()

        return host_out.numpy()[0], wait


def embed_images(images: Iterable, watermark_data, preserve_ratio: bool = True, custom_settings: dict | None = None,
                 workers: int | None = None, device_stage: Callable | None = None) -> list[Embedded]:
    """Embed ``watermark_data`` (PNG bytes or PIL image) into every image (bytes, file
    object or PIL image) -- embed_watermark_page.py:492-558 without the per-image
    serialisation.  Returns, in input order, the watermarked pixels and PNG bytes."""
    settings = custom_settings or {}
    block = int(settings.get("block_size", BLOCK_SIZE))
    alpha = float(settings.get("alpha", ALPHA))
    route = settings.get("svd_route") or os.environ.get("TMFWM_SVD_ROUTE") or SVD_ROUTE  # as watermarking._route
    stage = device_stage or GpuStage(watermark_data, block, alpha, preserve_ratio, route=route)
    n_workers = workers or min(16, max(2, (len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else 4)))
    sources: Sequence = list(images)
    with ThreadPoolExecutor(n_workers, thread_name_prefix="tmf-io") as pool:
        decoded: list[Future] = [pool.submit(_decode, s) for s in sources]
        encoded: list[Future] = []
        for fut in decoded:  # the device stage runs in order on this thread
            pixels, wait = stage(fut.result())
            encoded.append(pool.submit(_encode, pixels, wait))
        return [f.result() for f in encoded]
