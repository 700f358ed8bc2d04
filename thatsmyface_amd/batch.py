"""Device-resident batch API: frames already in HBM (torch tensors on a ROCm GPU).

This is the path the benchmark and multi-GPU driver use: a batch of N frames
(N, H, W, 3) uint8 on ``cuda:k`` is embedded / extracted by ONE kernel launch
each, enqueued on the caller's current torch stream.  torch provides device
memory and streams only; the arithmetic is libtmfwm.so's HIP kernels.
"""
from __future__ import annotations

import torch

from . import _lib
from .constants import SUPPORTED_BLOCK_SIZES

SEED_COVER = 0x5EED0001
SEED_WATERMARK = 0x5EED0002


def _stream(stream) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def _check_frames(t: torch.Tensor, name: str) -> None:
    if not t.is_cuda:
        raise ValueError(f"{name} must be a GPU tensor")
    if t.dtype != torch.uint8 or t.dim() != 4 or t.shape[-1] != 3:
        raise ValueError(f"{name} must be (N, H, W, 3) uint8, got {tuple(t.shape)} {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


def _count_ptr(stats):
    import ctypes

    if stats is None:
        return None, None
    c = ctypes.c_int64(0)
    return c, ctypes.addressof(c)


def embed_list_pass(block: int) -> bool:
    """Whether embed at this block size runs a list pass after its strip pass."""
    return bool(_lib.load().tmfwm_embed_list_pass(int(block)))


def embed_batch(frames: torch.Tensor, wm_tile: torch.Tensor, block: int = 8, alpha: float = 0.1,
                out: torch.Tensor | None = None, stream=None, stats: dict | None = None,
                route: str = "hybrid") -> torch.Tensor:
    """Embed one watermark tile into every frame (watermarking.py:135 per frame).
    stats (optional dict) receives "lapack_blocks": the blocks redone on the dgesdd route;
    asking for it synchronises the stream.  route: "hybrid" (Jacobi + the dgesdd route for
    the flagged blocks, the throughput route) or "reference" (the dgesdd route for every
    block: np.linalg.svd's arithmetic by construction)."""
    _check_frames(frames, "frames")
    n, h, w, _ = frames.shape
    if block not in SUPPORTED_BLOCK_SIZES:
        raise NotImplementedError(f"block {block}")
    if tuple(wm_tile.shape) != (h // block, w // block) or wm_tile.dtype != torch.uint8 or not wm_tile.is_cuda:
        raise ValueError(f"wm_tile must be ({h // block}, {w // block}) uint8 on the GPU, got {tuple(wm_tile.shape)}")
    wm_tile = wm_tile.contiguous()
    if out is None:
        out = torch.empty_like(frames)
    else:
        _check_frames(out, "out")
        if out.shape != frames.shape:
            raise ValueError("out shape mismatch")
    cnt, ptr = _count_ptr(stats)
    with torch.cuda.device(frames.device):
        L = _lib.load()
        _lib.check(L.tmfwm_embed_route(frames.data_ptr(), n, h, w, h * w * 3, wm_tile.data_ptr(), block, float(alpha),
                                       out.data_ptr(), _lib.MEM_DEVICE, _stream(stream), _lib.route_code(route), ptr),
                   "embed_batch")
    if stats is not None:
        stats["lapack_blocks"] = int(cnt.value)
        stats["list_pass_blocks"] = int(L.tmfwm_last_list_pass_blocks())
    return out


def extract_batch(wframes: torch.Tensor, oframes: torch.Tensor, block: int = 8, alpha: float = 0.1,
                  out: torch.Tensor | None = None, stream=None, stats: dict | None = None,
                  route: str = "hybrid") -> torch.Tensor:
    """Extract the watermark tile of every frame pair (watermarking.py:224 per pair).
    stats (optional dict) receives "lapack_blocks" (synchronises the stream); route as
    embed_batch's."""
    _check_frames(wframes, "wframes")
    _check_frames(oframes, "oframes")
    if wframes.shape != oframes.shape:
        raise ValueError("watermarked / original batch shapes differ")
    n, h, w, _ = wframes.shape
    if block not in SUPPORTED_BLOCK_SIZES:
        raise NotImplementedError(f"block {block}")
    if out is None:
        out = torch.empty((n, h // block, w // block), dtype=torch.uint8, device=wframes.device)
    cnt, ptr = _count_ptr(stats)
    with torch.cuda.device(wframes.device):
        L = _lib.load()
        _lib.check(L.tmfwm_extract_route(wframes.data_ptr(), oframes.data_ptr(), n, h, w, h * w * 3, block, float(alpha),
                                         out.data_ptr(), _lib.MEM_DEVICE, _stream(stream), _lib.route_code(route), ptr),
                   "extract_batch")
    if stats is not None:
        stats["lapack_blocks"] = int(cnt.value)
        stats["list_pass_blocks"] = int(L.tmfwm_last_list_pass_blocks())
    return out


def synth_frames(n: int, height: int, width: int, seed: int = SEED_COVER, frame0: int = 0,
                 device: torch.device | str | None = None, out: torch.Tensor | None = None) -> torch.Tensor:
    """Counter-based synthetic uint8 frames generated directly in HBM."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    if out is None:
        out = torch.empty((n, height, width, 3), dtype=torch.uint8, device=dev)
    with torch.cuda.device(out.device):
        L = _lib.load()
        _lib.check(L.tmfwm_synth_frames(seed, frame0, n, height * width * 3, out.data_ptr(), _stream(None)), "synth_frames")
    return out


def synth_photo_frames(n: int, height: int, width: int, seed: int = SEED_COVER, frame0: int = 0,
                       device: torch.device | str | None = None, chunk: int = 16) -> torch.Tensor:
    """Camera-like synthetic uint8 frames (tests/lapack_path.photo_cover's recipe on the device:
    a low-pass field + gradients + fine grain, the decaying DCT spectra of natural images),
    generated `chunk` frames at a time with one generator seed per frame (seed + frame index)."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    out = torch.empty((n, height, width, 3), dtype=torch.uint8, device=dev)
    y = torch.linspace(0, 1, height, device=dev).view(1, height, 1, 1)
    x = torch.linspace(0, 1, width, device=dev).view(1, 1, width, 1)
    for c0 in range(0, n, chunk):
        k = min(chunk, n - c0)
        f = torch.empty((k, height // 16 + 2, width // 16 + 2, 3), device=dev)
        g = torch.Generator(device=dev)
        for i in range(k):
            g.manual_seed(seed + frame0 + c0 + i)
            f[i] = torch.randn(f.shape[1:], generator=g, device=dev)
        f = f.repeat_interleave(16, 1).repeat_interleave(16, 2)[:, :height, :width]
        for ax in (1, 2):
            for _ in range(2):
                f = (torch.roll(f, 5, ax) + torch.roll(f, -5, ax) + f) / 3.0
        img = 128 + 45 * f + 60 * (x - 0.5) + 30 * (y - 0.5)
        g.manual_seed(seed + frame0 + c0 + 0x9E3779B9)
        img += 2.0 * torch.randn(img.shape, generator=g, device=dev)
        out[c0:c0 + k] = img.clamp_(0, 255).to(torch.uint8)
    return out


def synth_qr_tile(nbh: int, nbw: int, seed: int = SEED_WATERMARK, device=None) -> torch.Tensor:
    """The app's watermark tile: a QR code of a 48-byte payload (an AES-CBC ciphertext's size:
    IV + two blocks, base64 in the symbol, level H) rendered by text_to_qrcode (300 x 300) and
    resized to the block grid by resize_watermark with preserve_ratio=True, as the embed page does
    (embed_watermark_page.py:492-531; modules/qrcode_generator.py:10-44): 0 / 255 modules with
    LANCZOS edges, centred on a white canvas."""
    import numpy as np  # noqa: PLC0415

    from . import qrcode_generator, watermarking  # noqa: PLC0415

    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    payload = np.random.default_rng(seed).integers(0, 256, 48).astype(np.uint8).tobytes()
    img = qrcode_generator.text_to_qrcode(payload)
    with torch.cuda.device(dev):
        t = np.asarray(watermarking.resize_watermark(img, nbh, nbw, preserve_ratio=True), dtype=np.uint8)
    return torch.from_numpy(np.ascontiguousarray(t)).to(dev)


def synth_tile(nbh: int, nbw: int, seed: int = SEED_WATERMARK, device=None) -> torch.Tensor:
    """Synthetic watermark tile: the same generator over an nbh x nbw byte plane."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    out = torch.empty((nbh, nbw), dtype=torch.uint8, device=dev)
    with torch.cuda.device(dev):
        L = _lib.load()
        _lib.check(L.tmfwm_synth_frames(seed, 0, 1, nbh * nbw, out.data_ptr(), _stream(None)), "synth_tile")
    return out


def svd_blocks(D: torch.Tensor):
    """SVD stage alone on (n, b, b) float32 blocks: (U, S, Vt, sweeps) as the reference consumes them."""
    if not D.is_cuda or D.dtype != torch.float32 or D.dim() != 3 or D.shape[1] != D.shape[2]:
        raise ValueError("D must be (n, b, b) float32 on the GPU")
    D = D.contiguous()
    n, b, _ = D.shape
    U = torch.empty_like(D)
    Vt = torch.empty_like(D)
    S = torch.empty((n, b), dtype=torch.float32, device=D.device)
    sw = torch.empty((n,), dtype=torch.int32, device=D.device)
    with torch.cuda.device(D.device):
        L = _lib.load()
        _lib.check(L.tmfwm_svd_blocks(D.data_ptr(), n, b, U.data_ptr(), S.data_ptr(), Vt.data_ptr(), sw.data_ptr(),
                                      _lib.MEM_DEVICE, _stream(None)), "svd_blocks")
    return U, S, Vt, sw


def lapack_svd_blocks(D: torch.Tensor, want_vectors: bool = True):
    """np.linalg.svd on the dgesdd route (the reference's arithmetic) for (n, b, b) float32
    blocks on the GPU: (U, S, Vt), or (None, S, None) without vectors."""
    if not D.is_cuda or D.dtype != torch.float32 or D.dim() != 3 or D.shape[1] != D.shape[2]:
        raise ValueError("D must be (n, b, b) float32 on the GPU")
    D = D.contiguous()
    n, b, _ = D.shape
    S = torch.empty((n, b), dtype=torch.float32, device=D.device)
    U = torch.empty_like(D) if want_vectors else None
    Vt = torch.empty_like(D) if want_vectors else None
    with torch.cuda.device(D.device):
        L = _lib.load()
        _lib.check(L.tmfwm_lapack_svd_blocks(D.data_ptr(), n, b, U.data_ptr() if want_vectors else None, S.data_ptr(),
                                             Vt.data_ptr() if want_vectors else None, int(want_vectors), _lib.MEM_DEVICE,
                                             _stream(None)), "lapack_svd_blocks")
    return U, S, Vt


def prepare_tile(watermark_l: torch.Tensor, tile_height: int, tile_width: int, preserve_ratio: bool = False,
                 out: torch.Tensor | None = None, stream=None) -> torch.Tensor:
    """resize_watermark (watermarking.py:105-130) on a device-resident (h, w) uint8 grey
    watermark: Pillow-exact LANCZOS resample (+ centred paste on white when
    preserve_ratio).  Synchronises the stream (the resample tables come from the host)."""
    if not watermark_l.is_cuda or watermark_l.dtype != torch.uint8 or watermark_l.dim() != 2:
        raise ValueError("watermark_l must be a (h, w) uint8 GPU tensor")
    watermark_l = watermark_l.contiguous()
    if out is None:
        out = torch.empty((tile_height, tile_width), dtype=torch.uint8, device=watermark_l.device)
    elif tuple(out.shape) != (tile_height, tile_width) or out.dtype != torch.uint8 or not out.is_contiguous():
        raise ValueError("out must be a contiguous (tile_height, tile_width) uint8 tensor")
    with torch.cuda.device(watermark_l.device):
        L = _lib.load()
        _lib.check(L.tmfwm_prepare_tile(watermark_l.data_ptr(), watermark_l.shape[0], watermark_l.shape[1], tile_height,
                                        tile_width, int(bool(preserve_ratio)), out.data_ptr(), _lib.MEM_DEVICE, _stream(stream)),
                   "prepare_tile")
    return out
