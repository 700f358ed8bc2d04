"""ctypes binding of libtmfwm.so (C ABI declared in include/tmfwm.h).

The library is built in-tree (``thatsmyface_amd/libtmfwm.so``, see
``thatsmyface_amd/csrc/Makefile`` / ``__graft_entry__.build()``).  There is no
CPU fallback: if the library or a GPU is missing every call raises.
"""
from __future__ import annotations

import ctypes
import importlib.util
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# TMFWM_LIB selects an alternative build (e.g. the phase-profile libtmfwm_stamps.so)
LIB_PATH = os.environ.get("TMFWM_LIB") or os.path.join(_HERE, "libtmfwm.so")
ABI_VERSION = 10

MEM_HOST = 0
MEM_DEVICE = 1

ERR_INVALID = -22
ERR_NOMEM = -12
ERR_HIP = -5
ERR_UNSUPPORTED = -95
ERR_NODEVICE = -19
ERR_NODATA = -61

ROUTE_HYBRID = 0  # TMFWM_ROUTE_*: the SVD route of embed / extract (include/tmfwm.h)
ROUTE_REFERENCE = 1
ROUTE_RANK1 = 2  # ABI 10: the hybrid route behind the rank-1 pre-pass (embed at b = 8, 16; photo mode)
ROUTE_RANK1_REFERENCE = 3  # ABI 10: the rank-1 pre-pass in front of the dgesdd route (no Jacobi, no K)
ROUTES = {"hybrid": ROUTE_HYBRID, "reference": ROUTE_REFERENCE, "rank1": ROUTE_RANK1, "rank1_reference": ROUTE_RANK1_REFERENCE}

# pixel layouts of tmfwm_embed_px / tmfwm_extract_px (include/tmfwm.h, ABI 8)
PIX_RGB = 3
PIX_RGBX = 4  # PIL's in-memory mode "RGB" (R, G, B, pad)


def route_code(route) -> int:
    """"hybrid" / "reference" / "rank1" / "rank1_reference" (or the TMFWM_ROUTE_* value) -> the ABI's route value."""
    if isinstance(route, str):
        if route not in ROUTES:
            raise ValueError(f"route must be one of {sorted(ROUTES)}, got {route!r}")
        return ROUTES[route]
    if route not in (ROUTE_HYBRID, ROUTE_REFERENCE, ROUTE_RANK1, ROUTE_RANK1_REFERENCE):
        raise ValueError(f"route {route!r}")
    return int(route)


DT_F16 = 1
DT_F32 = 2
DT_F64 = 3

_u8p = ctypes.c_void_p
_I64 = ctypes.c_int64
_I32 = ctypes.c_int32
_D = ctypes.c_double
_VP = ctypes.c_void_p

# name -> (restype, argtypes): exactly the entry points of include/tmfwm.h
SIGNATURES = {
    "tmfwm_abi_version": (ctypes.c_int, []),
    "tmfwm_last_error": (ctypes.c_char_p, []),
    "tmfwm_device_count": (ctypes.c_int, []),
    "tmfwm_embed": (ctypes.c_int, [_VP, _I64, _I32, _I32, _I64, _VP, _I32, _D, _VP, _I32, _VP]),
    "tmfwm_extract": (ctypes.c_int, [_VP, _VP, _I64, _I32, _I32, _I64, _I32, _D, _VP, _I32, _VP]),
    "tmfwm_last_list_pass_blocks": (ctypes.c_int64, []),
    "tmfwm_embed_list_pass": (ctypes.c_int, [ctypes.c_int32]),
    "tmfwm_embed_ex": (ctypes.c_int, [_VP, _I64, _I32, _I32, _I64, _VP, _I32, _D, _VP, _I32, _VP, _VP]),
    "tmfwm_extract_ex": (ctypes.c_int, [_VP, _VP, _I64, _I32, _I32, _I64, _I32, _D, _VP, _I32, _VP, _VP]),
    "tmfwm_embed_route": (ctypes.c_int, [_VP, _I64, _I32, _I32, _I64, _VP, _I32, _D, _VP, _I32, _VP, _I32, _VP]),
    "tmfwm_extract_route": (ctypes.c_int, [_VP, _VP, _I64, _I32, _I32, _I64, _I32, _D, _VP, _I32, _VP, _I32, _VP]),
    "tmfwm_embed_px": (ctypes.c_int, [_VP, _I32, _I64, _I64, _I32, _I32, _VP, _I32, _D, _VP, _I32, _I64, _I32, _VP, _I32, _VP]),
    "tmfwm_extract_px": (ctypes.c_int, [_VP, _I32, _I64, _VP, _I32, _I64, _I64, _I32, _I32, _I32, _D, _VP, _I32, _VP, _I32, _VP]),
    "tmfwm_embed_multi": (ctypes.c_int, [_VP, _I64, _I32, _I32, _I64, _VP, _I32, _D, _VP, _VP, _I32, _VP]),
    "tmfwm_release_cached_buffers": (ctypes.c_int, []),
    "tmfwm_extract_multi": (ctypes.c_int, [_VP, _VP, _I64, _I32, _I32, _I64, _I32, _D, _VP, _VP, _I32, _VP]),
    "tmfwm_embed_multi_route": (ctypes.c_int, [_VP, _I64, _I32, _I32, _I64, _VP, _I32, _D, _VP, _VP, _I32, _I32, _VP]),
    "tmfwm_extract_multi_route": (ctypes.c_int, [_VP, _VP, _I64, _I32, _I32, _I64, _I32, _D, _VP, _VP, _I32, _I32, _VP]),
    "tmfwm_rgb_to_ycbcr": (ctypes.c_int, [_VP, _I64, _VP, _I32, _VP]),
    "tmfwm_ycbcr_to_rgb": (ctypes.c_int, [_VP, _I64, _VP, _I32, _VP]),
    "tmfwm_rgb_to_ycbcr_f32": (ctypes.c_int, [_VP, _I64, _VP, _I32, _VP]),
    "tmfwm_ycbcr_to_rgb_typed": (ctypes.c_int, [_VP, _I32, _I64, _VP, _I32, _VP]),
    "tmfwm_dct2d_blocks": (ctypes.c_int, [_VP, _I64, _I32, _I32, _I32, _VP]),
    "tmfwm_svd_blocks": (ctypes.c_int, [_VP, _I64, _I32, _VP, _VP, _VP, _VP, _I32, _VP]),
    "tmfwm_lapack_svd_blocks": (ctypes.c_int, [_VP, _I64, _I32, _VP, _VP, _VP, _I32, _I32, _VP]),
    "tmfwm_lapack_nrm2": (ctypes.c_int, [_VP, _I64, _I32, _I32, _VP, _I32, _VP]),
    "tmfwm_synth_frames": (ctypes.c_int, [ctypes.c_uint64, _I64, _I64, _I64, _VP, _VP]),
    "tmfwm_prepare_tile": (ctypes.c_int, [_VP, _I32, _I32, _I32, _I32, _I32, _VP, _I32, _VP]),
    "tmfwm_qr_encode": (ctypes.c_int, [_VP, _I32, _I32, _I32, _I32, _VP, _I32, _VP]),
    "tmfwm_qr_decode": (ctypes.c_int, [_VP, _I32, _I32, _I64, _VP, _I32, _VP]),
    "tmfwm_qr_decode_batch": (ctypes.c_int, [_VP, _I64, _I32, _I32, _VP, _I32, _VP]),
    "tmfwm_aes_cbc_encrypt": (ctypes.c_int, [_VP, _I32, _VP, _VP, _I64, _VP]),
    "tmfwm_aes_cbc_decrypt": (ctypes.c_int, [_VP, _I32, _VP, _VP, _I64, _VP]),
}

_lock = threading.Lock()
_lib = None


class TmfwmError(RuntimeError):
    """A HIP-side failure reported by libtmfwm.so."""


def _share_hip_runtime() -> None:
    """One HIP runtime per process.  PyTorch-ROCm bundles its own libamdhip64.so.7;
    libtmfwm.so needs the same soname.  Whichever copy is loaded first is the one
    every later user binds to, and torch does not work on a runtime other than its
    own, so when torch is installed its copy is loaded (RTLD_GLOBAL) before this
    library -- torch and libtmfwm then share one runtime in either import order.
    Without torch the system ROCm runtime (/opt/rocm/lib) is used."""
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.submodule_search_locations:
        return
    path = os.path.join(list(spec.submodule_search_locations)[0], "lib", "libamdhip64.so")
    if os.path.exists(path):
        ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)


def load():
    """Load and type the library once; raises ImportError if it was not built."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise ImportError(
                    f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                    "or `make -C thatsmyface_amd/csrc` (hipcc, gfx950)"
                )
            _share_hip_runtime()
            L = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            v = L.tmfwm_abi_version()
            if v != ABI_VERSION:
                raise ImportError(f"libtmfwm ABI {v} != expected {ABI_VERSION}")
            _lib = L
    return _lib


def last_error() -> str:
    msg = load().tmfwm_last_error()
    return msg.decode(errors="replace") if msg else ""


def check(rc: int, what: str) -> None:
    if rc == 0:
        return
    msg = f"{what}: {last_error()} (status {rc})"
    if rc == ERR_INVALID:
        raise ValueError(msg)
    if rc == ERR_UNSUPPORTED:
        raise NotImplementedError(msg)
    raise TmfwmError(msg)


def device_count() -> int:
    return int(load().tmfwm_device_count())
