"""thatsmyface_amd -- MI355X (gfx950) implementation of ThatsMyFace's block-wise
DCT+SVD watermark path (reference: modules/watermarking.py).

* ``thatsmyface_amd.watermarking`` -- drop-in for the reference module (same
  functions and signatures, PIL in / PIL out).
* ``thatsmyface_amd.batch`` -- device-resident batches (torch tensors in HBM).
* ``thatsmyface_amd.dist`` -- one process per GPU, frame sharding + RCCL
  broadcast of the watermark tile.

The arithmetic lives in ``libtmfwm.so`` (HIP kernels, C ABI in include/tmfwm.h).
"""
from .constants import ALPHA, BLOCK_SIZE, SUPPORTED_BLOCK_SIZES  # noqa: F401

__version__ = "0.1.0"
