"""Same module path as the reference's modules/constants.py (watermark constants only)."""
from ..constants import ALPHA, BLOCK_SIZE, MAX_SVD_COEFFICIENTS  # noqa: F401
