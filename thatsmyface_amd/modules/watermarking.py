"""Same module path as the reference's modules/watermarking.py."""
from ..constants import ALPHA, BLOCK_SIZE  # noqa: F401
from ..watermarking import (  # noqa: F401
    apply_dct_to_block,
    apply_idct_to_block,
    embed_watermark,
    extract_watermark,
    get_watermark_settings,
    resize_watermark,
    rgb_to_ycbcr,
    ycbcr_to_rgb,
)
