"""Watermark constants of the reference (modules/constants.py:7-9)."""

BLOCK_SIZE = 8  # constants.py:7
ALPHA = 0.1  # constants.py:8
MAX_SVD_COEFFICIENTS = 10  # constants.py:9 (unused by the reference too)

# every value of the app's block-size slider (embed_watermark_page.py:324-331: 4..16 step 2)
SUPPORTED_BLOCK_SIZES = (4, 6, 8, 10, 12, 14, 16)
