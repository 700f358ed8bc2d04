"""Watermark constants of the reference (modules/constants.py:7-9)."""

BLOCK_SIZE = 8  # constants.py:7
ALPHA = 0.1  # constants.py:8
MAX_SVD_COEFFICIENTS = 10  # constants.py:9 (unused by the reference too)

# every value of the app's block-size slider (embed_watermark_page.py:324-331: 4..16 step 2)
SUPPORTED_BLOCK_SIZES = (4, 6, 8, 10, 12, 14, 16)

# SVD route of the single-image drop-in calls (embed_watermark / extract_watermark; DESIGN.md
# 3.5): "reference" = np.linalg.svd's own arithmetic (the dgesdd route) for every block, the
# reference's bytes by construction; "hybrid" = the batch path's Jacobi route, with the dgesdd
# route for flagged blocks and for blocks whose bytes the byte certificate cannot decide.
# Per call: custom_settings["svd_route"]; per process: the TMFWM_SVD_ROUTE environment variable.
SVD_ROUTE = "reference"
