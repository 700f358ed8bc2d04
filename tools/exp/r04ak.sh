# round-4 study: extract<4>'s power vector from (D^T D / tr)^4 (four power steps per product; the
# Kato-Temple certificate unchanged).  sqN: ceil(ITERS / 4) + N products (strip pass 1 + N, list
# pass 2 + N); head = HEAD.  Outputs must hash equal; the question is the list-pass share.
# Variant source: tools/exp/r04ak_sq.patch on tmfwm_device.h, built with -DSQEXTRA=N (SRC_DIR).
set -euo pipefail
TAG=${TAG:-r04ak}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u tools/ab_variants.py --block 4 --frames 64 --rounds 3 head sq0 sq1 sq2 > $O/ab_sq_b4.log 2>&1
timeout -k 10 300 python -u tools/ab_variants.py --block 4 --frames 64 --rounds 2 --cover photo head sq0 sq1 sq2 > $O/ab_sq_b4_photo.log 2>&1
echo done
