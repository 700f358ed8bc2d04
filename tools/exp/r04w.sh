# round-4: extract<4> -- both images' rows up front (x4cur) against one image at a time (x4seq)
set -euo pipefail
TAG=${TAG:-r04w}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u tools/ab_variants.py --block 4 --frames 64 --rounds 3 x4cur x4seq > $O/ab_x4_b4.log 2>&1
echo done
