# round-4: extract<16> -- the original image's rows loaded before the first power iteration
# (x16pf, 146 VGPRs, 3 waves / SIMD) or both images interleaved as at b <= 12 (x16il, 190, 2)
set -euo pipefail
TAG=${TAG:-r04g}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u tools/ab_variants.py --block 16 --frames 256 --rounds 3 base x16pf x16il > $O/ab_x16_b16.log 2>&1
timeout -k 10 300 python -u tools/ab_variants.py --block 14 --frames 256 --rounds 2 base x16pf x16il > $O/ab_x16_b14.log 2>&1
echo done
