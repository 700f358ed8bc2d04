# round-4 study: embed<8> / extract<8> with 4 lanes per 8 x 8 block (2 rows per lane) instead of
# 2 (4 rows): l4 (register allocation unconstrained, 2 waves / SIMD) and l4w3 (launch bounds for
# 3 waves / SIMD, 160 VGPRs, no spill) against the shipped layout (l2base).  The lane count is part
# of the hybrid route's contract (the order of its dot products), so the hashes differ by design.
set -euo pipefail
TAG=${TAG:-r04r}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u tools/ab_variants.py --block 8 --frames 256 --rounds 3 l2base l4 l4w3 > $O/ab_l4_b8_noise.log 2>&1
timeout -k 10 300 python -u tools/ab_variants.py --block 8 --frames 128 --rounds 2 --cover photo l2base l4 l4w3 > $O/ab_l4_b8_photo.log 2>&1
echo done
