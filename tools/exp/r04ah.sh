# round-4: extract<b <= 8> at 4 waves per SIMD (128 VGPRs) instead of 3 (139 at b = 8); head = HEAD
set -euo pipefail
TAG=${TAG:-r04ah}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u tools/ab_variants.py --block 8 --frames 128 --rounds 3 head xw4 > $O/ab_xw4_b8.log 2>&1
timeout -k 10 300 python -u tools/ab_variants.py --block 8 --frames 64 --rounds 2 --cover photo head xw4 > $O/ab_xw4_b8_photo.log 2>&1
timeout -k 10 300 python -u tools/ab_variants.py --block 6 --frames 64 --rounds 2 head xw4 > $O/ab_xw4_b6.log 2>&1
echo done
