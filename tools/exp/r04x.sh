# round-4: wave-aggregated list appends (la: one atomicAdd per wave) against per-lane appends
# (lacur) -- extract<4>'s 15.8 K list-pass blocks per frame, embed<8>'s list pass, b = 16
set -euo pipefail
TAG=${TAG:-r04x}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u tools/ab_variants.py --block 4 --frames 64 --rounds 3 lacur la > $O/ab_la_b4.log 2>&1
timeout -k 10 300 python -u tools/ab_variants.py --block 8 --frames 256 --rounds 3 lacur la > $O/ab_la_b8.log 2>&1
timeout -k 10 300 python -u tools/ab_variants.py --block 8 --frames 128 --rounds 2 --cover photo lacur la > $O/ab_la_b8_photo.log 2>&1
timeout -k 10 300 python -u tools/ab_variants.py --block 16 --frames 128 --rounds 2 lacur la > $O/ab_la_b16.log 2>&1
echo done
