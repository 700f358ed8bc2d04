# round-4: list-pass waves per segment (lpN: N waves share each of the 2048 segments, grid 2048 N;
# lp1 = HEAD's layout through the new indexing) -- extract<4>'s 3 % list pass, embed<8>'s list pass
set -euo pipefail
TAG=${TAG:-r04ai}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u tools/ab_variants.py --block 4 --frames 64 --rounds 3 head lp1 lp4 lp8 > $O/ab_lp_b4.log 2>&1
timeout -k 10 300 python -u tools/ab_variants.py --block 8 --frames 128 --rounds 2 head lp1 lp4 lp8 > $O/ab_lp_b8.log 2>&1
timeout -k 10 300 python -u tools/ab_variants.py --block 8 --frames 64 --rounds 2 --cover photo head lp1 lp4 lp8 > $O/ab_lp_b8_photo.log 2>&1
echo done
