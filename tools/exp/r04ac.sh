# round-4: is extract<4>'s wait the strip pass's list appends?  noat replaces the append
# (atomicAdd on one counter + id store) by a byte store -- wrong output, timing only; shard
# appends to 2048 segments with a counter each (same outputs as cur, HEAD's kernels).
set -euo pipefail
TAG=${TAG:-r04ac}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u tools/ab_variants.py --block 4 --frames 64 --rounds 3 cur noat shard shard2 > $O/ab_b4.log 2>&1
timeout -k 10 300 python -u tools/ab_variants.py --block 8 --frames 128 --rounds 2 cur shard shard2 > $O/ab_b8.log 2>&1
timeout -k 10 300 python -u tools/ab_variants.py --block 8 --frames 64 --rounds 2 --cover photo cur shard shard2 > $O/ab_b8_photo.log 2>&1
timeout -k 10 300 python -u tools/ab_variants.py --block 6 --frames 64 --rounds 2 cur shard shard2 > $O/ab_b6.log 2>&1
timeout -k 10 300 python -u tools/ab_variants.py --block 16 --frames 64 --rounds 2 cur shard shard2 > $O/ab_b16.log 2>&1
echo done
