# round-4 diagnosis: extract<4>'s strip pass without its per-lane byte stores of the tile
# (nostore: timing only, its tiles are not written) against the current build (nscur)
set -euo pipefail
TAG=${TAG:-r04aa}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u tools/ab_variants.py --block 4 --frames 64 --rounds 2 nscur nostore > $O/ab_nostore_b4.log 2>&1
timeout -k 10 300 python -u tools/ab_variants.py --block 8 --frames 128 --rounds 2 nscur nostore > $O/ab_nostore_b8.log 2>&1
echo done
