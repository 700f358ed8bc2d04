# round-4: the compact workspace of the dgesdd route's embed pass at b = 6 / 8 too (fxc8) against
# the current build (fxcur, compact above b = 8 only)
set -euo pipefail
TAG=${TAG:-r04o}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u tools/exp/ref_route_time.py --block 8 --frames 16 --rounds 3 fxcur fxc8 > $O/ref_route_b8.log 2>&1
timeout -k 10 300 python -u tools/exp/ref_route_time.py --block 6 --frames 16 --rounds 2 fxcur fxc8 > $O/ref_route_b6.log 2>&1
echo done
