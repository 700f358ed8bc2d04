# round-4: the dgesdd route's embed pass with the compact workspace above b = 8 (fxc: no work
# slot, D / M / S inside A, U, e; six waves per CU at b = 16) against the current build (fxcur)
set -euo pipefail
TAG=${TAG:-r04n}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u tools/exp/ref_route_time.py --block 16 --frames 16 --rounds 2 fxcur fxc > $O/ref_route_b16.log 2>&1
timeout -k 10 300 python -u tools/exp/ref_route_time.py --block 12 --frames 16 --rounds 2 fxcur fxc > $O/ref_route_b12.log 2>&1
timeout -k 10 300 python -u tools/exp/ref_route_time.py --block 8 --frames 16 --rounds 1 fxcur fxc > $O/ref_route_b8.log 2>&1
echo done
