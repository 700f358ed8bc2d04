# round-4: the dgesdd route's passes -- extract without U / VT in its LDS workspace (fxs: 3 waves /
# SIMD at b = 8; fxs4: launch bounds for 4), dbdsqr's d / e replicated on the 8 lanes of a group
# instead of read by ds_bpermute (fxr; fxr3: with extract's launch bounds for 3) -- against the
# previous build (fxbase); identical output hashes required
set -euo pipefail
TAG=${TAG:-r04l}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u tools/exp/ref_route_time.py --block 8 --frames 16 --rounds 2 fxbase fxs fxs4 fxr fxr3 > $O/ref_route_b8.log 2>&1
timeout -k 10 300 python -u tools/exp/ref_route_time.py --block 16 --frames 16 --rounds 2 fxbase fxs fxr > $O/ref_route_b16.log 2>&1
echo done
