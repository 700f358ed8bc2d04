#!/bin/bash
# Round 5 closing pass, part 3: the hybrid route's bytes against the reference route's at scale
# on the shipped build (>= 66 M camera-like and >= 8 M noise blocks at b = 16,
# >= 66 M at b = 8), camera-like covers with a binary (QR) watermark and the bench's noise.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05p
mkdir -p $O
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" | tee -a $O/status.log; exit $rc; fi; }
run 600 python3 tools/exp/route_diff_gpu.py --block 16 --kind photo --wm qr --frames 2048 --batch 32 > $O/route_diff_b16_photo_qr_2048.log 2>&1
run 300 python3 tools/exp/route_diff_gpu.py --block 16 --kind noise --frames 256 --batch 32 > $O/route_diff_b16_noise_256.log 2>&1
run 300 python3 tools/exp/route_diff_gpu.py --block 8 --kind photo --wm qr --frames 512 --batch 32 > $O/route_diff_b8_photo_qr_512.log 2>&1
run 300 python3 tools/exp/route_diff_gpu.py --block 8 --kind noise --frames 256 --batch 32 > $O/route_diff_b8_noise_256.log 2>&1
echo ok >> $O/status.log
