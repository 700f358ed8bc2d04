#!/bin/bash
# Round 5, final build: the hybrid route against the reference route at every slider block size
# (camera-like covers, QR watermark, 512 4K frames each) and over whole 4096-frame batches at
# b = 8 and 16.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05z
mkdir -p $O
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" | tee -a $O/status.log; exit $rc; fi; }
for b in 4 6 10 12 14; do
  run 600 python3 tools/exp/route_diff_gpu.py --block $b --kind photo --wm qr --frames 512 --batch 32 > $O/route_diff_b${b}_photo_qr_512.log 2>&1
done
run 900 python3 tools/exp/route_diff_gpu.py --block 8 --kind photo --wm qr --frames 4096 --batch 64 > $O/route_diff_b8_photo_qr_4096.log 2>&1
run 900 python3 tools/exp/route_diff_gpu.py --block 16 --kind photo --wm qr --frames 4096 --batch 32 > $O/route_diff_b16_photo_qr_4096.log 2>&1
echo ok >> $O/status.log
