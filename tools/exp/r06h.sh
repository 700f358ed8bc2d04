#!/bin/bash
# Round 6: the rank-1 route's GPU tests, and camera-like 4096 x 4K bench lines with the app's own QR
# tile (synth_qr_tile: text_to_qrcode + resize_watermark(preserve_ratio=True)), hybrid vs rank1.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/${TAG:-r06h}
mkdir -p $O
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" | tee -a $O/status.log; exit $rc; fi; }
run 600 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "rank1" > $O/gpu_tests.log 2>&1
for rt in hybrid rank1; do
  run 900 python3 bench.py --covers photo --wm qr --route $rt > $O/bench_photo_appqr_${rt}.log 2>&1
done
echo ok >> $O/status.log
