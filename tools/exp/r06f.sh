#!/bin/bash
# Round 6: the rank-1 pre-pass (TMFWM_ROUTE_RANK1, photo mode): parity against the reference route
# (its own GPU tests), then us per 4K frame on one box, hybrid vs rank1, camera-like + QR / noise
# covers, output hashes (the same bytes on both routes).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/${TAG:-r06f}
mkdir -p $O
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" | tee -a $O/status.log; exit $rc; fi; }
run 600 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "rank1 or svd_blocks_gpu" > $O/gpu_tests.log 2>&1
for cfg in "photo qr" "photo noise" "noise noise"; do
  set -- $cfg
  for rt in hybrid rank1 hybrid rank1; do
    run 240 python3 tools/time_embed.py --frames 128 --reps 3 --block 8 --kind $1 --wm $2 --route $rt --hash >> $O/ab.log 2>&1
  done
done
echo ok >> $O/status.log
# configs[2]-sized lines on camera-like covers + QR tile: the hybrid route and the rank-1 route
run 900 python3 bench.py --covers photo --wm qr --route hybrid > $O/bench_photo_qr_hybrid.log 2>&1
run 900 python3 bench.py --covers photo --wm qr --route rank1 > $O/bench_photo_qr_rank1.log 2>&1
echo ok2 >> $O/status.log
