#!/bin/bash
# Round 6: the rank-1 route at b = 16: its GPU tests (and b = 8's again), us per 4K frame hybrid vs
# rank1 on camera-like covers, and configs[4]-sized (512 x 4K, b = 16) photo lines with the app's
# QR tile on both routes.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/${TAG:-r06i}
mkdir -p $O
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" | tee -a $O/status.log; exit $rc; fi; }
run 600 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "rank1" > $O/gpu_tests.log 2>&1
for cfg in "photo noise" "photo qr"; do
  set -- $cfg
  for rt in hybrid rank1 hybrid rank1; do
    run 240 python3 tools/time_embed.py --frames 64 --reps 3 --block 16 --kind $1 --wm $2 --route $rt --hash >> $O/ab.log 2>&1
  done
done
for rt in hybrid rank1; do
  run 900 python3 bench.py --covers photo --wm qr --block 16 --frames 512 --route $rt > $O/bench_c4_photo_appqr_${rt}.log 2>&1
done
echo ok >> $O/status.log
