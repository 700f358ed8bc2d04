#!/bin/bash
# Round 6: the rank-1 routes at the slider sizes added late in the round, at scale: a 256-frame 4K
# bench line per size and route on camera-like covers with the app's QR tile (every timed frame
# compared with the reference route), the hybrid route's line beside each; and the multi-GPU entry
# points on the rank-1 routes.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r06q
mkdir -p $O
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" | tee -a $O/status.log; exit $rc; fi; }
run 300 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "multi_entry_points_rank1" > $O/gpu_tests.log 2>&1
for B in 4 6 10 12 14; do
  for rt in hybrid rank1 rank1_reference; do
    run 400 python3 bench.py --frames 256 --block $B --covers photo --wm qr --route $rt --no-cpu-baseline > $O/bench_256x4k_b${B}_photo_qr_$rt.log 2>&1
  done
done
echo ok >> $O/status.log
