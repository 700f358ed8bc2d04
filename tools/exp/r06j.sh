#!/bin/bash
# Round 6: TMFWM_ROUTE_RANK1_REFERENCE (the rank-1 pre-pass in front of the dgesdd route): its GPU
# tests, us per 4K frame against the reference route (the drop-in's default) on camera-like and
# noise covers, b = 8 / 16, and the drop-in's single-image latency with svd_route rank1_reference.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/${TAG:-r06j}
mkdir -p $O
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" | tee -a $O/status.log; exit $rc; fi; }
run 600 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "rank1" > $O/gpu_tests.log 2>&1
for b in 8 16; do
  for cfg in "photo noise" "photo qr" "noise noise"; do
    set -- $cfg
    for rt in reference rank1_reference; do
      run 300 python3 tools/time_embed.py --frames 16 --reps 2 --block $b --kind $1 --wm $2 --route $rt --hash >> $O/ab.log 2>&1
    done
  done
done
run 300 python3 tools/app_latency.py --reps 30 > $O/latency.log 2>&1
echo ok >> $O/status.log
