#!/bin/bash
# Round 6: the rank-1 pre-pass priced on one box: us per 4K frame, hybrid vs rank1, b = 8, camera-like
# covers with the noise and the QR watermark and the bench's noise covers (hashes: the same bytes),
# then configs[2]-sized bench lines on camera-like covers, both watermarks, both routes.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/${TAG:-r06g}
mkdir -p $O
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" | tee -a $O/status.log; exit $rc; fi; }
for cfg in "photo noise" "photo qr" "noise noise"; do
  set -- $cfg
  for rt in hybrid rank1 hybrid rank1; do
    run 240 python3 tools/time_embed.py --frames 128 --reps 3 --block 8 --kind $1 --wm $2 --route $rt --hash >> $O/ab.log 2>&1
  done
done
for wm in noise qr; do
  for rt in hybrid rank1; do
    run 900 python3 bench.py --covers photo --wm $wm --route $rt > $O/bench_photo_${wm}_${rt}.log 2>&1
  done
done
echo ok >> $O/status.log
