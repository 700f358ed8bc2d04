#!/bin/bash
# Round 5: embed<16>'s reconstruction chain by value selects (vs16) against the LDS-offset picks of
# the final build (c9), noise and camera-like + QR covers, twice.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r05ad
mkdir -p $O
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" | tee -a $O/status.log; exit $rc; fi; }
for cw in "noise noise" "photo qr"; do
  set -- $cw
  for v in c9 vs16 c9 vs16; do
    TMFWM_LIB=$R/variants/libtmfwm_$v.so run 240 python3 tools/time_embed.py --frames 128 --reps 3 --block 16 --kind $1 --wm $2 >> $O/ab.log 2>&1
  done
done
echo ok >> $O/status.log
