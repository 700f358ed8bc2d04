#!/bin/bash
# Round 5: the strip pass's deferral threshold at b = 8 with the certificate (kDeferMax 2 / 4 / 8:
# df2, c8 = shipped, df8), noise and camera-like + QR covers, twice.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r05x
mkdir -p $O
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" | tee -a $O/status.log; exit $rc; fi; }
for cw in "noise noise" "photo qr"; do
  set -- $cw
  for v in c8 df2 df8 c8 df2 df8; do
    TMFWM_LIB=$R/variants/libtmfwm_$v.so run 240 python3 tools/time_embed.py --frames 128 --reps 3 --block 8 --kind $1 --wm $2 >> $O/ab.log 2>&1
  done
done
echo ok >> $O/status.log
