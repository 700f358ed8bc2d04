#!/bin/bash
# Round 5: embed<8>'s reconstruction chain by value selects (vs8) and pinned value selects (vs8p)
# against the shipped LDS-offset picks (c8), noise and camera-like + QR covers, two rounds.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r05s
mkdir -p $O
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" | tee -a $O/status.log; exit $rc; fi; }
for cw in "noise noise" "photo qr"; do
  set -- $cw
  for v in c8 vs8 vs8p c8 vs8 vs8p; do
    TMFWM_LIB=$R/variants/libtmfwm_$v.so run 240 python3 tools/time_embed.py --frames 128 --reps 3 --block 8 --kind $1 --wm $2 >> $O/ab.log 2>&1
  done
done
echo ok >> $O/status.log
