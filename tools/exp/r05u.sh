#!/bin/bash
# Round 5: embed<16>'s Bjorck steps with N's upper triangle through LDS (main build: 136 cross-lane
# sums per step instead of 256) against the shipped c8, noise and camera-like + QR covers, twice;
# the b = 16 parity tests on the main build.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r05u
mkdir -p $O
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" | tee -a $O/status.log; exit $rc; fi; }
lib() { if [ $1 = c8 ]; then echo $R/variants/libtmfwm_c8.so; else echo $R/thatsmyface_amd/libtmfwm.so; fi; }
run 600 python3 -u -m pytest tests/test_gpu_parity.py -k "hybrid_vs_reference or config4 or alpha_edges or near_tie" -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
for cw in "noise noise" "photo qr"; do
  set -- $cw
  for v in c8 main c8 main; do
    TMFWM_LIB=$(lib $v) run 240 python3 tools/time_embed.py --frames 128 --reps 3 --block 16 --kind $1 --wm $2 >> $O/ab.log 2>&1
  done
done
echo ok >> $O/status.log
