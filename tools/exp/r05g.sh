#!/bin/bash
# Round 5: c6 (branch-free interval construction, fractional-part byte test before the upper
# end's colour) against r04 / c3 at b = 8 / 16, noise and camera-like + QR covers; the
# hybrid-vs-reference tests on c6.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05g
mkdir -p $O
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" | tee -a $O/status.log; exit $rc; fi; }
for b in 8 16; do
  for cw in "noise noise" "photo qr"; do
    set -- $cw
    for v in r04 c3 c6; do
      TMFWM_LIB=$PWD/variants/libtmfwm_$v.so run 240 python3 tools/time_embed.py --frames 128 --reps 3 --block $b --kind $1 --wm $2 >> $O/ab.log 2>&1
    done
  done
done
TMFWM_LIB=$PWD/variants/libtmfwm_c6.so run 600 python3 -u -m pytest tests/test_gpu_parity.py -k "hybrid_vs_reference" -x -v --timeout 300 --timeout-method thread > $O/parity.log 2>&1
echo ok >> $O/status.log
