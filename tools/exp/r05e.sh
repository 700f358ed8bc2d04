#!/bin/bash
# Round 5: launch-bound / register variants of the certified kernels at b = 8, 10, 14, 16 (c3: the
# committed build; c4: E held as a float, b = 10 at 2 waves / SIMD, b = 14 unconstrained), one box.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05e
mkdir -p $O
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" | tee -a $O/status.log; exit $rc; fi; }
for b in 10 14 16 8; do
  for v in r04 c3 c4; do
    TMFWM_LIB=$PWD/variants/libtmfwm_$v.so run 240 python3 tools/time_embed.py --frames 128 --reps 3 --block $b >> $O/ab.log 2>&1
  done
done
echo ok >> $O/status.log
