#!/bin/bash
# Round 5: extract<16> at five waves per SIMD (xw5: 96 VGPRs) against the shipped four (c8).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r05ac
mkdir -p $O
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" | tee -a $O/status.log; exit $rc; fi; }
for k in noise photo; do
  for v in c8 xw5 c8 xw5; do
    TMFWM_LIB=$R/variants/libtmfwm_$v.so run 240 python3 tools/time_embed.py --frames 128 --reps 3 --block 16 --kind $k >> $O/ab.log 2>&1
  done
done
TMFWM_LIB=$R/variants/libtmfwm_xw5.so run 600 python3 -u -m pytest tests/test_gpu_parity.py -k "extract" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo ok >> $O/status.log
