#!/bin/bash
# Round 5: extract<14> / <16> with both images' power iterations interleaved (x16) against the
# shipped sequential form (c8), noise and camera-like covers, twice.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r05y
mkdir -p $O
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" | tee -a $O/status.log; exit $rc; fi; }
for b in 16 14; do
  for k in noise photo; do
    for v in c8 x16 c8 x16; do
      TMFWM_LIB=$R/variants/libtmfwm_$v.so run 240 python3 tools/time_embed.py --frames 128 --reps 3 --block $b --kind $k >> $O/ab.log 2>&1
    done
  done
done
TMFWM_LIB=$R/variants/libtmfwm_x16.so run 600 python3 -u -m pytest tests/test_gpu_parity.py -k "extract or hybrid_vs_reference" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo ok >> $O/status.log
