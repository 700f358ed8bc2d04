#!/bin/bash
# Round 5: the certified kernels with the reconstruction chain pinned in k-outer order (c5v: value
# selects at b != 8 / 16; c5o: LDS-offset picks at every b) against r04 / c3, b = 8..16, one box;
# then the hybrid-vs-reference parity tests on the main build.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05f
mkdir -p $O
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" | tee -a $O/status.log; exit $rc; fi; }
for b in 14 10 12 16 8; do
  for v in r04 c3 c5v c5o; do
    TMFWM_LIB=$PWD/variants/libtmfwm_$v.so run 240 python3 tools/time_embed.py --frames 128 --reps 3 --block $b >> $O/ab.log 2>&1
  done
done
for v in r04 c5v c5o; do
  TMFWM_LIB=$PWD/variants/libtmfwm_$v.so run 240 python3 tools/time_embed.py --frames 128 --reps 3 --block 16 --kind photo --wm qr >> $O/ab.log 2>&1
done
run 600 python3 -u -m pytest tests/test_gpu_parity.py -k "hybrid or embed" -x -v --timeout 300 --timeout-method thread > $O/parity.log 2>&1
echo ok >> $O/status.log
