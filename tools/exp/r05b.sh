#!/bin/bash
# Round 5, second pass: certificate variants (v4: source bytes to registers after the SVD, per-rank
# interval steps, flat-block rule; v5: the same with the source bytes re-read from L2 for the
# colour stage) against round 4 and the first certificate build, one box; then the GPU suite on v4.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05b
mkdir -p $O
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" | tee -a $O/status.log; exit $rc; fi; }
for cfg in "8 noise noise" "8 photo noise" "8 photo qr" "16 noise noise" "16 photo qr"; do
  set -- $cfg
  for v in r04 cert v4 v5; do
    TMFWM_LIB=$PWD/variants/libtmfwm_$v.so run 240 python3 tools/time_embed.py --frames 256 --reps 3 --block $1 --kind $2 --wm $3 >> $O/ab.log 2>&1
  done
done
run 300 python3 tools/exp/route_diff_gpu.py --block 8 --kind photo --wm qr --frames 256 --batch 32 > $O/route_diff_b8_photo_qr.log 2>&1
timeout -k 10 1200 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc" >> $O/status.log
echo ok >> $O/status.log
