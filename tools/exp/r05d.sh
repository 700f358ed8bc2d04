#!/bin/bash
# Round 5: certified build c3 (b-end picked by an LDS offset at b = 8 / 16, block-level straddle
# test) against round 4 at every slider block size (noise covers) and at b = 8 / 16 on camera-like
# covers with a QR watermark, one box; then the GPU suite on c3 (the tree's build).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05d
mkdir -p $O
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" | tee -a $O/status.log; exit $rc; fi; }
for cfg in "8 noise noise" "16 noise noise" "8 photo qr" "16 photo qr" "4 noise noise" "6 noise noise" "10 noise noise" "12 noise noise" "14 noise noise"; do
  set -- $cfg
  for v in r04 c3; do
    TMFWM_LIB=$PWD/variants/libtmfwm_$v.so run 240 python3 tools/time_embed.py --frames 128 --reps 3 --block $1 --kind $2 --wm $3 >> $O/ab.log 2>&1
  done
done
timeout -k 10 1200 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc" >> $O/status.log
echo ok >> $O/status.log
