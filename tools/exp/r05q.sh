#!/bin/bash
# Round 5: the source bytes re-read from global memory at the colour phase instead of parked in
# LDS and carried through the certificate (rl; embed<16> spilled VGPRs 27 -> 8) against the
# shipped build (c7), b = 8 / 16 / 14, noise and camera-like + QR; hybrid-vs-reference tests on rl.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r05q
mkdir -p $O
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" | tee -a $O/status.log; exit $rc; fi; }
for b in 16 8; do
  for cw in "noise noise" "photo qr"; do
    set -- $cw
    for v in c7 rl c7 rl; do
      TMFWM_LIB=$R/variants/libtmfwm_$v.so run 240 python3 tools/time_embed.py --frames 128 --reps 3 --block $b --kind $1 --wm $2 >> $O/ab.log 2>&1
    done
  done
done
for v in c7 rl; do TMFWM_LIB=$R/variants/libtmfwm_$v.so run 240 python3 tools/time_embed.py --frames 128 --reps 3 --block 14 >> $O/ab.log 2>&1; done
TMFWM_LIB=$R/variants/libtmfwm_rl.so run 600 python3 -u -m pytest tests/test_gpu_parity.py -k "hybrid_vs_reference" -x -v --timeout 300 --timeout-method thread > $O/parity.log 2>&1
echo ok >> $O/status.log
