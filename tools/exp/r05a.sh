#!/bin/bash
# Round 5, first GPU pass: cost of the byte certificate (A/B against the round-4 kernels on one
# box: noise / camera-like covers, uniform / QR watermark, b = 8 and 16), the hybrid route
# against the reference route at b = 16 with a QR watermark, the GPU suite, the configs[2] line
# (every timed frame checked against the reference route).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05a
mkdir -p $O
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" | tee -a $O/status.log; exit $rc; fi; }
for b in 8 16; do
  for cw in "noise noise" "photo noise" "photo qr"; do
    set -- $cw
    for v in r04 cert; do
      TMFWM_LIB=$PWD/variants/libtmfwm_$v.so run 240 python3 tools/time_embed.py --frames 256 --reps 3 --block $b --kind $1 --wm $2 >> $O/ab.log 2>&1
    done
  done
done
run 300 python3 tools/exp/route_diff_gpu.py --block 16 --kind photo --wm qr --frames 256 --batch 32 > $O/route_diff_b16_photo_qr.log 2>&1
run 300 python3 tools/exp/route_diff_gpu.py --block 16 --kind noise --frames 256 --batch 32 > $O/route_diff_b16_noise.log 2>&1
timeout -k 10 1200 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc" >> $O/status.log
case $rc in 0|1) ;; *) exit $rc ;; esac
run 900 python3 bench.py > $O/bench.log 2>&1
echo ok >> $O/status.log
