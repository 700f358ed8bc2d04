#!/bin/bash
# Round 6: the rank-1 pre-pass with the rigorous IDCT rounding bound (tools/exp/idct_bound.py
# tables) at every slider size.  (1) the rank1 GPU tests (every slider size against the reference
# route); (2) A/B on one box, the previous pre-pass (ab/prev, gamma_16 |C| model) vs this one
# (ab/cur), us per 4K frame and hashes, b = 8 / 16 camera-like covers; (3) the new sizes: hybrid vs
# rank1 vs rank1_reference at b = 4 / 12, camera-like + app QR; (4) bench lines at configs[2] /
# configs[4] scale, camera-like + app QR, rank1 route.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r06o
mkdir -p $O
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" | tee -a $O/status.log; exit $rc; fi; }
run 600 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "rank1" > $O/gpu_tests.log 2>&1
for cfg in "8 photo noise 128" "8 photo qr 128" "16 photo noise 64" "16 photo qr 64"; do
  set -- $cfg
  for v in prev cur prev cur; do
    for rt in rank1 rank1_reference; do
      TMFWM_LIB=$R/ab/libtmfwm_$v.so run 240 python3 tools/time_embed.py --frames $4 --reps 3 --block $1 --kind $2 --wm $3 --route $rt --hash >> $O/ab.log 2>&1
    done
  done
done
for B in 4 12; do
  for rt in hybrid rank1 rank1_reference reference; do
    run 300 python3 tools/time_embed.py --frames 32 --reps 2 --block $B --kind photo --wm qr --route $rt --hash >> $O/sizes.log 2>&1
  done
done
run 600 python3 bench.py --covers photo --wm qr --route rank1 --no-cpu-baseline > $O/bench_photo_qr_rank1.log 2>&1
run 600 python3 bench.py --covers photo --wm qr --route rank1 --block 16 --frames 512 --no-cpu-baseline > $O/bench_c4_photo_qr_rank1.log 2>&1
echo ok >> $O/status.log
