#!/bin/bash
# Round 6: the scaled Newton test with its column sums formed after the rounds in the pair partials'
# free LDS slots (r06c's build had grown embed<16>'s LDS past 8 waves per CU: +9 % there).
# SVD + hybrid-route parity tests, then A/B on one box vs the round-5 kernels (ab/r05), hashes.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/${TAG:-r06d}
mkdir -p $O
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" | tee -a $O/status.log; exit $rc; fi; }
run 600 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "svd_blocks_gpu or hybrid_vs_reference or list_pass or config4 or golden" > $O/gpu_tests.log 2>&1
for cfg in "8 noise noise 128" "8 photo qr 128" "16 noise noise 64" "16 photo qr 64" "12 noise noise 64" "14 photo qr 64"; do
  set -- $cfg
  for v in r05 cur r05 cur; do
    TMFWM_LIB=$R/ab/libtmfwm_$v.so run 240 python3 tools/time_embed.py --frames $4 --reps 3 --block $1 --kind $2 --wm $3 --hash >> $O/ab.log 2>&1
  done
done
echo ok >> $O/status.log
