#!/bin/bash
# Round 6 closing pass, part 3 (the shipped build): every slider block size (256 x 4K, hybrid route,
# a 16-frame sample against the reference route per line), the photo-mode lines at configs[2] scale
# (camera-like covers + the app's QR tile, b = 8: hybrid / rank1), and phase stamps at b = 8 / 16
# (libtmfwm_stamps.so, the same kernels with s_memtime stamps).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r06n
mkdir -p $O
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" | tee -a $O/status.log; exit $rc; fi; }
for B in 4 6 8 10 12 14 16; do
  run 300 python3 bench.py --frames 256 --block $B --steps 3 --cpu-frames 4 --lapack-frames 1 --structured-crops 0 --exact-frames 16 > $O/bench_256x4k_b$B.log 2>&1
done
for rt in hybrid rank1; do
  run 600 python3 bench.py --covers photo --wm qr --route $rt --no-cpu-baseline > $O/bench_photo_qr_$rt.log 2>&1
done
for B in 8 16; do
  run 180 python3 tools/phase_stamps.py --block $B --frames 64 > $O/stamps_b$B.log 2>&1
done
echo ok >> $O/status.log
