#!/bin/bash
# Round 6 closing pass, part 2 (the shipped build, profiles/valu.json from part 1): the default
# bench line (configs[2]) and its kernel trace, the configs[4] alpha sweep (512 x 4K, b = 16, every
# frame checked against the reference route), configs[1], and the drop-in-grade rank1_reference
# route on camera-like covers with the app's QR tile at configs[2] scale.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r06l
mkdir -p $O
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" | tee -a $O/status.log; exit $rc; fi; }
run 600 python3 bench.py > $O/bench.log 2>&1
for a in 0.01 0.05 0.1 0.15 0.2; do
  X=--no-cpu-baseline; [ $a = 0.1 ] && X=
  run 400 python3 bench.py --frames 512 --block 16 --alpha $a --steps 3 --warmup 1 $X > $O/bench_c4_512x4k_b16_a$a.log 2>&1
done
run 300 python3 bench.py --frames 256 --height 1080 --width 1920 > $O/bench_c1_256x1080p.log 2>&1
run 600 python3 bench.py --covers photo --wm qr --route rank1_reference --no-cpu-baseline > $O/bench_photo_qr_rank1_reference.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
    python3 $R/bench.py --no-cpu-baseline > $O/trace.log 2>&1 || { echo "FAILED trace" >> $O/status.log; exit 1; }
echo ok >> $O/status.log
