#!/bin/bash
# Round 5 closing pass for the b = 16 kernel with the source-byte reload (shipped build): its
# counter passes -> profiles/valu.json (tools/valu.py on the box; copied back as
# gpurun_out/r05r/valu.json), the configs[4] alpha sweep, the route comparison at b = 16, the
# hybrid-vs-reference tests.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r05r
mkdir -p $O
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" | tee -a $O/status.log; exit $rc; fi; }
LIB=$R/thatsmyface_amd/libtmfwm.so
bash $R/tools/pmc_embed.sh $LIB $O/pmc_b16 16 16 > $O/pmc_b16.log 2>&1 || { echo "FAILED pmc b16" >> $O/status.log; exit 1; }
cd $R
run 120 python3 tools/valu.py $O/pmc_b16 --build $(sha256sum $LIB | cut -c1-16) --out profiles/valu.json > $O/valu.log 2>&1
cp profiles/valu.json $O/valu.json
run 600 python3 -u -m pytest tests/test_gpu_parity.py -k "hybrid_vs_reference" -x -v --timeout 300 --timeout-method thread > $O/parity.log 2>&1
for a in 0.01 0.05 0.1 0.15 0.2; do
  X=--no-cpu-baseline; [ $a = 0.1 ] && X=
  run 400 python3 bench.py --frames 512 --block 16 --alpha $a --steps 3 --warmup 1 $X > $O/bench_c4_512x4k_b16_a$a.log 2>&1
done
run 600 python3 tools/exp/route_diff_gpu.py --block 16 --kind photo --wm qr --frames 2048 --batch 32 > $O/route_diff_b16_photo_qr_2048.log 2>&1
run 300 python3 tools/exp/route_diff_gpu.py --block 16 --kind noise --frames 256 --batch 32 > $O/route_diff_b16_noise_256.log 2>&1
echo ok >> $O/status.log
