#!/bin/bash
# Round 6 closing pass on the final build: smoke, the whole GPU suite, the default bench line
# (configs[2]) and its kernel trace, the rank1_reference route on camera-like covers + the app's QR
# tile at configs[2] scale, and the drop-in's single-image latency per route.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r06p
mkdir -p $O
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" | tee -a $O/status.log; exit $rc; fi; }
run 240 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc" >> $O/status.log
case $rc in 0|1) ;; *) exit $rc ;; esac
run 600 python3 bench.py > $O/bench.log 2>&1
run 600 python3 bench.py --covers photo --wm qr --route rank1_reference --no-cpu-baseline > $O/bench_photo_qr_rank1_reference.log 2>&1
run 300 python3 tools/app_latency.py --reps 30 > $O/latency.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
    python3 $R/bench.py --no-cpu-baseline > $O/trace.log 2>&1 || { echo "FAILED trace" >> $O/status.log; exit 1; }
echo ok >> $O/status.log
