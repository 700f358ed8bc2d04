#!/bin/bash
# Round 6 closing pass, part 1 (the shipped build): smoke, the counter passes behind
# profiles/valu.json (tools/pmc_embed.sh at b = 8 and 16; the Newton finish changed the embed
# kernels' code ids), then the whole GPU suite.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r06k
mkdir -p $O
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" | tee -a $O/status.log; exit $rc; fi; }
run 240 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
run 420 bash tools/pmc_embed.sh $R/thatsmyface_amd/libtmfwm.so $O/pmc_b8 8 16
run 420 bash tools/pmc_embed.sh $R/thatsmyface_amd/libtmfwm.so $O/pmc_b16 16 16
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo "gpu tests rc=$?" >> $O/status.log
echo ok >> $O/status.log
