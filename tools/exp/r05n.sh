#!/bin/bash
# Round 5 closing pass, part 1 (shipped build): counter passes at b = 8 / 16 (-> profiles/valu.json
# on the CPU side), the whole GPU suite, smoke.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r05n
mkdir -p $O
LIB=$R/thatsmyface_amd/libtmfwm.so
bash $R/tools/pmc_embed.sh $LIB $O/pmc_b8 8 16 > $O/pmc_b8.log 2>&1 || { echo "FAILED pmc b8" >> $O/status.log; exit 1; }
bash $R/tools/pmc_embed.sh $LIB $O/pmc_b16 16 16 > $O/pmc_b16.log 2>&1 || { echo "FAILED pmc b16" >> $O/status.log; exit 1; }
cd $R
timeout -k 10 240 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "FAILED smoke" >> $O/status.log; exit 1; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc" >> $O/status.log
echo ok >> $O/status.log
