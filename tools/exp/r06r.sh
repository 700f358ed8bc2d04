#!/bin/bash
# Round 6, last: smoke and the whole GPU suite on the final tree (the r06p build plus the rank-1
# routes' multi-GPU test), as the driver runs them at round end.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r06r
mkdir -p $O
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" | tee -a $O/status.log; exit $rc; fi; }
run 240 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
timeout -k 10 700 python3 -u -m pytest tests -x -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo "gpu tests rc=$?" >> $O/status.log
echo ok >> $O/status.log
