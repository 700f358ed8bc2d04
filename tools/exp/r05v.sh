#!/bin/bash
# Round 5, final build: the whole GPU suite, smoke, and the default bench line (configs[2]).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05v
mkdir -p $O
timeout -k 10 240 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "FAILED smoke" >> $O/status.log; exit 1; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc" >> $O/status.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 600 python3 bench.py > $O/bench.log 2>&1 || { echo "FAILED bench" >> $O/status.log; exit 1; }
echo ok >> $O/status.log
