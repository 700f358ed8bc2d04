#!/bin/bash
# Round 6 start: smoke + the default bench line on the round-5 shipped build (box sanity / baseline).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06a
mkdir -p $O
timeout -k 10 240 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "FAILED smoke" >> $O/status.log; exit 1; }
timeout -k 10 600 python3 bench.py > $O/bench.log 2>&1 || { echo "FAILED bench" >> $O/status.log; exit 1; }
echo ok >> $O/status.log
