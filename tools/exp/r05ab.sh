#!/bin/bash
# Round 5, the final library (extract<14> interleaved): the whole GPU suite and smoke.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05ab
mkdir -p $O
timeout -k 10 240 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "FAILED smoke" >> $O/status.log; exit 1; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo "gpu tests rc=$?" >> $O/status.log
