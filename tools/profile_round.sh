#!/bin/bash
# Round evidence on the GPU box: tools/profile_round.sh <tag>   (e.g. r01c)
#   1. the default bench line (4096 x 4K, configs[2])              -> gpurun_out/<tag>/bench.log
#   2. rocprofv3 --kernel-trace --stats of the same bench command   -> gpurun_out/<tag>/trace/
#   3. separate --pmc FETCH_SIZE / WRITE_SIZE passes (64 frames)    -> gpurun_out/<tag>/pmc_{fetch,write}/
#   4. SQ instruction-mix passes (tools/pmc_embed.sh, 16 frames)     -> gpurun_out/<tag>/sq/
# Then, on the CPU side: tools/traffic.py -> profiles/traffic.json, tools/valu.py -> profiles/valu.json
# Every GPU step has its own time limit; the first failure ends the script.
set -euo pipefail
TAG=${1:?tag}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 "$ROOT/bench.py" > "$OUT/bench.log" 2>&1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --no-cpu-baseline > "$OUT/trace.log" 2>&1
for C in FETCH_SIZE WRITE_SIZE; do
  n=$(echo "$C" | cut -d_ -f1 | tr A-Z a-z)
  timeout -k 10 300 rocprofv3 --pmc "$C" -d "$OUT/pmc_$n" -o p --output-format csv -- \
      python3 "$ROOT/bench.py" --frames 64 --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/pmc_$n.log" 2>&1
done
"$ROOT/tools/pmc_embed.sh" "$ROOT/thatsmyface_amd/libtmfwm.so" "$OUT/sq"
echo "profile_round $TAG done"
