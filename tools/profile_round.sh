#!/bin/bash
# Round evidence on the GPU box: tools/profile_round.sh <tag>   (e.g. r02e)
#   1. the default bench line (4096 x 4K, configs[2])                 -> gpurun_out/<tag>/bench.log
#   2. rocprofv3 --kernel-trace --stats of the same bench command      -> gpurun_out/<tag>/trace/
#   3. counter passes at b = 8 and b = 16 (tools/pmc_embed.sh: SQ mix, GRBM clock, FETCH/WRITE)
#                                                                       -> gpurun_out/<tag>/pmc_b{8,16}/
#   4. phase stamps (libtmfwm_stamps.so, if built: make -C thatsmyface_amd/csrc stamps)
#                                                                       -> gpurun_out/<tag>/stamps_b{8,16}.log
# Then, on the CPU side: tools/valu.py gpurun_out/<tag>/pmc_b8 (and pmc_b16) --build <lib_build>
# -> profiles/valu.json, which bench.py reads for roofline.traffic / valu_issue.
# Every GPU step has its own time limit; the first failure ends the script.
set -euo pipefail
TAG=${1:?tag}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT="$ROOT/gpurun_out/$TAG"
LIB="$ROOT/thatsmyface_amd/libtmfwm.so"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 "$ROOT/bench.py" > "$OUT/bench.log" 2>&1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --no-cpu-baseline > "$OUT/trace.log" 2>&1
"$ROOT/tools/pmc_embed.sh" "$LIB" "$OUT/pmc_b8" 8 16
"$ROOT/tools/pmc_embed.sh" "$LIB" "$OUT/pmc_b16" 16 16
if [ -f "$ROOT/thatsmyface_amd/libtmfwm_stamps.so" ]; then
  for B in 8 16; do
    timeout -k 10 180 python3 "$ROOT/tools/phase_stamps.py" --block $B --frames 64 > "$OUT/stamps_b$B.log" 2>&1
  done
fi
echo "profile_round $TAG done"
