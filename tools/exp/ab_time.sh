#!/bin/bash
# A/B timing of library variants on the GPU box, all in one call (boxes differ by ~5 %):
#   tools/exp/ab_time.sh <outdir> <variant>...   (variants/libtmfwm_<variant>.so)
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
OUT=$R/gpurun_out/$1; shift
mkdir -p "$OUT"
for v in "$@"; do
  TMFWM_LIB=$R/variants/libtmfwm_$v.so timeout -k 10 180 python3 "$R/tools/time_embed.py" --frames 512 --reps 5 >> "$OUT/time.log" 2>&1
done
cat "$OUT/time.log"
