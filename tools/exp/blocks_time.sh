#!/bin/bash
# time_embed at several block sizes for several variants: tools/exp/blocks_time.sh <outdir> "<blocks>" <variant>...
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
OUT=$R/gpurun_out/$1; BL=$2; shift 2
mkdir -p "$OUT"
for b in $BL; do for v in "$@"; do
  TMFWM_LIB=$R/variants/libtmfwm_$v.so timeout -k 10 180 python3 "$R/tools/time_embed.py" --frames 128 --reps 3 --block $b >> "$OUT/blocks.log" 2>&1
done; done
grep lib "$OUT/blocks.log"
