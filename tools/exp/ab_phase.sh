#!/bin/bash
# A/B evidence for embed_kernel<b> variants on one box: timing (tools/ab_variants.py), phase
# stamps (variants/libtmfwm_<name>_stamps.so) and the SQ instruction-mix counter pass.
#   tools/exp/ab_phase.sh <outdir> <block> <name>...
set -euo pipefail
OUT=$(mkdir -p "$1" && cd "$1" && pwd); B=$2; shift 2
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
mkdir -p "$OUT"
timeout -k 10 300 python3 "$ROOT/tools/ab_variants.py" --block "$B" --frames 64 --rounds 3 "$@" > "$OUT/ab.log" 2>&1
for N in "$@"; do
  if [ -f "$ROOT/variants/libtmfwm_${N}_stamps.so" ]; then
    TMF_STAMPS_LIB="$ROOT/variants/libtmfwm_${N}_stamps.so" timeout -k 10 180 python3 "$ROOT/tools/phase_stamps.py" --block "$B" --frames 64 > "$OUT/stamps_$N.log" 2>&1
  fi
  (cd /tmp && export TMPDIR=/tmp && TMFWM_LIB="$ROOT/variants/libtmfwm_$N.so" timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace \
      --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 \
      -d "$OUT/pmc_$N" -o p --output-format csv -- python3 "$ROOT/tools/time_embed.py" --frames 16 --reps 1 --block "$B" > "$OUT/pmc_$N.log" 2>&1)
done
echo "ab_phase done"
