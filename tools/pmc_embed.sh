#!/bin/bash
# SQ counter passes (8 counters each, separate runs) over tools/time_embed.py for one
# library build: tools/pmc_embed.sh <lib.so> <outdir>.  Run on the GPU box.
set -e
LIB=$1; OUT=$2
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32"
P2="SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH"
P3="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_LEVEL_WAVES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CU_CYCLES"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  TMFWM_LIB=$LIB timeout -k 10 120 rocprofv3 --pmc $P -d "$OUT/p$i" -o p --output-format csv -- python3 "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}/tools/time_embed.py" --frames 16 --reps 1 > "$OUT/p$i.log" 2>&1
done
