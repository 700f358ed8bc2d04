#!/bin/bash
# Counter passes over tools/time_embed.py for one library build and block size, one
# rocprofv3 run per pass (rocprofv3 does not split counters over passes):
#   tools/pmc_embed.sh <lib.so> <outdir> [block=8] [frames=16]
# p1-p3: SQ instruction mix and wave cycles; p4: GRBM_GUI_ACTIVE with the kernel trace
# (effective clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel time); p5/p6: FETCH_SIZE and
# WRITE_SIZE (HBM traffic).  The block size is recorded in <outdir>/block for tools/valu.py.
# Run on the GPU box.
set -euo pipefail
LIB=$1; OUT=$2; BLOCK=${3:-8}; FRAMES=${4:-16}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p "$OUT"
echo "$BLOCK $FRAMES" > "$OUT/block"
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32"
P2="SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH"
P3="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_LEVEL_WAVES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CU_CYCLES"
P4="GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$P1" "$P2" "$P3" "$P4" FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  TMFWM_LIB=$LIB timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $P -d "$OUT/p$i" -o p --output-format csv -- \
      python3 "$ROOT/tools/time_embed.py" --frames "$FRAMES" --reps 1 --block "$BLOCK" > "$OUT/p$i.log" 2>&1
done
echo "pmc_embed b=$BLOCK done"
