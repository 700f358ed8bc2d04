#!/bin/bash
# Round 5: LDS counters (bank conflicts, array cycles) of embed<8> / embed<16>, r04 vs c6 (one
# counter pass per library and block size over tools/time_embed.py, 16 frames).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r05h
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P="SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES"
for b in 8 16; do
  for v in r04 c6; do
    TMFWM_LIB=$R/variants/libtmfwm_$v.so timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $P -d $O/${v}_b$b -o p --output-format csv -- \
      python3 $R/tools/time_embed.py --frames 16 --reps 1 --block $b > $O/${v}_b$b.log 2>&1 || { echo "FAILED $v $b" >> $O/status.log; exit 1; }
  done
done
echo ok >> $O/status.log
