#!/bin/bash
# Round 5: c7 (bank-spread LDS tile strides at b = 8 / 16) against c6 / r04, its LDS counters,
# and the hybrid-vs-reference tests on c7.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r05i
mkdir -p $O
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" | tee -a $O/status.log; exit $rc; fi; }
for b in 8 16; do
  for cw in "noise noise" "photo qr"; do
    set -- $cw
    for v in r04 c6 c7; do
      TMFWM_LIB=$R/variants/libtmfwm_$v.so run 240 python3 tools/time_embed.py --frames 128 --reps 3 --block $b --kind $1 --wm $2 >> $O/ab.log 2>&1
    done
  done
done
TMFWM_LIB=$R/variants/libtmfwm_c7.so run 600 python3 -u -m pytest tests/test_gpu_parity.py -k "hybrid_vs_reference" -x -v --timeout 300 --timeout-method thread > $O/parity.log 2>&1
cd /tmp && export TMPDIR=/tmp
P="SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES"
for b in 8 16; do
  TMFWM_LIB=$R/variants/libtmfwm_c7.so timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $P -d $O/c7_b$b -o p --output-format csv -- \
    python3 $R/tools/time_embed.py --frames 16 --reps 1 --block $b > $O/c7_b$b.log 2>&1 || { echo "FAILED pmc $b" >> $O/status.log; exit 1; }
done
echo ok >> $O/status.log
