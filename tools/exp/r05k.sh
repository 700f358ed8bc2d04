#!/bin/bash
# Round 5: the main build (dgesdd-route group LDS skewed over the banks; the hybrid route's
# dgesdd-route list segmented like the list passes') against c7: reference-route timings at
# b = 8 / 12 / 16, kernel traces of the hybrid route on camera-like + QR covers at b = 16 / 8,
# LDS counters of the reference route, and the related GPU tests.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r05k
mkdir -p $O
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" | tee -a $O/status.log; exit $rc; fi; }
lib() { if [ $1 = c7 ]; then echo $R/variants/libtmfwm_c7.so; else echo $R/thatsmyface_amd/libtmfwm.so; fi; }
run 900 python3 -u -m pytest tests/test_gpu_parity.py -k "lapack or golden or reference or hybrid or segment or list" -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
for b in 8 12 16; do
  for v in c7 main; do
    TMFWM_LIB=$(lib $v) run 240 python3 tools/time_embed.py --frames 16 --reps 2 --block $b --route reference >> $O/ab.log 2>&1
  done
done
cd /tmp && export TMPDIR=/tmp
for b in 16 8; do
  for v in c7 main; do
    TMFWM_LIB=$(lib $v) timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --stats -d $O/app_${v}_b$b -o p --output-format csv -- \
      python3 $R/tools/time_embed.py --frames 128 --reps 3 --block $b --kind photo --wm qr >> $O/app.log 2>&1 || { echo "FAILED trace $v $b" >> $O/status.log; exit 1; }
  done
done
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
for b in 8 16; do
  timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $P1 -d $O/ref_b$b -o p --output-format csv -- \
    python3 $R/tools/time_embed.py --frames 4 --reps 1 --block $b --route reference > $O/ref_b$b.log 2>&1 || { echo "FAILED pmc $b" >> $O/status.log; exit 1; }
done
echo ok >> $O/status.log
