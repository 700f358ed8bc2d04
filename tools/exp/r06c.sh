#!/bin/bash
# Round 6: the Newton finish's scaled acceptance test (the certificate's bound K).
# (1) smoke + the whole GPU suite on the new build (the Jacobi route bit-identical to the re-specified
# oracle, incl. the graded corpus); (2) A/B on one box, us per 4K frame: round-5 kernels (ab/r05)
# vs the new build (ab/cur) vs the new build + per-row ballot in the colour test (ab/ob1), b = 8 / 16,
# noise and camera-like + QR covers, output hashes; (3) drop-in latency, the round-4 tree vs this
# one; (4) extract<16> / <8> wait and latency counters; (5) the default bench line.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r06c
mkdir -p $O
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" | tee -a $O/status.log; exit $rc; fi; }
run 240 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc" >> $O/status.log
case $rc in 0|1) ;; *) exit $rc ;; esac
for cfg in "8 noise noise 128" "8 photo qr 128" "16 noise noise 64" "16 photo qr 64"; do
  set -- $cfg
  for v in r05 cur ob1 r05 cur ob1; do
    TMFWM_LIB=$R/ab/libtmfwm_$v.so run 240 python3 tools/time_embed.py --frames $4 --reps 3 --block $1 --kind $2 --wm $3 --hash >> $O/ab.log 2>&1
  done
done
for i in 1 2; do
  (cd $R/abtree_r04 && run 300 python3 tools/app_latency.py --reps 30 > $O/latency_r04_$i.log 2>&1) || exit 1
  run 300 python3 tools/app_latency.py --reps 30 > $O/latency_r06_$i.log 2>&1
done
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P2="SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU"
P3="SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH SQ_IFETCH SQ_LEVEL_WAVES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F32"
P4="GRBM_GUI_ACTIVE GRBM_COUNT"
for b in 16 8; do
  i=0
  for P in "$P1" "$P2" "$P3" "$P4"; do
    i=$((i+1))
    timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $P -d $O/x$b/p$i -o p --output-format csv -- \
      python3 $R/tools/time_embed.py --frames 16 --reps 1 --block $b > $O/x${b}_p$i.log 2>&1 || { echo "FAILED pmc $b $i" >> $O/status.log; exit 1; }
  done
done
cd $R
run 600 python3 bench.py > $O/bench.log 2>&1
echo ok >> $O/status.log
