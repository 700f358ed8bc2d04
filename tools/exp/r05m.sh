#!/bin/bash
# Round 5: the segmented dgesdd-route list alone (main build) against c7 (flat list): kernel
# traces of the hybrid route at b = 16 / 8 on camera-like + QR and noise covers; related tests.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r05m
mkdir -p $O
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" | tee -a $O/status.log; exit $rc; fi; }
lib() { if [ $1 = c7 ]; then echo $R/variants/libtmfwm_c7.so; else echo $R/thatsmyface_amd/libtmfwm.so; fi; }
run 600 python3 -u -m pytest tests/test_gpu_parity.py -k "near_tie or hybrid_vs_reference or segment or list_pass" -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
cd /tmp && export TMPDIR=/tmp
for b in 16 8; do
  for cw in "photo qr" "noise noise"; do
    set -- $cw
    for v in c7 main; do
      TMFWM_LIB=$(lib $v) timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --stats -d $O/app_${v}_b${b}_$1 -o p --output-format csv -- \
        python3 $R/tools/time_embed.py --frames 128 --reps 3 --block $b --kind $1 --wm $2 >> $O/app.log 2>&1 || { echo "FAILED trace $v $b" >> $O/status.log; exit 1; }
    done
  done
done
echo ok >> $O/status.log
