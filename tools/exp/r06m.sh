#!/bin/bash
# Round 6: embed<16>'s counted traffic.  Its fetch is 2x the source bytes:
# the colour phase's re-read of the source misses L2.  Variant nt16: the output bytes stored
# non-temporal at b = 16 (no L2 allocation for a stream read by nobody), so that the source lines
# survive until the re-read.  A/B on one box (cur vs nt16, b = 16 noise and camera-like + QR, us per
# 4K frame and output hashes), then FETCH_SIZE / WRITE_SIZE of each at b = 16 and of each at b = 8
# (unchanged code there: a control).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r06m
mkdir -p $O
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" | tee -a $O/status.log; exit $rc; fi; }
for cfg in "16 noise noise 64" "16 photo qr 64"; do
  set -- $cfg
  for v in cur nt16 cur nt16; do
    TMFWM_LIB=$R/ab/libtmfwm_$v.so run 240 python3 tools/time_embed.py --frames $4 --reps 3 --block $1 --kind $2 --wm $3 --hash >> $O/ab.log 2>&1
  done
done
cd /tmp && export TMPDIR=/tmp
for v in cur nt16; do
  for P in FETCH_SIZE WRITE_SIZE; do
    TMFWM_LIB=$R/ab/libtmfwm_$v.so timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $P -d $O/pmc_$v/$P -o p --output-format csv -- \
      python3 $R/tools/time_embed.py --frames 16 --reps 1 --block 16 > $O/pmc_${v}_$P.log 2>&1 || { echo "FAILED pmc $v $P" >> $O/status.log; exit 1; }
  done
done
echo ok >> $O/status.log
