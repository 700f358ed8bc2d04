# round-4: extract<4>'s stalls -- the counters this rocprofv3 offers (listed), then one SQ pass
# with the wait / memory-instruction counters at b = 4 and b = 8
set -euo pipefail
TAG=${TAG:-r04y}
O=gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --list-avail > $GRAFT_REPO_ROOT/$O/list_avail.txt 2>&1 || true
grep -o "SQ_[A-Z0-9_]*" $GRAFT_REPO_ROOT/$O/list_avail.txt | sort -u > $GRAFT_REPO_ROOT/$O/sq_counters.txt || true
P="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_LDS"
for B in 4 8; do
  timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $P -d $GRAFT_REPO_ROOT/$O/sq_b$B -o p --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/time_embed.py --frames 16 --reps 1 --block $B > $GRAFT_REPO_ROOT/$O/sq_b$B.log 2>&1
done
echo done
