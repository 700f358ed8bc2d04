# round-4 diagnosis of extract<4>: memory- and LDS-latency counters at b = 4 and b = 8
set -euo pipefail
TAG=${TAG:-r04ab}
O=gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_LDS_BANK_CONFLICT SQ_IFETCH SQ_INSTS_VMEM_RD"
for B in 4 8; do
  timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $P -d $GRAFT_REPO_ROOT/$O/lat_b$B -o p --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/time_embed.py --frames 16 --reps 1 --block $B > $GRAFT_REPO_ROOT/$O/lat_b$B.log 2>&1
done
echo done
