# round-4: why extract<4> is slow -- its work split, and a kernel trace of the same script
set -euo pipefail
TAG=${TAG:-r04u}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u tools/exp/x4_stats.py > $O/x4_stats.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/trace_x4 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/exp/x4_stats.py > $GRAFT_REPO_ROOT/$O/trace_x4.log 2>&1
echo done
