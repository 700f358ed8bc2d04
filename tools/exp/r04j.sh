# round-4: where a host-memory 1080p call's time goes by pixel layout (px_time.py) and the
# kernel / copy timeline of the zero-copy drop-in call (rocprofv3 kernel + memory-copy trace)
set -euo pipefail
TAG=${TAG:-r04j}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u tools/exp/px_time.py > $O/px_time_1080p.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $GRAFT_REPO_ROOT/$O/trace_app -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/app_latency.py --reps 5 > $GRAFT_REPO_ROOT/$O/trace_app.log 2>&1
echo done
