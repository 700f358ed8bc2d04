# round-4: kernel trace of the b = 4 per-b line on the shipped build (extract<4> after the segmented
# list and the (D^T D)^4 power vector)
set -euo pipefail
TAG=${TAG:-r04am}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace_b4 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --frames 256 --block 4 --steps 3 --no-cpu-baseline --lapack-frames 1 --structured-crops 0 > $O/trace_b4.log 2>&1
echo done
