# round-4: the fixup pass picks a whole wave per block for short lists (GPU suite), configs[1]
# with 5 steps as round 3 ran it, and its kernel trace
set -euo pipefail
TAG=${TAG:-r04e}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python bench.py --frames 256 --height 1080 --width 1920 --steps 5 --cpu-frames 16 --lapack-frames 4 --structured-crops 0 > $O/bench_c1_256x1080p.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/trace_c1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --frames 256 --height 1080 --width 1920 --steps 5 --no-cpu-baseline --lapack-frames 0 > $GRAFT_REPO_ROOT/$O/trace_c1.log 2>&1
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/exp/ref_route_time.py --block 8 --frames 16 --rounds 1 gp8 > $O/ref_route_b8.log 2>&1
echo done
