set -euo pipefail
O=gpurun_out/${TAG:-r03d}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python bench.py --frames 256 --height 1080 --width 1920 --steps 5 --no-cpu-baseline --lapack-frames 0 > $O/bench_c1.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/trace_c1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --frames 256 --height 1080 --width 1920 --steps 5 --no-cpu-baseline --lapack-frames 0 > $GRAFT_REPO_ROOT/$O/trace_c1.log 2>&1
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/app_latency.py > $O/app_latency.log 2>&1
echo done
