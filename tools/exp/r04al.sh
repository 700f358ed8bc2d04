# round-4: validation of the (D^T D)^4 power vector at b = 4 (build 0beaa79a; only extract_kernel<4>'s
# code changed): smoke, GPU suite, the b = 4 per-b line, the default bench line
set -euo pipefail
TAG=${TAG:-r04al}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python bench.py --frames 256 --block 4 --steps 3 --cpu-frames 4 --lapack-frames 1 --structured-crops 0 --exact-frames 16 > $O/bench_256x4k_b4.log 2>&1
timeout -k 10 600 python bench.py > $O/bench.log 2>&1
echo done
