# round-4: GPU suite with the full-size reference-route and route-comparison tests, the default
# bench line (configs[2]) with its exact-route sample, and configs[4]
set -euo pipefail
TAG=${TAG:-r04h}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 600 python bench.py > $O/bench.log 2>&1
timeout -k 10 300 python bench.py --frames 512 --block 16 --cpu-frames 8 --lapack-frames 2 --structured-crops 0 > $O/bench_c4_512x4k_b16.log 2>&1
echo done
