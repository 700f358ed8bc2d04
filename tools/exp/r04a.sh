# round-4 first pass: GPU suite on the ABI-7 build, app-path latency breakdown, reference-route throughput
set -euo pipefail
TAG=${TAG:-r04a}
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/gpu_tests.log 2>&1
timeout -k 10 300 python -u tools/app_latency.py > gpurun_out/$TAG/app_latency_1080p.log 2>&1
timeout -k 10 300 python bench.py --frames 256 --height 1080 --width 1920 --route reference --steps 2 --cpu-frames 4 --lapack-frames 2 --structured-crops 0 > gpurun_out/$TAG/bench_c1_reference_route.log 2>&1
echo done
