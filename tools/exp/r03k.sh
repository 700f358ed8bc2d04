# GPU tests, then the b = 16 config (configs[4]) and the headline bench; TAG names the output dir
set -euo pipefail
O=gpurun_out/${TAG:-r03k}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 600 python bench.py --frames 512 --block 16 --alpha 0.1 --steps 3 --cpu-frames 8 --lapack-frames 2 --structured-crops 0 > $O/bench_c4_512x4k_b16.log 2>&1
timeout -k 10 900 python bench.py > $O/bench_4096x4k.log 2>&1
echo done
