# round-3 closing pass on the shipped build: GPU suite, tools/profile_round.sh (bench line,
# rocprofv3 trace of the same command, counter passes b = 8 / 16, phase stamps), configs[4] line
set -euo pipefail
TAG=${TAG:-r03j}
mkdir -p gpurun_out/$TAG
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/gpu_tests.log 2>&1
bash tools/profile_round.sh $TAG
timeout -k 10 600 python bench.py --frames 512 --block 16 --alpha 0.1 --steps 3 --cpu-frames 8 --lapack-frames 2 --structured-crops 0 > gpurun_out/$TAG/bench_c4_512x4k_b16.log 2>&1
echo done
