# round-4 pass on the shipped build: GPU suite, tools/profile_round.sh (bench line, rocprofv3
# trace of the same command, counter passes b = 8 / 16, phase stamps)
set -euo pipefail
TAG=${TAG:-r04c}
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/gpu_tests.log 2>&1
bash tools/profile_round.sh $TAG
echo done
