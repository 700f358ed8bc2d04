# round-4: the GPU suite with the segmented-list tests (test_list_pass_segments_vs_oracle)
set -euo pipefail
TAG=${TAG:-r04ag}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "list_pass" -v -s --timeout 240 --timeout-method thread > $O/list_pass_tests.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
TAG=r04ah bash tools/exp/r04ah.sh
echo done
