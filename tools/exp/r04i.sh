# round-4: 4-byte pixel entry points (tmfwm_embed_px / tmfwm_extract_px) and the drop-in's
# zero-copy PIL path -- new tests first, then the whole GPU suite, then the app latency
set -euo pipefail
TAG=${TAG:-r04i}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "pixel_layouts or zero_copy" > $O/px_tests.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python -u tools/app_latency.py > $O/app_latency_1080p.log 2>&1
echo done
