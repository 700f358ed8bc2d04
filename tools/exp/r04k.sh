# round-4: host-memory calls read their block counts after their one synchronisation (pinned
# count sink) and the drop-in's output buffers are page-locked (tmfwm_host_alloc)
set -euo pipefail
TAG=${TAG:-r04k}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_capi.py -m gpu -x -q --timeout 120 --timeout-method thread -k "pixel_layouts or zero_copy or dropin or golden or nonconv" > $O/tests.log 2>&1
timeout -k 10 300 python -u tools/app_latency.py > $O/app_latency_1080p.log 2>&1
timeout -k 10 300 python -u tools/exp/px_time.py > $O/px_time_1080p.log 2>&1
echo done
