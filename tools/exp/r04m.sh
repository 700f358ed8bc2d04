# round-4: the current build end to end -- smoke, the whole GPU suite, configs[1] on both routes,
# and the app latency (the reference route's extract pass with the smaller LDS workspace)
set -euo pipefail
TAG=${TAG:-r04m}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python bench.py --frames 256 --height 1080 --width 1920 --steps 5 --cpu-frames 16 --lapack-frames 4 --structured-crops 0 > $O/bench_c1_256x1080p.log 2>&1
timeout -k 10 300 python bench.py --frames 256 --height 1080 --width 1920 --steps 3 --route reference --cpu-frames 8 --lapack-frames 4 --structured-crops 0 > $O/bench_c1_reference_route.log 2>&1
timeout -k 10 300 python -u tools/app_latency.py > $O/app_latency_1080p.log 2>&1
# embed pass of the dgesdd route with D and M aliased into the workspace (fxa) against this build (fxs)
timeout -k 10 300 python -u tools/exp/ref_route_time.py --block 8 --frames 16 --rounds 2 fxs fxa > $O/ref_route_b8.log 2>&1
timeout -k 10 300 python -u tools/exp/ref_route_time.py --block 16 --frames 16 --rounds 2 fxs fxa > $O/ref_route_b16.log 2>&1
echo done
