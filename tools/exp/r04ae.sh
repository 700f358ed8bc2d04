# round-4 closing pass after the segmented list appends: smoke, the whole GPU suite, the round's
# evidence (tools/profile_round.sh), the configs[4] / configs[1] lines (both routes), the app
# latency, and the b = 4 and 8 lines of the per-b table (r04t's command)
set -euo pipefail
TAG=${TAG:-r04ae}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
bash tools/profile_round.sh $TAG > $O/profile_round.log 2>&1
timeout -k 10 300 python bench.py --frames 512 --block 16 --cpu-frames 8 --lapack-frames 2 --structured-crops 0 > $O/bench_c4_512x4k_b16.log 2>&1
timeout -k 10 300 python bench.py --frames 256 --height 1080 --width 1920 --steps 5 --cpu-frames 16 --lapack-frames 4 --structured-crops 0 > $O/bench_c1_256x1080p.log 2>&1
timeout -k 10 300 python bench.py --frames 256 --height 1080 --width 1920 --steps 3 --route reference --cpu-frames 8 --lapack-frames 4 --structured-crops 0 > $O/bench_c1_reference_route.log 2>&1
for B in 4 8; do
  timeout -k 10 300 python bench.py --frames 256 --block $B --steps 3 --cpu-frames 4 --lapack-frames 1 --structured-crops 0 --exact-frames 16 > $O/bench_256x4k_b$B.log 2>&1
done
timeout -k 10 300 python -u tools/app_latency.py > $O/app_latency_1080p.log 2>&1
echo done
