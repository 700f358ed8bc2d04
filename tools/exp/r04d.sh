# round-4 config lines on the shipped build (after tools/valu.py has the r04c counters):
# configs[4] (512 x 4K, b = 16), configs[1] (256 x 1080p), the reference route, app latency
set -euo pipefail
TAG=${TAG:-r04d}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python bench.py --frames 512 --block 16 --alpha 0.1 --steps 3 --cpu-frames 8 --lapack-frames 2 --structured-crops 0 > $O/bench_c4_512x4k_b16.log 2>&1
timeout -k 10 300 python bench.py --frames 256 --height 1080 --width 1920 --steps 3 --cpu-frames 16 --lapack-frames 4 --structured-crops 0 > $O/bench_c1_256x1080p.log 2>&1
timeout -k 10 300 python bench.py --frames 256 --height 1080 --width 1920 --route reference --steps 2 --cpu-frames 4 --lapack-frames 4 --structured-crops 0 > $O/bench_c1_reference_route.log 2>&1
timeout -k 10 300 python -u tools/app_latency.py > $O/app_latency_1080p.log 2>&1
timeout -k 10 600 python -u tools/exp/multi_time.py --frames 96 > $O/multi_time_96x4k.log 2>&1
timeout -k 10 300 python -u tools/ab_variants.py --block 16 --frames 64 --rounds 3 base ls32 > $O/ab_ls32_b16.log 2>&1
timeout -k 10 200 python -u tools/ab_variants.py --block 14 --frames 64 --rounds 2 base ls32 > $O/ab_ls32_b14.log 2>&1
echo done
