# Round-3 config lines on the current build: extract iteration A/B (noise + camera-like
# covers), configs[4] (512 x 4K, b = 16) and configs[1] (256 x 1080p) bench lines, the
# single-image app latency; TAG names the output dir
set -euo pipefail
O=gpurun_out/${TAG:-r03w}; mkdir -p $O
timeout -k 10 300 python -u tools/ab_variants.py --block 8 --frames 128 --rounds 2 it4 it3 it2 > $O/ab_it_noise.log 2>&1
timeout -k 10 300 python -u tools/ab_variants.py --block 8 --frames 64 --rounds 2 --cover photo it4 it3 it2 > $O/ab_it_photo.log 2>&1
timeout -k 10 600 python bench.py --frames 512 --block 16 --alpha 0.1 --steps 3 --cpu-frames 8 --lapack-frames 2 --structured-crops 0 > $O/bench_c4_512x4k_b16.log 2>&1
timeout -k 10 300 python bench.py --frames 256 --height 1080 --width 1920 --steps 5 --cpu-frames 16 --lapack-frames 4 --structured-crops 0 > $O/bench_c1_256x1080p.log 2>&1
timeout -k 10 300 python tools/app_latency.py > $O/app_latency_1080p.log 2>&1
echo done
