# round-4: the hybrid route's bytes against the GPU reference route at scale (route_diff_gpu.py),
# and configs[1] with the warmed timing hooks and the bench's exact-route sample
set -euo pipefail
TAG=${TAG:-r04f}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u tools/exp/route_diff_gpu.py --block 16 --kind photo --frames 512 --batch 32 > $O/route_diff_b16_photo.log 2>&1
timeout -k 10 300 python -u tools/exp/route_diff_gpu.py --block 16 --kind noise --frames 256 --batch 32 > $O/route_diff_b16_noise.log 2>&1
timeout -k 10 300 python -u tools/exp/route_diff_gpu.py --block 8 --kind photo --frames 512 --batch 32 > $O/route_diff_b8_photo.log 2>&1
timeout -k 10 300 python -u tools/exp/route_diff_gpu.py --block 8 --kind noise --frames 256 --batch 32 > $O/route_diff_b8_noise.log 2>&1
timeout -k 10 300 python bench.py --frames 256 --height 1080 --width 1920 --steps 5 --cpu-frames 16 --lapack-frames 4 --structured-crops 0 > $O/bench_c1_256x1080p.log 2>&1
echo done
