# round-4 closing pass, second half (r04z ended at the phase stamps: the stamps library lacked
# the ABI's newest symbols): phase stamps, configs[4], configs[1] on both routes, the app latency,
# and the extract-enclosure A/B (xc: short fma chains, against xcur)
set -euo pipefail
TAG=${TAG:-r04q}
O=gpurun_out/$TAG
mkdir -p $O
for B in 8 16; do
  timeout -k 10 180 python3 tools/phase_stamps.py --block $B --frames 64 > $O/stamps_b$B.log 2>&1
done
timeout -k 10 300 python bench.py --frames 512 --block 16 --cpu-frames 8 --lapack-frames 2 --structured-crops 0 > $O/bench_c4_512x4k_b16.log 2>&1
timeout -k 10 300 python bench.py --frames 256 --height 1080 --width 1920 --steps 5 --cpu-frames 16 --lapack-frames 4 --structured-crops 0 > $O/bench_c1_256x1080p.log 2>&1
timeout -k 10 300 python bench.py --frames 256 --height 1080 --width 1920 --steps 3 --route reference --cpu-frames 8 --lapack-frames 4 --structured-crops 0 > $O/bench_c1_reference_route.log 2>&1
timeout -k 10 300 python -u tools/app_latency.py > $O/app_latency_1080p.log 2>&1
timeout -k 10 300 python -u tools/ab_variants.py --block 16 --frames 256 --rounds 3 xcur xc > $O/ab_xc_b16.log 2>&1
timeout -k 10 300 python -u tools/ab_variants.py --block 8 --frames 256 --rounds 3 xcur xc > $O/ab_xc_b8.log 2>&1
echo done
