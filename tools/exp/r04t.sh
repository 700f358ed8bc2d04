# round-4: every slider block size on the shipped build -- 256 x 4K frames per line (hybrid route,
# parity sample vs the oracle and its dgesdd route, 16-frame exact-route sample)
set -euo pipefail
TAG=${TAG:-r04t}
O=gpurun_out/$TAG
mkdir -p $O
for B in 4 6 8 10 12 14 16; do
  timeout -k 10 300 python bench.py --frames 256 --block $B --steps 3 --cpu-frames 4 --lapack-frames 1 --structured-crops 0 --exact-frames 16 > $O/bench_256x4k_b$B.log 2>&1
done
echo done
