# round-4 evidence on the shipped build: the hybrid route's bytes against the reference route over
# 2048 camera-like 4K frames at b = 16 (66 M blocks), and a rocprofv3 kernel trace of configs[4]
set -euo pipefail
TAG=${TAG:-r04s}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u tools/exp/route_diff_gpu.py --block 16 --kind photo --frames 2048 --batch 32 --seed 7 > $O/route_diff_b16_photo_2048.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/trace_c4 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --frames 512 --block 16 --no-cpu-baseline --lapack-frames 0 --exact-frames 0 > $GRAFT_REPO_ROOT/$O/trace_c4.log 2>&1
echo done
