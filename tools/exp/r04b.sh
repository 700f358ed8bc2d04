# round-4 A/B: reconstruction chain loop order (embed spills), dgesdd-route group parallelism
set -euo pipefail
TAG=${TAG:-r04b}
O=gpurun_out/$TAG
mkdir -p $O
# the group-parallel dgesdd route (main build) against the oracle first
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "reference_route or lapack or golden or nonconvergence or list_pass or near_tie" > $O/gpu_tests_groupar.log 2>&1
timeout -k 10 300 python -u tools/exp/ref_route_time.py --block 8 --frames 16 --rounds 2 base gp8 gp16 gp16w fx4 > $O/ref_route_b8.log 2>&1
timeout -k 10 300 python -u tools/exp/ref_route_time.py --block 16 --frames 8 --rounds 2 base gp8 gp16w fx4 > $O/ref_route_b16.log 2>&1
timeout -k 10 300 python -u tools/ab_variants.py --block 16 --frames 64 --rounds 3 base chain both > $O/ab_b16.log 2>&1
timeout -k 10 300 python -u tools/ab_variants.py --block 8 --frames 128 --rounds 3 base chain both > $O/ab_b8.log 2>&1
timeout -k 10 200 python -u tools/ab_variants.py --block 12 --frames 64 --rounds 2 base chain > $O/ab_b12.log 2>&1
timeout -k 10 200 python -u tools/ab_variants.py --block 16 --frames 32 --rounds 2 --cover photo base chain > $O/ab_b16_photo.log 2>&1
echo done
