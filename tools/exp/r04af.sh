# round-4: extract<4>'s strip pass with more power iterations before certifying (piN: N instead
# of 3 at b = 4 only) -- fewer list-pass blocks against longer strip-pass waves; head = HEAD
set -euo pipefail
TAG=${TAG:-r04af}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "list_pass" -v -s --timeout 240 --timeout-method thread > $O/list_pass_tests.log 2>&1
timeout -k 10 300 python -u tools/ab_variants.py --block 4 --frames 64 --rounds 3 head pi4 pi5 pi6 > $O/ab_pi_b4.log 2>&1
timeout -k 10 300 python -u tools/ab_variants.py --block 4 --frames 64 --rounds 2 --cover photo head pi4 pi5 pi6 > $O/ab_pi_b4_photo.log 2>&1
echo done
