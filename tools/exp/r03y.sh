# GPU suite on the current build, then A/B of the phase-1 sweep count and the list pass at
# b = 10..16 (variants cur / s5 / s5d, tools/build_variant.sh); TAG names the output dir
set -uo pipefail
O=gpurun_out/${TAG:-r03y}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
for b in 16 12 14 10; do
  timeout -k 10 300 python -u tools/ab_variants.py --block $b --frames 32 --rounds 2 ${VARIANTS:-cur s5 s5d} > $O/ab_b$b.log 2>&1 || exit 1
done
timeout -k 10 300 python -u tools/ab_variants.py --block 16 --frames 32 --rounds 2 --cover photo ${VARIANTS:-cur s5 s5d} > $O/ab_b16_photo.log 2>&1
timeout -k 10 300 python -u tools/ab_variants.py --block 8 --frames 128 --rounds 3 cur x3 > $O/ab_b8_x3.log 2>&1
timeout -k 10 300 python -u tools/ab_variants.py --block 8 --frames 64 --rounds 2 --cover photo cur x3 > $O/ab_b8_x3_photo.log 2>&1
timeout -k 10 300 python -u tools/ab_variants.py --block 16 --frames 32 --rounds 2 cur x3 > $O/ab_b16_x3.log 2>&1
echo done
