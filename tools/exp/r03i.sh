# opaque q in the f64 sweep (b >= 14): GPU suite on the current build, A/B against HEAD (variants cur / oq)
set -uo pipefail
O=gpurun_out/${TAG:-r03i}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
for b in 16 12 14 10; do
  timeout -k 10 300 python -u tools/ab_variants.py --block $b --frames 32 --rounds 2 cur oq > $O/ab_b$b.log 2>&1 || exit 1
done
timeout -k 10 300 python -u tools/ab_variants.py --block 16 --frames 32 --rounds 2 --cover photo cur oq > $O/ab_b16_photo.log 2>&1
echo done
