# camera-like covers at b = 10..14: phase-1 sweep count variants (cur: 4, s5: 5 from b = 10, s5x: 5 for b = 10..14)
set -uo pipefail
O=gpurun_out/${TAG:-r03z}; mkdir -p $O
for b in 12 14 10; do
  timeout -k 10 300 python -u tools/ab_variants.py --block $b --frames 32 --rounds 2 --cover photo cur s5 s5x > $O/ab_b${b}_photo.log 2>&1 || exit 1
done
echo done
