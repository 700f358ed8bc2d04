# round-4: extract's sigma_1 enclosure with its b-term sums as several short fma chains (xc)
# against the current build (xcur); the output hashes must agree
set -euo pipefail
TAG=${TAG:-r04p}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u tools/ab_variants.py --block 16 --frames 256 --rounds 3 xcur xc > $O/ab_xc_b16.log 2>&1
timeout -k 10 300 python -u tools/ab_variants.py --block 8 --frames 256 --rounds 3 xcur xc > $O/ab_xc_b8.log 2>&1
echo done
