#!/bin/bash
# Round 5: where the byte certificate's cycles go -- phase stamps and SQ instruction mix of
# embed_kernel<8> / <16> for the round-4 kernels (r04) and the certified build (c2), one box.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
O=$R/gpurun_out/r05c
mkdir -p $O
for B in 8 16; do
  timeout -k 10 900 bash tools/exp/ab_phase.sh $O/b$B $B r04 c2 || { echo "ab_phase b$B rc=$?" >> $O/status.log; exit 1; }
done

# kernel trace of the certified build on b = 16 camera-like covers with a QR watermark (fixup share)
(cd /tmp && export TMPDIR=/tmp && TMFWM_LIB=$R/variants/libtmfwm_c2.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_b16_qr -o run --output-format csv -- python3 $R/tools/time_embed.py --frames 128 --reps 3 --block 16 --kind photo --wm qr > $O/trace_b16_qr.log 2>&1) || echo "trace rc=$?" >> $O/status.log
echo ok >> $O/status.log
