#!/bin/bash
# rocprofv3 derived VALU metrics for one library build, one counter per pass:
#   tools/exp/valu_pmc.sh <outdir> <variant|tree>
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
OUT=$R/gpurun_out/$1
LIB=$R/variants/libtmfwm_$2.so
[ "$2" = tree ] && LIB=$R/thatsmyface_amd/libtmfwm.so
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for C in VALUBusy VALUUtilization GRBM_GUI_ACTIVE; do
  TMFWM_LIB=$LIB timeout -s KILL 90 rocprofv3 --pmc $C -d "$OUT/$C" -o p --output-format csv -- \
      python3 "$R/tools/time_embed.py" --frames 16 --reps 1 > "$OUT/$C.log" 2>&1
done
echo valu_pmc done
