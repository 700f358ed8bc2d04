# round-4: counter passes at b = 4 (why extract<4> takes 80 us per 4K frame)
set -euo pipefail
TAG=${TAG:-r04v}
O=gpurun_out/$TAG
mkdir -p $O
bash tools/pmc_embed.sh $GRAFT_REPO_ROOT/thatsmyface_amd/libtmfwm.so $GRAFT_REPO_ROOT/$O/pmc_b4 4 16 > $O/pmc_b4.log 2>&1
echo done
