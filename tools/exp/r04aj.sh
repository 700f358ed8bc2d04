# round-4 end rehearsal on the shipped build: what the driver runs (smoke, the default bench line),
# the bench now reading profiles/valu.json regenerated for this build (valu_issue, traffic)
set -euo pipefail
TAG=${TAG:-r04aj}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 600 python bench.py > $O/bench.log 2>&1
echo done
