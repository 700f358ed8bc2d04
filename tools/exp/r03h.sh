# driver-flow sanity on the shipped build: smoke(), a 2-rank gloo rehearsal of bench.py's
# multi-rank path on the one GPU, and --gpus 2 refusing on a 1-GPU box (exit 2)
set -uo pipefail
O=gpurun_out/${TAG:-r03h}; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 600 python bench.py --gpus 2 --backend gloo --frames 64 --steps 2 --cpu-frames 4 --lapack-frames 2 --structured-crops 0 > $O/gloo_2ranks.log 2>&1 || exit 1
timeout -k 10 120 python bench.py --gpus 2 > $O/gpus2_refused.log 2>&1; echo "rc=$?" >> $O/gpus2_refused.log
echo done
