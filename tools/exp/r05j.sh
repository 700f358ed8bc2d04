#!/bin/bash
# Round 5: (1) counters of the reference route's kernels (embed_fixup_kernel / extract_fixup_kernel,
# every block on the dgesdd route) at b = 8 / 16; (2) the fixup-list append's cost: kernel trace of
# embed<16> on camera-like covers + QR watermark (0.8 % of blocks append) with the shipped build
# and with the append's atomic replaced by a plain store (variants/libtmfwm_noapp.so).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r05j
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
P2="SQ_WAVES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_LEVEL_WAVES SQ_INSTS_VALU_TRANS_F64"
P3="GRBM_GUI_ACTIVE GRBM_COUNT"
for b in 8 16; do
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $P -d $O/ref_b$b/p$i -o p --output-format csv -- \
      python3 $R/tools/time_embed.py --frames 4 --reps 1 --block $b --route reference > $O/ref_b${b}_p$i.log 2>&1 || { echo "FAILED pmc $b $i" >> $O/status.log; exit 1; }
  done
  timeout -k 10 240 python3 $R/tools/time_embed.py --frames 32 --reps 2 --block $b --route reference >> $O/ref_time.log 2>&1 || { echo "FAILED time $b" >> $O/status.log; exit 1; }
done
for v in main noapp; do
  L=$R/thatsmyface_amd/libtmfwm.so; [ $v = noapp ] && L=$R/variants/libtmfwm_noapp.so
  TMFWM_LIB=$L timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --stats -d $O/app_$v -o p --output-format csv -- \
    python3 $R/tools/time_embed.py --frames 128 --reps 3 --block 16 --kind photo --wm qr > $O/app_$v.log 2>&1 || { echo "FAILED trace $v" >> $O/status.log; exit 1; }
done
echo ok >> $O/status.log
