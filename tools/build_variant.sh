#!/bin/bash
# Build an experimental library variant: tools/build_variant.sh <name> [extra hipcc flags...]
# -> ab/libtmfwm_<name>.so (git-ignored; travels to the GPU box; load it with TMFWM_LIB).
# The kernel TUs take the extra flags; with FALLBACK=1 in the environment the dgesdd-route
# TU (tmfwm_fallback.hip) is recompiled with them too, otherwise the ABI / tile / QR /
# dgesdd-route objects are the main build's (make -C thatsmyface_amd/csrc first).
# E8SCHED=<strategy> overrides the machine scheduler of the embed<8> TU (default max-ilp).
# SRC_SED='<sed script>' compiles the kernel TUs from a copy of the sources edited by that
# script (e.g. SRC_SED='s/kPowerIters = 6/kPowerIters = 4/'): experiments without switches
# in the product code.  SRC_REV=<git revision> compiles the kernel TUs of that revision
# instead (e.g. the build before a change, for an A/B on one box).  SRC_DIR=<dir> compiles the
# kernel TUs from a copy of the csrc tree kept elsewhere (e.g. a git worktree with an
# experimental edit).  NOMAKE=1 skips the main build's make (its objects are linked as they are).
set -euo pipefail
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/thatsmyface_amd/csrc
[ "${NOMAKE:-0}" = "1" ] || make -s -C "$C" >/dev/null
T=$(mktemp -d)
K=$C
if [ -n "${SRC_DIR:-}" ]; then
  K=$T/thatsmyface_amd/csrc
  mkdir -p "$K" "$T/include"
  cp "$SRC_DIR"/thatsmyface_amd/csrc/*.h "$SRC_DIR"/thatsmyface_amd/csrc/*.hip "$K"/
  cp "$SRC_DIR"/include/*.h "$T/include/"
elif [ -n "${SRC_REV:-}" ]; then
  git -C "$ROOT" archive "$SRC_REV" thatsmyface_amd/csrc include | tar -x -C "$T"
  K=$T/thatsmyface_amd/csrc
elif [ -n "${SRC_SED:-}" ]; then
  K=$T/thatsmyface_amd/csrc  # the tree's layout: tmfwm_internal.h includes ../../include/tmfwm.h
  mkdir -p "$K" "$T/include"
  cp "$C"/*.h "$C"/*.hip "$K"/
  cp "$ROOT"/include/*.h "$T/include/"
  sed -i "$SRC_SED" "$K"/*.h "$K"/*.hip
fi
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fno-slp-vectorize -Wall $*"
/opt/rocm/bin/hipcc $F -c "$K/tmfwm_kernels.hip" -o "$T/k.o" &
/opt/rocm/bin/hipcc $F -mllvm -amdgpu-sched-strategy=${E8SCHED:-max-ilp} -c "$K/tmfwm_embed8.hip" -o "$T/e8.o" &
/opt/rocm/bin/hipcc $F -c "$K/tmfwm_rank1.hip" -o "$T/r1.o" &
R1L=
if [ -f "$K/tmfwm_rank1_lists.hip" ]; then  # (before round 6's last builds: in tmfwm_rank1.hip)
  R1L="$T/r1l.o"
  /opt/rocm/bin/hipcc $F -c "$K/tmfwm_rank1_lists.hip" -o "$T/r1l.o" &
fi
FB="$C/tmfwm_fallback.o $C/tmfwm_fixup4.o $C/tmfwm_fixup6.o $C/tmfwm_fixup8.o $C/tmfwm_fixup10.o $C/tmfwm_fixup12.o $C/tmfwm_fixup14.o $C/tmfwm_fixup16.o"
if [ "${FALLBACK:-0}" = "1" ]; then
  FB="$T/fb.o"
  /opt/rocm/bin/hipcc $F -c "$K/tmfwm_fallback.hip" -o "$T/fb.o" &
  for b in 4 6 8 10 12 14 16; do
    /opt/rocm/bin/hipcc $F -c "$K/tmfwm_fixup$b.hip" -o "$T/fx$b.o" &
    FB="$FB $T/fx$b.o"
  done
fi
wait
mkdir -p "$ROOT/ab"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/ab/libtmfwm_$NAME.so" "$T/k.o" "$T/e8.o" "$T/r1.o" $R1L \
    "$C/tmfwm_capi.o" "$C/tmfwm_multi.o" "$C/tmfwm_qr.o" "$C/tmfwm_tile.o" "$C/tmfwm_pixels.o" $FB -fopenmp -ldl -lpthread
rm -rf "$T"
echo "ab/libtmfwm_$NAME.so"
