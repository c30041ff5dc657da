#!/bin/bash
# Build (here) or run (on the box) tools/solo_bench.hip for a set of solo-kernel knob settings.
#   tools/solo_variants.sh build "KD:PRIO:STAMPS[:DMA[:EXP[:NCB]]] ..."   -> tools/nm_bin/solo_<KD>_<PRIO>_<STAMPS>
#   tools/solo_variants.sh run   "KD:PRIO:STAMPS[:DMA[:EXP[:NCB]]] ..."   (GPU; each run under its own time limit)
set -u
MODE=$1
SETS=${2:-"3:0:0"}
OUT=tools/solo_bin
mkdir -p $OUT
for s in $SETS; do
  kd=$(echo $s | cut -d: -f1); pr=$(echo $s | cut -d: -f2); stm=$(echo $s | cut -d: -f3); dma=$(echo $s | cut -s -d: -f4); dma=${dma:-0}; ex=$(echo $s | cut -s -d: -f5); ex=${ex:-0}; ncb=$(echo $s | cut -s -d: -f6); ncb=${ncb:-2}
  bin=$OUT/solo_${kd}_${pr}_${stm}_${dma}_${ex}_${ncb}
  if [ "$MODE" = build ]; then
    /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -mno-amdgpu-ieee -fno-honor-nans \
      -I include -I pointcloud_style_transfer_amd/csrc -DPCST_SOLO_KD=$kd -DPCST_SOLO_PRIO=$pr \
      -DPCST_SOLO_STAMPS=$stm -DPCST_SOLO_DMA=$dma -DPCST_SOLO_EXP=$ex -DPCST_SOLO_NCB=$ncb tools/solo_bench.hip -o $bin || exit 1
  else
    timeout -k 10 60 $bin 40 || exit $?
  fi
done
