#!/bin/bash
# Build (here or on the box) and run the noise-MLP timing harness for a set of knob settings.
#   tools/nm_variants.sh build "EXP:NCB ..."   -> gpurun_out/nm/nm_<EXP>_<NCB>
#   tools/nm_variants.sh run   "EXP:NCB ..."   (GPU; each run under its own time limit)
set -u
MODE=$1
SETS=${2:-"0:1"}
OUT=tools/nm_bin
mkdir -p $OUT
for s in $SETS; do
  # SET = EXP:NCB[:PAIRX[:RD[:EPI]]]
  e=$(echo $s | cut -d: -f1); n=$(echo $s | cut -d: -f2); x=$(echo $s | cut -s -d: -f3)
  rd=$(echo $s | cut -s -d: -f4); ep=$(echo $s | cut -s -d: -f5)
  bin=$OUT/nm_${e}_${n}${x:+_x$x}${rd:+_rd$rd}${ep:+_ep$ep}
  extra="-DPCST_NM_EXPERIMENT=$e -DPCST_NM_NCB=$n ${x:+-DPCST_NM_PAIRX=$x} ${rd:+-DPCST_NM_RD=$rd} ${ep:+-DPCST_NM_EPI_GROUP=$ep}"
  # "v0:0" = a saved earlier kernel (tools/_scratch/noise_mlp_v0.hip)
  if [ "$e" = v0 ]; then extra='-DNM_SRC="_scratch/noise_mlp_v0.hip"'; fi
  if [ "$MODE" = build ]; then
    /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -mno-amdgpu-ieee -fno-honor-nans \
      -I include -I pointcloud_style_transfer_amd/csrc \
      $extra tools/nm_variants.hip -o $bin || exit 1
  else
    timeout -k 10 60 $bin 50 1 || exit $?
  fi
done
