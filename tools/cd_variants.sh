#!/bin/bash
# Chamfer row-min S x R variants, timing then the chamfer tests per variant.  Each variant is an
# experiment build of the library (Makefile XDEF=-DPCST_X_CD_VARIANT=V, loaded through PCST_LIB);
# build them on the CPU first:  VARS="11 21" tools/cd_variants.sh build
set -u
VARS=${VARS:-11 21 41 12 22 42 14}
if [ "${1:-}" = build ]; then
  for V in $VARS; do
    make -s -C pointcloud_style_transfer_amd/csrc OUT=../libpcst_hip_v_cd$V.so BUILD=build_v_cd$V \
      "XDEF=-DPCST_X_CD_VARIANT=$V" || exit 1
  done
  exit 0
fi
OUT=gpurun_out/cd3; mkdir -p $OUT
for V in $VARS; do
  PCST_LIB=pointcloud_style_transfer_amd/libpcst_hip_v_cd$V.so timeout -k 10 120 python tools/bench_chamfer.py > $OUT/v$V.json 2>/dev/null || exit 1
  echo "V=$V $(cat $OUT/v$V.json)"
done
for V in ${TVARS:-22 14}; do
  PCST_LIB=pointcloud_style_transfer_amd/libpcst_hip_v_cd$V.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k chamfer > $OUT/pytest$V.log 2>&1; rc=$?; tail -1 $OUT/pytest$V.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
