#!/bin/bash
# Chamfer row-min S x R variants (PCST_CD_VARIANT), timing then the chamfer tests per variant
set -u
OUT=gpurun_out/cd3; mkdir -p $OUT
for V in ${VARS:-11 21 41 12 22 42 14}; do
  PCST_CD_VARIANT=$V timeout -k 10 120 python tools/bench_chamfer.py > $OUT/v$V.json 2>/dev/null || exit 1
  echo "V=$V $(cat $OUT/v$V.json)"
done
for V in ${TVARS:-22 14}; do
  PCST_CD_VARIANT=$V timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k chamfer > $OUT/pytest$V.log 2>&1; rc=$?; tail -1 $OUT/pytest$V.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
