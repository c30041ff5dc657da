#!/bin/bash
# 32x32x16 (code 1) vs 16x16x32 (code 2) bf16 noise-MLP kernels: harness timing (60000 points,
# then 32 clouds), alternating, then the noise-MLP GPU tests.  Usage: tools/nm16_check.sh TAG
set -u
TAG=${1:-nm16}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
B=tools/nm_bin/nm_0_1
for rep in 1 2 3; do
  for prec in 1 2; do
    timeout -k 10 60 $B 100 $prec 2 >> "$OUT/harness.txt" || exit $?
  done
done
for prec in 1 2; do
  timeout -k 10 60 $B 5 $prec 64 >> "$OUT/harness.txt" || exit $?
done
cat "$OUT/harness.txt"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread \
  -k "noise_mlp" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|bf16 \(code" "$OUT/pytest.log" | tail -8
exit $rc
