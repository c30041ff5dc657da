#!/bin/bash
# A/B of noise-MLP harness binaries (tools/nm_variants.sh build), precision 2 (16x16x32 pair
# kernel), alternating, at 2 clouds (60000 points, the bench launch) and 64 clouds (32-cloud
# batch), then (optional) the noise-MLP GPU tests.  Usage: tools/nm_ab.sh TAG "bin1 bin2 ..." [tests]
set -u
TAG=$1; BINS=$2; T=${3:-}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in 1 2 3; do
  for b in $BINS; do
    echo -n "$b c2: "; timeout -k 10 60 tools/nm_bin/$b 100 2 2 || exit $?
  done
done
for b in $BINS; do
  echo -n "$b c64: "; timeout -k 10 60 tools/nm_bin/$b 5 2 64 || exit $?
done
if [ -n "$T" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -v -s --timeout 200 --timeout-method thread \
    -k "$T" > "$OUT/pytest.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|PASSED|FAILED|bf16 \(code|50-step" "$OUT/pytest.log" | tail -20
  exit $rc
fi
