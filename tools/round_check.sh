#!/bin/bash
# GPU-box round check: pytest -m gpu, bench (with cpu_baseline), rocprofv3 kernel-trace
# stats of the same bench, and FETCH_SIZE / WRITE_SIZE PMC passes (one counter group per
# run, as MI355X_MICROARCH.md prescribes).  Stops at the first crash or timeout.
# Usage: tools/round_check.sh TAG [--no-tests]
set -u
TAG=${1:-run}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${1:-}" != "--no-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      > "$OUT/pytest.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"
  [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; tail -1 "$OUT/bench.json"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python bench.py --no-cpu-baseline > "$OUT/bench_prof.json" 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && exit $rc
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_$C" -o pmc -- \
      python bench.py --steps 30 --no-cpu-baseline > "$OUT/pmc_$C.log" 2>&1
  rc=$?; echo "pmc $C rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
