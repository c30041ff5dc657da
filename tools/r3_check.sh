#!/bin/bash
# Round-3 GPU check: pytest -m gpu (optionally -k EXPR), then the driver's bench command.
# Stops at the first failure / crash / timeout.  Usage: tools/r3_check.sh TAG [pytest -k EXPR] [--no-bench]
set -u
TAG=${1:-run}; K=${2:-}; NB=${3:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
timeout -k 10 1000 python -u -m pytest tests -m gpu --maxfail=${MAXFAIL:-5} -v -s --timeout 400 --timeout-method thread \
    "${KA[@]}" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR" "$OUT/pytest.log" | tail -60; tail -4 "$OUT/pytest.log"
[ $rc -ne 0 ] && exit $rc
[ "$NB" = "--no-bench" ] && exit 0
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; tail -c 4000 "$OUT/bench.json"; [ $rc -ne 0 ] && { tail -5 "$OUT/bench.err"; exit $rc; }
exit 0
