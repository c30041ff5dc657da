#!/bin/bash
# Quick GPU loop: a pytest subset (-k EXPR), then bench.py (no oracle leg) under rocprofv3
# kernel stats.  Usage: tools/quick2.sh TAG "EXPR" [bench args...]
set -u
TAG=$1; K=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -s --timeout 200 --timeout-method thread -k "$K" \
    > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python bench.py --no-cpu-baseline "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; head -c 900 "$OUT/bench.json"; echo; tail -3 "$OUT/bench.err"; [ $rc -ne 0 ] && exit $rc
python tools/kstats.py "$OUT/prof/run_kernel_stats.csv" 12
