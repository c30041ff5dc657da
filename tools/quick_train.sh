#!/bin/bash
# Quick GPU loop for the training path: a pytest subset (-k EXPR), then the configs[2] trainer
# step under rocprofv3 kernel stats.  Usage: tools/quick_train.sh TAG "EXPR"
set -u
TAG=$1; K=$2
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -s --timeout 200 --timeout-method thread -k "$K" \
    > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/tprof" -o run -- \
    python tools/bench_train.py --steps 5 --warmup 2 > "$OUT/train.json" 2> "$OUT/train.err"
rc=$?; echo "train rc=$rc"; cat "$OUT/train.json"; [ $rc -ne 0 ] && { tail -5 "$OUT/train.err"; exit $rc; }
python tools/kstats.py "$OUT/tprof/run_kernel_stats.csv" 30
