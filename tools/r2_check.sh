#!/bin/bash
# Round-2 GPU check: determinism probe, pytest -m gpu, the default bench (with the oracle leg).
# Stops at the first failure / crash / timeout.  Usage: tools/r2_check.sh TAG [pytest -k EXPR]
set -u
TAG=${1:-run}; K=${2:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 180 python -u tools/determinism_probe.py > "$OUT/probe.json" 2> "$OUT/probe.err"
rc=$?; echo "probe rc=$rc"; tail -2 "$OUT/probe.json"; [ $rc -ne 0 ] && { tail -5 "$OUT/probe.err"; exit $rc; }
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
timeout -k 10 1100 python -u -m pytest tests -m gpu ${PYX:--x} -v -s --timeout 240 --timeout-method thread \
    "${KA[@]}" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; tail -c 3000 "$OUT/bench.json"; [ $rc -ne 0 ] && { tail -5 "$OUT/bench.err"; exit $rc; }
exit 0
