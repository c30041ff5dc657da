#!/bin/bash
# Round-3 check of the deferred kNN search: its tests, the step probe A/B, the driver bench,
# then the 32-cloud build placement probe.  Stops at the first failure.  Usage: tools/r3_search.sh TAG
set -u
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_models.py -m gpu -x -v \
    --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" "$OUT/pytest.log" | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/step_probe.py --modes srch,nosrch,noev --reps 5 > "$OUT/step_probe.txt" 2>&1
rc=$?; cat "$OUT/step_probe.txt" | tail -4; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; python -c "import json;d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['frac'])"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/b32_probe.py > "$OUT/b32_probe.txt" 2>&1
rc=$?; tail -12 "$OUT/b32_probe.txt"; exit $rc
