#!/bin/bash
# Round-3 check of the MLP-side wait: its tests, the loop tests, step probe A/B (mw vs noev), bench.
set -u
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_step.py -m gpu -x -v -k "then_wait or mlp_waits" \
    --timeout 120 --timeout-method thread > "$OUT/pytest_mw.log" 2>&1
rc=$?; echo "pytest mw rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" "$OUT/pytest_mw.log" | tail -6; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_models.py tests/test_gpu_pipeline.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/step_probe.py --modes mw,noev --reps 9 > "$OUT/step_probe.txt" 2>&1
rc=$?; tail -3 "$OUT/step_probe.txt"; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-encoder > "$OUT/bench$i.json" 2> "$OUT/bench$i.err"
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
python -c "import json;d=json.loads(open('$OUT/bench$i.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['avg_launch_ms'])"
done
