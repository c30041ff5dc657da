#!/bin/bash
# Round-3: the 32-cloud kNN build placement probe, the 32-cloud bench, and the tests of the loop
# paths it touches.  Stops at the first failure.  Usage: tools/r3_b32.sh TAG
set -u
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/b32_probe.py --modes seq,hi_nopad,hi_pad,srch > "$OUT/b32_probe.txt" 2>&1
rc=$?; tail -9 "$OUT/b32_probe.txt"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --gpus 1 --clouds-per-gpu 32 --steps 20 --warmup 3 --no-cpu-baseline --no-encoder --no-other-precision > "$OUT/bench_b32.json" 2> "$OUT/bench_b32.err"
rc=$?; echo "b32 bench rc=$rc"; [ $rc -ne 0 ] && { tail -3 "$OUT/bench_b32.err"; exit $rc; }
python -c "import json;d=json.loads(open('$OUT/bench_b32.json').read().strip().splitlines()[-1]);print('b32', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_step.py tests/test_gpu_configs.py -m gpu -x -v \
    --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" "$OUT/pytest.log" | tail -8; exit $rc
