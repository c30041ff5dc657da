#!/bin/bash
# Round-3 final validation: full GPU suite, smoke, the driver's bench command, its rocprof kernel stats,
# and the 32-cloud bench.  Stops at the first failure.  Usage: tools/r3_final.sh TAG
set -u
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" "$OUT/pytest.log" | head; tail -1 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
rc=$?; tail -1 "$OUT/smoke.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -3 "$OUT/bench.err"; exit $rc; }
python -c "import json;d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['avg_launch_ms'])"
bash tools/r3_prof.sh "${TAG}p" | tail -28 || exit 1
timeout -k 10 300 python bench.py --gpus 1 --clouds-per-gpu 32 --steps 20 --warmup 3 --no-cpu-baseline --no-encoder --no-other-precision > "$OUT/bench_b32.json" 2> "$OUT/bench_b32.err"
rc=$?; echo "b32 rc=$rc"; [ $rc -ne 0 ] && exit $rc
python -c "import json;d=json.loads(open('$OUT/bench_b32.json').read().strip().splitlines()[-1]);print('b32', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
