#!/bin/bash
# A/B check on the box: selected GPU tests, then driver-window benches (20 steps from t=999)
# with env settings given as "NAME=VAL,NAME=VAL ..." variants.
# Usage: tools/ab_check.sh TAG "pytest -k expr" "variant1 variant2 ..." [extra bench args]
set -u
TAG=$1; K=$2; VARS=$3; EXTRA=${4:-}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "$K" \
    > "$OUT/pytest.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" "$OUT/pytest.log" | tail -6
  [ $rc -ne 0 ] && exit $rc
fi
i=0
for v in $VARS; do
  i=$((i+1))
  envs=$(echo "$v" | tr ',' ' ')
  [ "$v" = base ] && envs=""
  env $envs timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-encoder $EXTRA \
    > "$OUT/bench_$i.json" 2> "$OUT/bench_$i.err"
  rc=$?; [ $rc -ne 0 ] && { echo "bench $v rc=$rc"; tail -5 "$OUT/bench_$i.err"; exit $rc; }
  python - "$OUT/bench_$i.json" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:40s} {d['value']:9.1f} steps/s  {d['ms_per_step']:.4f} ms/step  mlp {d['roofline']['avg_launch_ms']*1e3:.1f} us  frac {d['roofline']['frac']}")
PY
done
exit 0
