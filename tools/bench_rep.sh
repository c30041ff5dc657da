#!/bin/bash
# The driver's bench command N times back to back (no oracle leg): tools/bench_rep.sh TAG [N] [extra args]
set -u
TAG=$1; N=${2:-3}; shift; shift || true; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for i in $(seq $N); do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-encoder --no-other-precision "$@" > "$OUT/b$i.json" 2> "$OUT/b$i.err" || { tail -3 "$OUT/b$i.err"; exit 1; }
  python -c "import json,sys;d=json.loads(open('$OUT/b$i.json').read().strip().splitlines()[-1]);print('run $i', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
done
