#!/bin/bash
# 32 clouds per GPU (BASELINE configs[4]'s per-GPU share): bench + rocprofv3 kernel stats/trace.
set -u
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py --gpus 1 --clouds-per-gpu 32 --steps 20 --warmup 3 --no-cpu-baseline --no-encoder --no-other-precision > "$OUT/bench_b32.json" 2> "$OUT/bench_b32.err" || { tail -3 "$OUT/bench_b32.err"; exit 1; }
python -c "import json;d=json.loads(open('$OUT/bench_b32.json').read().strip().splitlines()[-1]);print('b32', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python bench.py --gpus 1 --clouds-per-gpu 32 --steps 10 --warmup 2 --no-cpu-baseline --no-encoder --no-other-precision > "$OUT/pbench.json" 2> "$OUT/pbench.err" || { tail -3 "$OUT/pbench.err"; exit 1; }
python tools/kstats.py "$OUT/prof/run_kernel_stats.csv" 22
