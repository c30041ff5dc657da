#!/bin/bash
# Trainer step (configs[2]): bench in fp16 and bf16 autocast, then a rocprofv3 kernel-trace/stats
# run of the fp16 bench.  Usage: tools/r3_train.sh TAG
set -u
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for dt in float16 bfloat16; do
  timeout -k 10 300 python tools/bench_train.py --amp-dtype $dt > "$OUT/train_$dt.json" 2> "$OUT/train_$dt.err" || { tail -5 "$OUT/train_$dt.err"; exit 1; }
  tail -1 "$OUT/train_$dt.json" | head -c 700; echo
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python tools/bench_train.py --steps 5 --warmup 2 > "$OUT/ptrain.json" 2> "$OUT/ptrain.err" || { tail -5 "$OUT/ptrain.err"; exit 1; }
python tools/kstats.py "$OUT/prof/run_kernel_stats.csv" 25
