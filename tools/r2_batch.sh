#!/bin/bash
# configs[4] per-GPU share (32 clouds, eager and graph) and the configs[2] trainer step, with
# kernel stats.  Usage: tools/r2_batch.sh TAG
set -u
TAG=${1:-batch}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py --clouds-per-gpu 32 --steps 50 --warmup 3 --no-cpu-baseline --no-encoder \
    > "$OUT/b32.json" 2> "$OUT/b32.err"
rc=$?; echo "b32 rc=$rc"; head -c 700 "$OUT/b32.json"; echo; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/bench_graph.py > "$OUT/graph.json" 2> "$OUT/graph.err"
rc=$?; echo "graph rc=$rc"; cat "$OUT/graph.json"; [ $rc -ne 0 ] && { tail -5 "$OUT/graph.err"; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/tprof" -o run -- \
    python tools/bench_train.py --steps 5 --warmup 2 > "$OUT/train.json" 2> "$OUT/train.err"
rc=$?; echo "train rc=$rc"; cat "$OUT/train.json"; [ $rc -ne 0 ] && { tail -5 "$OUT/train.err"; exit $rc; }
python tools/kstats.py "$OUT/tprof/run_kernel_stats.csv" 30
