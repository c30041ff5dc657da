#!/bin/bash
# Session-3 evidence: r2_prof (kernel stats + PMC of the default bench), the driver-window
# kernel stats, the 32-cloud step and the trainer step.  Usage: tools/s3_prof.sh TAG
set -u
TAG=${1:-s3prof}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
bash tools/r2_prof.sh "$TAG" || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/drv" -o run -- \
    python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-encoder > "$OUT/drv_bench.json" 2> "$OUT/drv_bench.err"
rc=$?; echo "drv prof rc=$rc"; [ $rc -ne 0 ] && exit $rc
python tools/kstats.py "$OUT/drv/run_kernel_stats.csv" 25 > "$OUT/drv_kernel_top.txt"
timeout -k 10 300 python bench.py --clouds-per-gpu 32 --steps 20 --warmup 3 --no-cpu-baseline --no-encoder \
    > "$OUT/b32.json" 2> "$OUT/b32.err"
rc=$?; echo "b32 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/bench_train.py > "$OUT/train.json" 2> "$OUT/train.err"
rc=$?; echo "train rc=$rc"; tail -c 600 "$OUT/train.json"; exit $rc
