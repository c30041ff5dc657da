#!/bin/bash
# The driver's bench invocation (--steps 20 --warmup 5) plain and under rocprofv3 kernel stats:
# tools/drv_bench_prof.sh TAG
set -u
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-encoder \
    > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; head -c 400 "$OUT/bench.json"; echo; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-encoder > "$OUT/pbench.json" 2> "$OUT/pbench.err"
rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && exit $rc
python tools/kstats.py "$OUT/prof/run_kernel_stats.csv" 25
