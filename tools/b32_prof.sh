#!/bin/bash
# Kernel stats of the configs[4] per-GPU share (32 clouds, eager), current tree.  Usage: tools/b32_prof.sh TAG
set -u
TAG=${1:-b32}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py --clouds-per-gpu 32 --steps 20 --warmup 3 --no-cpu-baseline --no-encoder \
    > "$OUT/b32.json" 2> "$OUT/b32.err"
rc=$?; echo "b32 rc=$rc"; head -c 400 "$OUT/b32.json"; echo; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python bench.py --clouds-per-gpu 32 --steps 20 --warmup 3 --no-cpu-baseline --no-encoder \
    > "$OUT/b32_prof.json" 2> "$OUT/b32_prof.err"
rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && exit $rc
python tools/kstats.py "$OUT/prof/run_kernel_stats.csv" 25
