#!/bin/bash
# Kernel traces of the driver's bench invocation and of tools/step_probe.py (bench layout) on one
# box, for a per-step gap comparison (tools/timeline.py).  Usage: tools/s2_trace.sh TAG
set -u
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/bench" -o run -- \
    python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-encoder --no-other-precision \
    > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/probe" -o run -- \
    python tools/step_probe.py --reps 1 --modes bench > "$OUT/probe.txt" 2> "$OUT/probe.err" || exit 1
cat "$OUT/probe.txt"; head -c 300 "$OUT/bench.json"
