#!/bin/bash
# Kernel traces of tools/step_probe.py in the seq and noev layouts (gap analysis).
set -u
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for m in ${MODES:-seq noev}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$m" -o run -- \
      python tools/step_probe.py --reps 1 --modes $m > "$OUT/$m.txt" 2> "$OUT/$m.err" || exit 1
  cat "$OUT/$m.txt"
done
