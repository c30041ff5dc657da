#!/bin/bash
# rocprofv3 kernel trace + stats of the driver's bench window (--steps 20 --warmup 5), keeping the
# per-dispatch trace CSV for timeline analysis (tools/timeline.py).  Usage: tools/r3_prof.sh TAG [bench args]
set -u
TAG=$1; shift; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-encoder --no-other-precision "$@" \
    > "$OUT/pbench.json" 2> "$OUT/pbench.err"
rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/pbench.err"; exit $rc; }
head -c 600 "$OUT/pbench.json"; echo
python tools/kstats.py "$OUT/prof/run_kernel_stats.csv" 25
