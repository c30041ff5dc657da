#!/bin/bash
# GPU-box check: pytest -m gpu, then a rocprofv3 kernel-trace profile of the default bench.
# Stops at the first crash/timeout (exit >= 124 or signal); plain test failures (exit 1)
# still let the profile run.  Usage: tools/gpu_check.sh TAG [pytest-args...]
set -u
TAG=${1:-run}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 700 python -m pytest tests -m gpu -q "$@" > "$OUT/pytest.log" 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python bench.py --steps 1000 --warmup 3 --no-cpu-baseline > "$OUT/bench.log" 2>&1
rc2=$?
echo "bench rc=$rc2"; tail -1 "$OUT/bench.log"
exit $(( rc2 != 0 ? rc2 : rc ))
