#!/bin/bash
# rocprofv3 kernel stats of the driver-window bench under env variants:
#   tools/prof_ab.sh TAG "VAR1 VAR2 ..." [extra bench args]   (VAR = NAME=V,NAME=V or base)
set -u
TAG=$1; VARS=$2; EXTRA=${3:-}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for v in $VARS; do
  i=$((i+1)); envs=$(echo "$v" | tr ',' ' '); [ "$v" = base ] && envs=""
  for e in $envs; do export "$e"; done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$i" -o run -- \
    python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-encoder $EXTRA > "$OUT/pbench_$i.json" 2> "$OUT/pbench_$i.err"
  rc=$?; echo "== $v prof rc=$rc"; [ $rc -ne 0 ] && exit $rc
  for e in $envs; do unset "${e%%=*}"; done
  python tools/kstats.py "$OUT/prof_$i/run_kernel_stats.csv" 14
done
exit 0
