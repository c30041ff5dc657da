#!/bin/bash
# Experiment loop (GPU box): the bench under rocprofv3 kernel stats for the product library
# and every experiment build pointcloud_style_transfer_amd/libpcst_hip_v_*.so (PCST_LIB).
# Usage: tools/lib_variants.sh TAG "kstats substring regex" [bench args]
set -u
TAG=$1; PAT=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
for so in pointcloud_style_transfer_amd/libpcst_hip.so pointcloud_style_transfer_amd/libpcst_hip_v_*.so; do
  n=$(basename "$so" .so)
  PCST_LIB=$so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$n" -o run -- \
      python bench.py --no-cpu-baseline "$@" > "$OUT/$n.json" 2> "$OUT/$n.err" || exit 1
  echo "== $n $(python -c "import json,sys; print(json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['value'])" "$OUT/$n.json")"
  python tools/kstats.py "$OUT/$n/run_kernel_stats.csv" 40 | grep -E "$PAT"
done
