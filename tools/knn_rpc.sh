#!/bin/bash
# kRefsPerCell variants: driver window (20 steps) and 300 steps, kNN kernel stats per variant
set -u
OUT=gpurun_out/rpc; mkdir -p $OUT; export TMPDIR=/tmp
for so in pointcloud_style_transfer_amd/libpcst_hip.so pointcloud_style_transfer_amd/libpcst_hip_v_*.so; do
  n=$(basename "$so" .so)
  for S in 20 300; do
    PCST_LIB=$so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$n.$S" -o run -- \
        python bench.py --no-cpu-baseline --no-encoder --steps $S --warmup 5 > "$OUT/$n.$S.json" 2> "$OUT/$n.$S.err" || exit 1
    echo "== $n steps=$S $(python -c "import json,sys; print(json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['ms_per_step'])" "$OUT/$n.$S.json")"
    python tools/kstats.py "$OUT/$n.$S/run_kernel_stats.csv" 40 | grep -E "knn_(query|outlier|count)"
  done
done
