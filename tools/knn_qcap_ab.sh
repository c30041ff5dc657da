#!/bin/bash
# A/B of the kNN query grid cap over all clouds (experiment builds libpcst_hip_v_q*.so, KNN_QUERY_TOTAL)
# on the 32-cloud bench, two alternating passes.
set -u
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
for pass in 1 2; do
  for so in pointcloud_style_transfer_amd/libpcst_hip.so pointcloud_style_transfer_amd/libpcst_hip_v_q*.so; do
    n=$(basename "$so" .so)
    PCST_LIB=$so timeout -k 10 200 python bench.py --gpus 1 --clouds-per-gpu 32 --steps 20 --warmup 3 --no-cpu-baseline \
        --no-encoder --no-other-precision > "$OUT/$n.$pass.json" 2> "$OUT/$n.$pass.err" || { tail -3 "$OUT/$n.$pass.err"; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" "$OUT/$n.$pass.json" "$n.$pass"
  done
done
