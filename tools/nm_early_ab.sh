#!/bin/bash
# A/B of the noise MLP's weight-part issue order: the product library against
# libpcst_hip_v_late.so (PCST_NM_EARLY=0), driver-window bench, alternating, two passes.
set -u
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
for pass in 1 2; do
  for so in pointcloud_style_transfer_amd/libpcst_hip.so pointcloud_style_transfer_amd/libpcst_hip_v_late.so; do
    n=$(basename "$so" .so)
    PCST_LIB=$so timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-encoder \
        --no-other-precision > "$OUT/$n.$pass.json" 2> "$OUT/$n.$pass.err" || { tail -3 "$OUT/$n.$pass.err"; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])" "$OUT/$n.$pass.json" "$n.$pass"
  done
done
