#!/bin/bash
# A/B of experiment library builds on the driver's bench command (alternating, 2 passes):
#   tools/ab_lib.sh TAG "prod vc512 ..." [extra bench args]   (prod = the product library)
set -u
TAG=$1; LIBS=$2; shift; shift; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for rep in 1 2; do
  for L in $LIBS; do
    if [ "$L" = prod ]; then unset PCST_LIB; else export PCST_LIB=pointcloud_style_transfer_amd/libpcst_hip_v_$L.so; fi
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-encoder --no-other-precision "$@" > "$OUT/$L.$rep.json" 2> "$OUT/$L.$rep.err" || { tail -3 "$OUT/$L.$rep.err"; exit 1; }
    python -c "import json;d=json.loads(open('$OUT/$L.$rep.json').read().strip().splitlines()[-1]);print('$L', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
  done
done
unset PCST_LIB
