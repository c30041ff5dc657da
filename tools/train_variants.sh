#!/bin/bash
# Trainer A/B (GPU box): tools/bench_train.py for the product library and every experiment build
# pointcloud_style_transfer_amd/libpcst_hip_v_*.so (PCST_LIB), twice in alternation, then one
# rocprofv3 kernel-stats pass each.  Usage: tools/train_variants.sh TAG "kstats regex"
set -u
TAG=$1; PAT=$2
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
for rep in 1 2; do
  for so in pointcloud_style_transfer_amd/libpcst_hip.so pointcloud_style_transfer_amd/libpcst_hip_v_*.so; do
    n=$(basename "$so" .so)
    PCST_LIB=$so timeout -k 10 300 python tools/bench_train.py > "$OUT/$n.$rep.json" 2> "$OUT/$n.$rep.err" || { tail -5 "$OUT/$n.$rep.err"; exit 1; }
    echo "== $n rep $rep $(python -c "import json,sys; print(json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['ms_per_step'])" "$OUT/$n.$rep.json") ms/step"
  done
done
for so in pointcloud_style_transfer_amd/libpcst_hip.so pointcloud_style_transfer_amd/libpcst_hip_v_*.so; do
  n=$(basename "$so" .so)
  PCST_LIB=$so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$n" -o run -- \
      python tools/bench_train.py --steps 5 --warmup 2 > "$OUT/$n.prof.json" 2> "$OUT/$n.prof.err" || exit 1
  echo "== $n"; python tools/kstats.py "$OUT/$n/run_kernel_stats.csv" 40 | grep -E "$PAT"
done
