#!/bin/bash
# time knn3_interp on recorded trajectory inputs for each experiment build
OUT=gpurun_out/$1; mkdir -p gpurun_out
timeout -k 10 200 python tools/knn_replay.py record /tmp/knn_rec.pt > $OUT 2>&1 || exit 1
for so in pointcloud_style_transfer_amd/libpcst_hip.so pointcloud_style_transfer_amd/libpcst_hip_v_*.so; do
  echo "== $so" >> $OUT
  PCST_LIB=$so timeout -k 10 100 python tools/knn_replay.py time /tmp/knn_rec.pt 2>&1 | grep -v amdgpu.ids | tail -2 >> $OUT || exit 1
done
