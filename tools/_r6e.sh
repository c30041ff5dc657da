cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r6f
for lib in prod nodense; do
for m in alone beside; do
  L=$PWD/pointcloud_style_transfer_amd/libpcst_hip.so; [ $lib = nodense ] && L=$PWD/pointcloud_style_transfer_amd/libpcst_hip_v_nodense.so
  PCST_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6f/${lib}_$m -o run -- python tools/voxel_probe_knobs.py --reps 20 --modes $m > gpurun_out/r6f/probe_${lib}_$m.log 2>&1 || exit 1
  echo "== $lib $m"; python tools/kstats.py gpurun_out/r6f/${lib}_$m/run_kernel_stats.csv 10
done
done
