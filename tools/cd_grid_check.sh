#!/bin/bash
# grid-pruned Chamfer: exactness tests, then timings over cloud kinds / both paths
set -u
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "chamfer" > gpurun_out/cg_t.log 2>&1; rc=$?; tail -2 gpurun_out/cg_t.log; [ $rc -ne 0 ] && exit $rc
for args in "--kind gauss --mode 1" "--kind gauss --mode 2" "--kind lidar --noise 0.02 --mode 2" "--kind lidar --noise 0.3 --mode 2" "--kind lidar --noise 3 --mode 2" "--kind lidar --noise 30 --mode 2"; do
  timeout -k 10 120 python tools/bench_chamfer.py $args 2>/dev/null | tail -1 || exit 1
done
