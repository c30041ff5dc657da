set -u
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "knn or upsample or hier or configs" > gpurun_out/knn_t.log 2>&1; rc=$?; tail -2 gpurun_out/knn_t.log; [ $rc -ne 0 ] && exit $rc
bash tools/drv_bench_prof.sh db5 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/full5 -o run -- python bench.py --no-cpu-baseline --no-encoder > gpurun_out/full5.json 2> gpurun_out/full5.err || exit 1
head -c 300 gpurun_out/full5.json; echo
python tools/kstats.py gpurun_out/full5/run_kernel_stats.csv 8
