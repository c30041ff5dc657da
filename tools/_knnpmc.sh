# SQ counters of the kNN query / outlier kernels over the driver's window (single-stream layout)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && OUT=gpurun_out/$1 && mkdir -p $OUT
PB="tools/bench_knobs.py --gpus 1 --steps 10 --warmup 2 --no-cpu-baseline --no-encoder --no-other-precision --no-extra"
PCST_KNN_OVERLAP=0 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU \
    SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/p1 -o pmc -- \
    python $PB > $OUT/p1.log 2>&1 || { echo "p1 failed"; tail -5 $OUT/p1.log; exit 1; }
PCST_KNN_OVERLAP=0 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_ANY \
    SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS --output-format csv -d $OUT/p2 -o pmc -- \
    python $PB > $OUT/p2.log 2>&1 || { echo "p2 failed"; tail -5 $OUT/p2.log; exit 1; }
for k in "knn_query_kernel<3, true>" knn_outlier_brick noise_mlp_solo voxf_reps voxf_insert voxf_emit; do
  echo "== $k"; python tools/pmc_sq.py $OUT "$k"
done | tee $OUT/knn_sq.txt
