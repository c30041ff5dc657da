#!/bin/bash
# Profiles of the bench command: kernel-trace stats, FETCH/WRITE PMC passes (noise-MLP and
# encoder traffic), SQ counters of the noise MLP.  Each pass under its own time limit; stops at
# the first failure.  Usage: tools/r2_prof.sh TAG
set -u
TAG=${1:-prof}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python bench.py --no-cpu-baseline > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err"
rc=$?; echo "stats rc=$rc"; [ $rc -ne 0 ] && exit $rc
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_$C" -o pmc -- \
      python bench.py --steps 30 --no-cpu-baseline > "$OUT/pmc_$C.log" 2>&1
  rc=$?; echo "pmc $C rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv \
    -d "$OUT/pmc_sq" -o pmc -- python bench.py --steps 30 --no-cpu-baseline --no-encoder \
    > "$OUT/pmc_sq.log" 2>&1
rc=$?; echo "pmc sq rc=$rc"; [ $rc -ne 0 ] && exit $rc
python tools/pmc_summary.py "$OUT" noise_mlp --json "$OUT/noise_mlp_traffic.json" > "$OUT/pmc_summary.txt"
python tools/pmc_encoder.py "$OUT" "$OUT/encoder_traffic.json"
python tools/kstats.py "$OUT/prof/run_kernel_stats.csv" 25 > "$OUT/kernel_top.txt"; cat "$OUT/kernel_top.txt"
exit 0
