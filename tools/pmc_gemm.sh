#!/bin/bash
# gemm micro-bench timing + counter passes: tools/pmc_gemm.sh TAG [ONLY]
set -u
TAG=$1; ONLY=${2:-}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 120 python tools/bench_gemm.py > "$OUT/time.txt" 2> "$OUT/time.err"
rc=$?; cat "$OUT/time.txt"; [ $rc -ne 0 ] && { tail -5 "$OUT/time.err"; exit $rc; }
i=0
for P in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU" \
         "SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $P --output-format csv -d "$OUT/p$i" -o pmc -- \
      python tools/bench_gemm.py --reps 2 --only "$ONLY" > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/p$i.log"; exit $rc; }
done
for K in gemm_bf_kernel gemm_ex_kernel wgrad_ex_kernel; do echo "== $K"; python tools/pmc_sq.py "$OUT" $K; done
