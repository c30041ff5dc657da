#!/bin/bash
# SQ counter passes over the driver-window bench for one kernel family:
# tools/pmc_bench_kernel.sh TAG SUBSTR
set -u
TAG=$1; SUB=$2; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
i=0
for P in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU" \
         "SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$OUT/p$i" -o pmc -- \
      python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-encoder > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/p$i.log"; exit $rc; }
done
python tools/pmc_sq.py "$OUT" "$SUB"
