#!/bin/bash
# Chamfer forward timing + SQ counter passes: tools/pmc_chamfer.sh TAG
set -u
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 120 python tools/bench_chamfer.py > "$OUT/time.json" 2> "$OUT/time.err"
rc=$?; cat "$OUT/time.json"; [ $rc -ne 0 ] && { tail -5 "$OUT/time.err"; exit $rc; }
i=0
for P in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU" \
         "SQ_WAVES SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $P --output-format csv -d "$OUT/p$i" -o pmc -- \
      python tools/bench_chamfer.py --reps 2 > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/p$i.log"; exit $rc; }
done
python tools/pmc_sq.py "$OUT" chamfer_rowmin
