#!/bin/bash
# Encoder HBM counters: tools/pmc_enc.sh TAG -> gpurun_out/TAG/pmc_{FETCH_SIZE,WRITE_SIZE} and
# profiles/encoder_traffic.json (tools/pmc_encoder.py).  One counter pass per run; the step's
# single-stream layout (counter passes serialise the queues' dispatches).
set -u
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
PB="tools/bench_knobs.py --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline --no-other-precision --no-extra"
for C in FETCH_SIZE WRITE_SIZE; do
  PCST_KNN_OVERLAP=0 timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_$C" -o pmc -- \
      python $PB > "$OUT/pmc_$C.log" 2>&1
  rc=$?; echo "pmc $C rc=$rc"; if [ $rc -ne 0 ]; then tail -5 "$OUT/pmc_$C.log"; exit $rc; fi
done
python tools/pmc_encoder.py "$OUT" "$OUT/encoder_traffic.json"
