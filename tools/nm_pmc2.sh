#!/bin/bash
# Two SQ counter passes over the bench's noise MLP (30 steps, no encoder / oracle legs).
set -u
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv \
    -d "$OUT/a" -o pmc -- python bench.py --steps 30 --no-cpu-baseline --no-encoder > "$OUT/a.log" 2>&1
rc=$?; echo "pass a rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES \
    SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES --output-format csv \
    -d "$OUT/b" -o pmc -- python bench.py --steps 30 --no-cpu-baseline --no-encoder > "$OUT/b.log" 2>&1
rc=$?; echo "pass b rc=$rc"; exit $rc
