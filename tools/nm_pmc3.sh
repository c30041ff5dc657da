#!/bin/bash
# Two SQ counter passes over one noise-MLP harness binary: tools/nm_pmc3.sh BIN TAG
# (summary: python tools/pmc_sq.py gpurun_out/TAG noise_mlp)
set -u
BIN=$1; TAG=$2; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE \
  --output-format csv -d "$OUT/pa" -o pmc -- $BIN 10 1 > "$OUT/pa.log" 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES \
  SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES \
  --output-format csv -d "$OUT/pb" -o pmc -- $BIN 10 1 > "$OUT/pb.log" 2>&1 || exit $?
