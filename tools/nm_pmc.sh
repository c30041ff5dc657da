#!/bin/bash
# PMC pass over one noise-MLP harness binary (built by tools/nm_variants.sh).
# Usage: tools/nm_pmc.sh BIN TAG
set -u
BIN=$1; TAG=$2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE \
  --output-format csv -d gpurun_out/$TAG -o pmc -- $BIN 10 1
