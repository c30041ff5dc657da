#!/bin/bash
# SQ counter passes over the solo noise-MLP kernel (tools/solo_bench.hip build KD:PRIO:STAMPS:DMA,
# the bench launch of 2 x 30000 points only): tools/solo_pmc.sh TAG BIN
set -u
TAG=$1; BIN=$2; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"
P3="SQ_WAVES SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
i=1
for PS in "$P1" "$P2" "$P3"; do
  timeout -s KILL 60 rocprofv3 --pmc $PS --output-format csv -d "$OUT/p$i" -o pmc -- "$BIN" 20 2 3 > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; exit $rc; fi
  i=$((i+1))
done
python tools/pmc_sq.py "$OUT" noise_mlp_solo | tee "$OUT/solo_sq.txt"
