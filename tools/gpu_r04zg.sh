#!/bin/bash
# PMC record of the round-4 attention defaults at the 7B layer (forward stage 7, backward mode 7):
# SQ timing / instruction mix, then FETCH_SIZE and WRITE_SIZE each in a pass of its own
set -o pipefail
OUT=gpurun_out/r04zg
mkdir -p $OUT
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
i=0
for CNT in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CNT --kernel-include-regex attn -d $OUT/p$i -o p --output-format csv -- python tools/attn_one.py 7 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python tools/pmc_kernels.py $(find $OUT/p1 $OUT/p2 $OUT/p3 $OUT/p4 -name "*counter_collection.csv") > $OUT/summary.json
cat $OUT/summary.json
