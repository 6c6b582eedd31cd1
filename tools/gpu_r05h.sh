#!/bin/bash
# PMC passes over the 4-wave GEMM lab variants and hipBLASLt (gate|up forward, same process)
set -o pipefail
OUT=gpurun_out/r05h
mkdir -p $OUT
export TMPDIR=/tmp
V=${V:-0,128,1000}
CMD="python tools/lab/gemm_lab.py --lib tools/lab/bin/libgemm4w_lab.so --variants $V --shapes gate_up --rounds 1 --iters 3"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM"
i=0
for CNT in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CNT --kernel-include-regex "gemm4|Cijk" -d $OUT/p$i -o p --output-format csv -- $CMD > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python tools/pmc_dispatch.py $OUT/p1/p_counter_collection.csv $OUT/p2/p_counter_collection.csv > $OUT/pmc.txt 2>&1
cat $OUT/pmc.txt
