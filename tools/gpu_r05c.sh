#!/bin/bash
# round-3 4-wave lab kernel (AGPR accumulators, LDS-DMA 4 stages, hand interleave = variant 17) vs
# production vs hipBLASLt: rates, then PMC passes on the same run
set -o pipefail
OUT=gpurun_out/r05c
mkdir -p $OUT
export TMPDIR=/tmp
LIB=tools/lab/bin/libgemm4w.so
timeout -k 10 200 python -u tools/lab/gemm_lab.py --lib $LIB --variants 12,17,19,15 --shapes gate_up,lm_head,qkv --prod > $OUT/rates.txt 2>&1 || { cat $OUT/rates.txt; exit 1; }
cat $OUT/rates.txt
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
i=0
for CNT in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $CNT --kernel-include-regex "gemm|Cijk" -d $OUT/p$i -o p --output-format csv -- python tools/lab/gemm_lab.py --lib $LIB --variants 17,15 --shapes lm_head --prod --rounds 1 --iters 2 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python tools/pmc_dispatch.py $OUT/p1/p_counter_collection.csv $OUT/p2/p_counter_collection.csv > $OUT/pmc.json
cat $OUT/pmc.json
