#!/bin/bash
# PMC of the 4-wave GEMM (tile mode 4) vs the 8-wave default vs hipBLASLt on the big forward shapes
set -o pipefail
OUT=gpurun_out/r05f
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--modes=-1,4 --rounds 1 --reps 3 fwd:8704:22016:4096 fwd:8704:32064:4096"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
P3="FETCH_SIZE GRBM_GUI_ACTIVE"
P4="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
i=0
for CNT in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CNT --kernel-include-regex "gemm|Cijk" -d $OUT/p$i -o p --output-format csv -- python tools/gemm_vs_lib.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python tools/pmc_dispatch.py $OUT/p1/p_counter_collection.csv $OUT/p2/p_counter_collection.csv $OUT/p3/p_counter_collection.csv $OUT/p4/p_counter_collection.csv > $OUT/pmc.json
cat $OUT/pmc.json
