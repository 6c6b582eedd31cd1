#!/bin/bash
# Round-6: PMC of the SwiGLU-backward dX GEMM against the same product plain (tools/swiglu_dx_bench.py),
# two counter passes (tools/attn_pmc.sh's groups), summary by tools/pmc_kernels.py
set -o pipefail
OUT=gpurun_out/${1:-swg_pmc}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
i=0
for CNT in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $CNT --kernel-include-regex "gemm256_k<0, 1" -d $OUT/p$i -o p --output-format csv -- python tools/swiglu_dx_bench.py --rounds 1 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python tools/pmc_kernels.py $(find $OUT/p1 -name "*counter_collection.csv") $(find $OUT/p2 -name "*counter_collection.csv") > $OUT/summary.json
cat $OUT/summary.json
