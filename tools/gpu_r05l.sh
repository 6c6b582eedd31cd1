#!/bin/bash
# attention kernels (LM D=128 causal fwd/bwd, ViT D=64 fwd) at the production shapes: timing + PMC
set -o pipefail
OUT=gpurun_out/r05l
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/attn_bench.py > $OUT/attn_bench.txt 2>&1 || { tail -5 $OUT/attn_bench.txt; exit 1; }
cat $OUT/attn_bench.txt
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM"
i=0
for CNT in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CNT --kernel-include-regex "attn" -d $OUT/p$i -o p --output-format csv -- python tools/attn_bench.py > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python tools/pmc_dispatch.py $OUT/p1/p_counter_collection.csv $OUT/p2/p_counter_collection.csv > $OUT/pmc.txt 2>&1
python3 -c "
import json
t=open('$OUT/pmc.txt').read(); d=json.loads(t[t.index('{'):])
keys=['us','eff_clock_ghz','mfma_busy','wait_any_frac','wait_inst_any_frac','active_inst_any_frac','valu_per_mfma','salu_per_mfma','lds_per_mfma','vmem_rd_per_mfma']
for n,v in d.items(): print('%-60s'%n[:60], ' '.join('%s=%.3f'%(k[:10],v.get(k,0)) for k in keys))
"
