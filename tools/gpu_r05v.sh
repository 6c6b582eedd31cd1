#!/bin/bash
# LoRA step after the dx fusion: kernel trace + stats, and the PMC passes of the new lora_dx_k
set -o pipefail
OUT=gpurun_out/r05v
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ARGS="--trainable lora --no-sub --no-cpu-baseline"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python bench.py --steps 3 --warmup 1 $ARGS > $OUT/bench_traced.log 2>&1 || { tail -5 $OUT/bench_traced.log; exit 1; }
python tools/prof_summary.py $OUT/trace/run_kernel_trace.csv --top 60 > $OUT/summary.txt || exit 1
for pass in "FETCH_SIZE:fetch" "WRITE_SIZE:write" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY:sq"; do
  CNT=${pass%%:*}; TAG=${pass##*:}
  timeout -s KILL 300 rocprofv3 --pmc $CNT --kernel-include-regex lora_dx -d $OUT/pmc_$TAG -o p --output-format csv -- python bench.py --steps 1 --warmup 1 $ARGS > $OUT/pmc_$TAG.log 2>&1 || { tail -3 $OUT/pmc_$TAG.log; exit 1; }
done
python tools/pmc_family.py $OUT/pmc_fetch/p_counter_collection.csv $OUT/pmc_write/p_counter_collection.csv $OUT/pmc_sq/p_counter_collection.csv "lora_dx_k<" config3-lora > $OUT/lora_dx_pmc.json || exit 1
cat $OUT/lora_dx_pmc.json
head -30 $OUT/summary.txt | cut -c1-160
