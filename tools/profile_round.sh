#!/bin/bash
# Round profile on the GPU box: kernel trace + stats of the bench command, then three PMC passes
# (FETCH_SIZE, WRITE_SIZE, SQ MFMA/wait counters) over the roofline kernel's dispatches.
# Usage: bash tools/profile_round.sh <out-subdir> ["<kernel name>"]   (outputs under gpurun_out/)
set -e
OUT=gpurun_out/${1:-prof}
KERNEL=${2:-"gemm256_k<1, 1, 1, 256, 256, 0>"}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_traced.log 2>&1
python tools/prof_summary.py $OUT/trace/run_kernel_trace.csv --top 60 > $OUT/summary.txt
for pass in "FETCH_SIZE:fetch" "WRITE_SIZE:write" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY:sq"; do
  CNT=${pass%%:*}; TAG=${pass##*:}
  timeout -k 10 300 rocprofv3 --pmc $CNT --kernel-include-regex gemm256 -d $OUT/pmc_$TAG -o p --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/pmc_$TAG.log 2>&1
done
python tools/pmc_family.py $OUT/pmc_fetch/p_counter_collection.csv $OUT/pmc_write/p_counter_collection.csv $OUT/pmc_sq/p_counter_collection.csv "$KERNEL" > $OUT/roofline_traffic.json
echo done
