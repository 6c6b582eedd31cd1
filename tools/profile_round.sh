#!/bin/bash
# Round profile on the GPU box for ONE workload: kernel trace + stats of its bench command, then
# three PMC passes (FETCH_SIZE, WRITE_SIZE, SQ MFMA/wait counters) over the GEMM dispatches, and
# the record for its roofline kernel keyed by workload (append it to profiles/roofline_traffic.json).
# Usage: bash tools/profile_round.sh <out-subdir> <workload key> "<kernel name>" [bench args...]
#   workload keys: config3-full (default args), config3-lora (--trainable lora),
#   config5-full (--config llava-1.5-13b --batch 4 --text-len 1025), config2-vit (--workload vit --batch 64)
set -e
OUT=gpurun_out/${1:-prof}
WL=${2:-config3-full}
KERNEL=${3:-"gemm256_k<1, 1, 1, 256, 256, 0>"}
shift 3 || true
ARGS="--no-sub --no-cpu-baseline $*"
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python bench.py --steps 3 --warmup 1 $ARGS > $OUT/bench_traced.log 2>&1
python tools/prof_summary.py $OUT/trace/run_kernel_trace.csv --top 60 > $OUT/summary.txt
for pass in "FETCH_SIZE:fetch" "WRITE_SIZE:write" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY:sq"; do
  CNT=${pass%%:*}; TAG=${pass##*:}
  timeout -s KILL 300 rocprofv3 --pmc $CNT --kernel-include-regex gemm -d $OUT/pmc_$TAG -o p --output-format csv -- python bench.py --steps 1 --warmup 1 $ARGS > $OUT/pmc_$TAG.log 2>&1
done
# records for the given kernel and for the roofline kernel the traced bench line itself names
RK=$(python -c "import json; l=[x for x in open('$OUT/bench_traced.log') if x.startswith('{')]; print(json.loads(l[-1])['roofline']['kernel'].split(':')[0])")
python tools/pmc_family.py $OUT/pmc_fetch/p_counter_collection.csv $OUT/pmc_write/p_counter_collection.csv $OUT/pmc_sq/p_counter_collection.csv "$KERNEL||$RK" "$WL" > $OUT/roofline_traffic.json
echo done
