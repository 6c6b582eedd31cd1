#!/bin/bash
# K-major dX, second look: isolated dX/transpose rates, the LoRA recipe A/B, kernel stats (sync).
set -o pipefail
OUT=gpurun_out/kmajor2
mkdir -p $OUT
timeout -k 10 240 python -u tools/dx_layout_probe.py > $OUT/dx_probe.log 2>&1 || { tail -20 $OUT/dx_probe.log; exit 1; }
cat $OUT/dx_probe.log
for mode in off sync; do
  CULLAVO_KMAJOR=$mode timeout -k 10 300 python -u bench.py --no-cpu-baseline --trainable lora > $OUT/lora_$mode.log 2>&1 || { echo "bench $mode failed"; tail -20 $OUT/lora_$mode.log; exit 1; }
  echo "lora $mode: $(grep -o '"value": [0-9.]*' $OUT/lora_$mode.log) $(grep -o '"ms_per_step": [0-9.]*' $OUT/lora_$mode.log)"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export CULLAVO_KMAJOR=sync
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/traced.log 2>&1 || { tail -20 $OUT/traced.log; exit 1; }
python tools/prof_summary.py $OUT/trace/run_kernel_trace.csv --top 30 > $OUT/summary.txt
head -32 $OUT/summary.txt
