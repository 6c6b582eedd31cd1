#!/bin/bash
# Split-K plan A/B for the small-grid LoRA GEMMs: the dropout-GEMM bench per target, then the
# LoRA-recipe step at the default and the best alternative, alternating.
set -o pipefail
OUT=gpurun_out/splitk
mkdir -p $OUT
for t in 512 1024 2048 256 512; do
  echo "target $t" >> $OUT/lora_drop.txt
  CULLAVO_SPLITK_TARGET=$t timeout -k 10 120 python tools/lora_drop_bench.py >> $OUT/lora_drop.txt 2>&1 || exit 1
done
cat $OUT/lora_drop.txt
for i in 1 2; do
  timeout -k 10 300 python bench.py --trainable lora --no-cpu-baseline > $OUT/bench_512_$i.txt 2>&1 || exit 2
  CULLAVO_SPLITK_TARGET=1024 timeout -k 10 300 python bench.py --trainable lora --no-cpu-baseline > $OUT/bench_1024_$i.txt 2>&1 || exit 3
done
for f in $OUT/bench_*.txt; do echo $f $(tail -1 $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"); done
