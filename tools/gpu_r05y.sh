#!/bin/bash
# LoRA step: split-K target sweep of the adapters' skinny products (CULLAVO_SPLITK_TARGET)
set -o pipefail
OUT=gpurun_out/r05y
mkdir -p $OUT
export TMPDIR=/tmp
for t in 512 1024 768 256 512; do
  CULLAVO_SPLITK_TARGET=$t timeout -k 10 400 python -u bench.py --trainable lora --no-sub --no-cpu-baseline --detail-out $OUT/lora_sk$t.json > $OUT/lora_sk$t.log 2>&1 || { tail -20 $OUT/lora_sk$t.log; exit 1; }
  echo "target=$t"; python -c "import json; d=json.load(open('$OUT/lora_sk$t.json')); print(d['value'], d['ms_per_step'])"
done
