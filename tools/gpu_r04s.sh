#!/bin/bash
# LoRA recipe fused / unfused A/B, then the default bench line (with its sub-workloads)
set -o pipefail
OUT=gpurun_out/r04s
mkdir -p $OUT
for f in 1 0 1 0; do
  CULLAVO_LORA_FUSE=$f timeout -k 10 300 python -u bench.py --trainable lora --no-sub --no-cpu-baseline --steps 6 --warmup 2 \
    > $OUT/lora_fuse$f.json 2> $OUT/lora_fuse$f.err || { tail -5 $OUT/lora_fuse$f.err; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/lora_fuse$f.json').read().splitlines()[-1]);print('fuse $f', d['value'], d['ms_per_step'], [(s['shape'],s['kernel'][-7:],s['ms_per_step']) for s in d['gemm_shapes'][:8]])"
done
timeout -k 10 900 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
tail -c 3000 $OUT/bench.json
