#!/bin/bash
# LoRA tiles staged under the last K-tile: LoRA tests + recipe A/B
set -o pipefail
OUT=gpurun_out/r04j
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_lora.py tests/test_capi.py -m gpu -x -q --timeout 200 \
  --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "^E " $OUT/tests.log | head; exit $rc; }
for f in 1 0 1 0; do
  CULLAVO_LORA_FUSE=$f timeout -k 10 300 python -u bench.py --trainable lora --no-sub --no-cpu-baseline --steps 6 --warmup 2 \
    > $OUT/lora_fuse$f.json 2> $OUT/lora_fuse$f.err || { tail -5 $OUT/lora_fuse$f.err; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/lora_fuse$f.json').read().splitlines()[-1]);print('fuse $f', d['value'], d['ms_per_step'], [(s['shape'],s['ms_per_step']) for s in d['gemm_shapes'][:7]])"
done
