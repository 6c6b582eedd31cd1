#!/bin/bash
# full GPU suite at this head, smoke(), then the LoRA recipe fused / unfused A/B
set -o pipefail
OUT=gpurun_out/r04o
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $OUT/gpu_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
for f in 1 0 1 0; do
  CULLAVO_LORA_FUSE=$f timeout -k 10 300 python -u bench.py --trainable lora --no-sub --no-cpu-baseline --steps 6 --warmup 2 \
    > $OUT/lora_fuse$f.json 2> $OUT/lora_fuse$f.err || { tail -5 $OUT/lora_fuse$f.err; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/lora_fuse$f.json').read().splitlines()[-1]);print('fuse $f', d['value'], d['ms_per_step'], [(s['shape'],s['kernel'][-8:],s['ms_per_step']) for s in d['gemm_shapes'][:8]])"
done
