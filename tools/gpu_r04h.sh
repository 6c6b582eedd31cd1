#!/bin/bash
# fused LoRA on the 288-row tile + fused decode linears: tests, LoRA bench A/B, decode b1/b8, stream lab
set -o pipefail
OUT=gpurun_out/r04h
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/test_lora.py tests/test_generation.py tests/test_capi.py -m gpu -x -q \
  --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "^E |Error|assert" $OUT/tests.log | head -20; exit $rc; }
for f in 1 0 1 0; do
  CULLAVO_LORA_FUSE=$f timeout -k 10 300 python -u bench.py --trainable lora --no-sub --no-cpu-baseline --steps 6 --warmup 2 \
    > $OUT/lora_fuse$f.json 2> $OUT/lora_fuse$f.err || { tail -5 $OUT/lora_fuse$f.err; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/lora_fuse$f.json').read().splitlines()[-1]);print('fuse $f', d['value'], d['ms_per_step'], [(s['shape'],s['ms_per_step']) for s in d['gemm_shapes'][:7]])"
done
for b in 1 8; do
  timeout -k 10 300 python -u bench.py --workload decode --batch $b --steps 8 --warmup 1 > $OUT/decode_b$b.json 2> $OUT/decode_b$b.err || { tail -5 $OUT/decode_b$b.err; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/decode_b$b.json').read());print('decode b$b', d['ms_per_step'], d['value'], d['roofline']['achieved'], d['step_roofline']['achieved'])"
done
timeout -k 10 120 tools/lab/bin/stream_lab > $OUT/stream_lab.txt 2>&1; cat $OUT/stream_lab.txt
