#!/bin/bash
# fused LoRA (tests + LoRA-recipe bench fused / unfused), GEMV variants on the decode bench
set -o pipefail
OUT=gpurun_out/r04g
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_lora.py tests/test_generation.py tests/test_capi.py -m gpu -x -q \
  --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "^E |Error|assert" $OUT/tests.log | head -20; exit $rc; }
for f in 1 0 1; do
  CULLAVO_LORA_FUSE=$f timeout -k 10 300 python -u bench.py --trainable lora --no-sub --no-cpu-baseline --steps 6 --warmup 2 \
    > $OUT/lora_fuse$f.json 2> $OUT/lora_fuse$f.err || { tail -5 $OUT/lora_fuse$f.err; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/lora_fuse$f.json').read().splitlines()[-1]);print('fuse $f', d['value'], d['ms_per_step'], [(s['shape'],s['ms_per_step']) for s in d['gemm_shapes'][:6]])"
done
for v in 0 1 2 3; do
  CULLAVO_GEMV=$v timeout -k 10 300 python -u bench.py --workload decode --batch 1 --steps 8 --warmup 1 > $OUT/decode_v$v.json 2> $OUT/decode_v$v.err || { tail -5 $OUT/decode_v$v.err; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/decode_v$v.json').read());print('gemv $v b1', d['ms_per_step'], d['roofline']['achieved'], d['step_roofline']['achieved'])"
done
for v in 1 3; do
  CULLAVO_GEMV=$v timeout -k 10 300 python -u bench.py --workload decode --batch 8 --steps 8 --warmup 1 > $OUT/decode8_v$v.json 2> $OUT/decode8_v$v.err || { tail -5 $OUT/decode8_v$v.err; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/decode8_v$v.json').read());print('gemv $v b8', d['ms_per_step'], d['roofline']['achieved'], d['step_roofline']['achieved'])"
done
