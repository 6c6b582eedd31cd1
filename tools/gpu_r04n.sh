#!/bin/bash
# stage-7 forward / mode-8 backward parity + timing, decode with the 8-load GEMV
set -o pipefail
OUT=gpurun_out/r04n
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_ops_gpu.py tests/test_oob_guard.py tests/test_generation.py -k "attention or attn or gemv or decode or generate" \
  > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/tests.log | head -30; exit $rc; }
ATTN_STAGE_AB=4,7,4,7 timeout -k 10 300 python -u tools/attn_bench.py > $OUT/attn_stage7.txt 2>&1 || { tail -5 $OUT/attn_stage7.txt; exit 1; }
cat $OUT/attn_stage7.txt
for bsz in 1 8; do
  timeout -k 10 300 python -u bench.py --workload decode --batch $bsz --no-cpu-baseline > $OUT/decode_b$bsz.json 2> $OUT/decode_b$bsz.err || { tail -5 $OUT/decode_b$bsz.err; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/decode_b$bsz.json').read().splitlines()[-1]);print('decode b$bsz', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('step_roofline',{}).get('frac'))"
done
