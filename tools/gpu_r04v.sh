#!/bin/bash
set -o pipefail
OUT=gpurun_out/r04v
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_generation.py tests/test_ops_gpu.py -k "rope or rmsnorm or decode or generate or gemv" > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/tests.log | head -20; exit $rc; }
for bsz in 1 8 1 8; do
  timeout -k 10 300 python -u bench.py --workload decode --batch $bsz --no-cpu-baseline > $OUT/decode_b$bsz.json 2> $OUT/decode_b$bsz.err || { tail -5 $OUT/decode_b$bsz.err; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/decode_b$bsz.json').read().splitlines()[-1]);print('decode b$bsz', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic'], d.get('step_roofline',{}).get('frac'))"
done
