#!/bin/bash
# fused decode linears (RMSNorm statistics after the first weight batch): micro-bench + decode step
set -o pipefail
OUT=gpurun_out/r04i
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_generation.py -m gpu -x -q -k "decode_linear or graph" --timeout 200 \
  --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "^E " $OUT/tests.log | head; exit $rc; }
for b in 1 8; do
  timeout -k 10 120 python -u tools/decode_linear_bench.py --batch $b 2>&1 | grep -v amdgpu.ids | tee -a $OUT/decode_linear_bench.txt
done
timeout -k 10 300 python -u bench.py --workload decode --batch 1 --steps 8 --warmup 1 > $OUT/decode_b1.json 2> $OUT/decode_b1.err || exit 1
python -c "import json;d=json.loads(open('$OUT/decode_b1.json').read());print('decode b1', d['ms_per_step'], d['value'], d['roofline']['achieved'], d['step_roofline']['achieved'])"
