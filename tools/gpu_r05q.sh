#!/bin/bash
# decode GEMV: software-pipelined variant (CULLAVO_GEMV_PIPE=1): tests with it on, then decode A/B
set -o pipefail
OUT=gpurun_out/r05q
mkdir -p $OUT
export TMPDIR=/tmp
CULLAVO_GEMV_PIPE=1 timeout -k 10 400 python -u -m pytest tests/test_generation.py tests/test_ops_gpu.py -x -q -k "decode or gemv or generation or linear" --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for b in 1 8; do
  for pp in 1 0; do
    CULLAVO_GEMV_PIPE=$pp timeout -k 10 300 python -u bench.py --workload decode --batch $b --no-sub --no-cpu-baseline --detail-out $OUT/dec_b${b}_pipe$pp.json > $OUT/dec_b${b}_pipe$pp.log 2>&1 || { tail -20 $OUT/dec_b${b}_pipe$pp.log; exit 1; }
    echo "b=$b pipe=$pp"; python -c "import json,sys; d=json.load(open('$OUT/dec_b${b}_pipe$pp.json')); print(d['value'], d['ms_per_step'], d['roofline']['achieved'], d['step_roofline']['frac'])"
  done
done
