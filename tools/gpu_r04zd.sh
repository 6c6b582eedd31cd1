#!/bin/bash
# decode fusions: RMSNorm (row statistics loads now in flight together) / SwiGLU inside the GEMV
set -o pipefail
OUT=gpurun_out/r04zd
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_generation.py > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/tests.log | head -20; exit $rc; }
for rep in 1 2; do
for f in none norm norm,swiglu; do
for b in 1 8; do
  fx=$f; [ $f = none ] && fx=""
  CULLAVO_DECODE_FUSE=$fx timeout -k 10 300 python -u bench.py --workload decode --batch $b --no-sub --no-cpu-baseline > $OUT/decode_${f}_b$b.json 2> $OUT/decode_${f}_b$b.err || { tail -5 $OUT/decode_${f}_b$b.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/decode_${f}_b$b.json').read().strip().splitlines()[-1]);print('$f b$b', d['value'], d['ms_per_step'])"
done; done; done
