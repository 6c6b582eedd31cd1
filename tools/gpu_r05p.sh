#!/bin/bash
# decode: RMSNorm in the tail of o_proj / down_proj (cullavo_decode_linear_norm): generation tests, then pnorm on/off
set -o pipefail
OUT=gpurun_out/r05p
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_generation.py -x -q --timeout 200 --timeout-method thread > $OUT/gen_tests.log 2>&1
rc=$?; tail -3 $OUT/gen_tests.log; [ $rc -eq 0 ] || exit $rc
for b in 1 4 8; do
  for f in "gu,rope,pnorm" "gu,rope"; do
    CULLAVO_DECODE_FUSE=$f timeout -k 10 300 python -u bench.py --workload decode --batch $b --no-sub --no-cpu-baseline --detail-out $OUT/dec_b${b}_$f.json > $OUT/dec_b${b}_$f.log 2>&1 || { tail -20 $OUT/dec_b${b}_$f.log; exit 1; }
    echo "b=$b fuse=$f"; python -c "import json,sys; d=json.load(open('$OUT/dec_b${b}_$f.json')); print(d['value'], d['ms_per_step'], d.get('step_roofline'))"
  done
done
