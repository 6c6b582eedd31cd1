#!/bin/bash
# pipelined attention forward (stage 7): bitwise tests against stage 4, then the A/B timing
set -o pipefail
OUT=gpurun_out/r04m
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_ops_gpu.py tests/test_oob_guard.py -k "attention or attn" \
  > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/tests.log | head -20; exit $rc; }
ATTN_STAGE_AB=4,7,4,7 timeout -k 10 300 python -u tools/attn_bench.py > $OUT/attn_stage7.txt 2>&1 || { tail -5 $OUT/attn_stage7.txt; exit 1; }
cat $OUT/attn_stage7.txt
