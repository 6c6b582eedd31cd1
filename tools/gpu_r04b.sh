#!/bin/bash
# ping-pong GEMM (tile modes 12 / 13): parity on every GEMM test shape, race screen, then the
# 7B step shapes against the production plan and hipBLASLt
set -o pipefail
OUT=gpurun_out/r04b
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "tpp4 or tpp5 or pipelined_repeatable" > $OUT/tests.log 2>&1
rc=$?
tail -5 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/gemm_bench.py --modes=-1,12,13 --iters 20 > $OUT/gemm_bench.txt 2>&1
rc=$?
cat $OUT/gemm_bench.txt | cut -c1-250
exit $rc
