#!/bin/bash
# 32x32x16 ping-pong GEMM (tile modes 15 / 16): parity + race screen, then the 7B step shapes
set -o pipefail
OUT=gpurun_out/r04e
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "tpp4x32 or tpp5x32 or pipelined_repeatable" > $OUT/tests.log 2>&1
rc=$?; tail -5 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/gemm_bench.py --modes=-1,15,16,12 --iters 20 > $OUT/gemm_bench.txt 2>&1
rc=$?; grep -v amdgpu.ids $OUT/gemm_bench.txt | sed 's/T=8704 //; s/err [0-9.e+-]*//g' | cut -c1-170; exit $rc
