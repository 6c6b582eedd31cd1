#!/bin/bash
# dK/dV kernel with asm-pipelined fragment reads (bwd stage bit 0): attention parity tests, then A/B
set -o pipefail
OUT=gpurun_out/r05n
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_oob_guard.py -x -q -k "attn or attention" --timeout 200 --timeout-method thread > $OUT/attn_tests.log 2>&1
rc=$?; tail -3 $OUT/attn_tests.log; [ $rc -eq 0 ] || exit $rc
ATTN_STAGE_AB=7,17,7,17,37,37 timeout -k 10 300 python -u tools/attn_bench.py > $OUT/attn_ab.txt 2>&1 || { tail -5 $OUT/attn_ab.txt; exit 1; }
cat $OUT/attn_ab.txt
