#!/bin/bash
# stripped library + 4-wave GEMM (tile mode 4): the GPU suite, then rates against the 8-wave
# default and hipBLASLt (same process, same operands, outputs compared)
set -o pipefail
OUT=gpurun_out/r05e
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/gpu_tests.log | head -20; exit $rc; }
timeout -k 10 200 python -u tools/gemm_vs_lib.py --modes=-1,4 fwd:8704:22016:4096 fwd:8704:32064:4096 fwd:8704:12288:4096 fwd:8704:4096:4096 fwd:8704:4096:11008 dx:8704:4096:11008 dx:8704:22016:4096 dw:22016:4096:8704 dw:4096:11008:8704 > $OUT/rates.txt 2>&1; rc=$?
cat $OUT/rates.txt; exit $rc
