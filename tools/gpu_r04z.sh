#!/bin/bash
set -o pipefail
OUT=gpurun_out/r04z
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_ops_gpu.py tests/test_oob_guard.py tests/test_full_size.py tests/test_model_gpu.py -k "attention or attn or decoder_layer or golden or forward" > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/tests.log | head -20; exit $rc; }
ATTN_STAGE_AB=4,7,4,7 timeout -k 10 300 python -u tools/attn_bench.py > $OUT/attn.txt 2>&1 || { tail -5 $OUT/attn.txt; exit 1; }
grep -v amdgpu.ids $OUT/attn.txt | cut -c1-60
