#!/bin/bash
# Round-6: the SwiGLU-backward dX through the direct epilogue (direct_epilogue_swiglu) -- tests, the dX
# GEMM per shape (direct / prefetch / general / plain), steps alternating against the previous library
set -o pipefail
TAG=${1:-r06r}; OUT=gpurun_out/$TAG; mkdir -p $OUT
PREV=tools/lab/so/prev/libcullavo_prev.so
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ops_gpu.py tests/test_model_gpu.py tests/test_accuracy_gpu.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -u tools/swiglu_dx_bench.py --rounds 5 > $OUT/swg.txt 2>&1 || { tail -20 $OUT/swg.txt; exit 1; }
grep -v amdgpu.ids $OUT/swg.txt
bash tools/ab.sh $TAG/step 3 "c3=|" "c3prev=CULLAVO_LIB_AB=$PREV|"
