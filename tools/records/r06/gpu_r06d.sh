#!/bin/bash
set -o pipefail
TAG=${1:-r06d}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_ops_gpu.py tests/test_accuracy_gpu.py \
  -k "direct_epilogue or round_split or msplit or accuracy or attention_against or gemm_288" > $OUT/targeted.log 2>&1 \
  || { echo "targeted tests failed"; tail -40 $OUT/targeted.log; exit 1; }
tail -2 $OUT/targeted.log
bash tools/ab.sh $TAG/step 3 "split=|" "nosplit=CULLAVO_GEMM_MSPLIT=0|"
