#!/bin/bash
# Round-6: the 288-row tiles at K < 2048 as the default -- GEMM / accuracy tests, then config-3 and ViT
# steps alternating against bit 9 (round 5's plan for short K)
set -o pipefail
TAG=${1:-r06m}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ops_gpu.py tests/test_accuracy_gpu.py tests/test_lora.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
bash tools/ab.sh $TAG/step 3 "c3=|" "c3_no288=CULLAVO_GEMM_EPILOGUE=513|" "vit=|--workload vit" "vit_no288=CULLAVO_GEMM_EPILOGUE=513|--workload vit"
