#!/bin/bash
# Round-6: eager M-tail split (cullavo_gemm_set_msplit(2)) -- ViT fc1 per shape, M-split tests, ViT steps alternating
set -o pipefail
TAG=${1:-r06k}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ops_gpu.py -k "msplit or split or direct_epilogue" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -u tools/epi_ab.py --rounds 5 --modes direct,eager --cases vit_fc1,vit_qkv > $OUT/ab.txt 2>&1 || { tail -20 $OUT/ab.txt; exit 1; }
grep -v amdgpu.ids $OUT/ab.txt
bash tools/ab.sh $TAG/step 3 "vit=|--workload vit" "vit_eager=CULLAVO_GEMM_MSPLIT=2|--workload vit"
