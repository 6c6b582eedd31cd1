#!/bin/bash
# Round-6: the down-projection dW beside the SwiGLU-fused dX GEMM (CULLAVO_SWG_OVERLAP) -- bitwise
# test, then whole config-3 steps alternating; and the attention dQ records (ring / blocked dS^T)
set -o pipefail
TAG=${1:-r06j}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_model_gpu.py -k side_stream > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
bash tools/ab.sh $TAG/step 3 "base=|" "swg=CULLAVO_SWG_OVERLAP=1|"
