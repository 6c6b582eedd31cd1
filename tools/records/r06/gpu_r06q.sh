#!/bin/bash
# Round-6: SwiGLU backward's sigmoid by v_rcp_f32 (fused epilogue and swiglu_bwd_k) -- tests, the
# dX GEMM per shape (new vs the previous library), steps alternating
set -o pipefail
TAG=${1:-r06q}; OUT=gpurun_out/$TAG; mkdir -p $OUT
PREV=tools/lab/so/prev/libcullavo_prev.so
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ops_gpu.py tests/test_model_gpu.py tests/test_parity_modes.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for r in 1 2; do
  timeout -k 10 200 python -u tools/swiglu_dx_bench.py --rounds 3 > $OUT/new_$r.txt 2>&1 || { tail -20 $OUT/new_$r.txt; exit 1; }
  CULLAVO_LIB_AB=$PREV timeout -k 10 200 python -u tools/swiglu_dx_bench.py --rounds 3 > $OUT/prev_$r.txt 2>&1 || { tail -20 $OUT/prev_$r.txt; exit 1; }
done
for r in 1 2; do echo "new $r"; grep -v "amdgpu.ids\|CULLAVO_LIB_AB" $OUT/new_$r.txt; echo "prev $r"; grep -v "amdgpu.ids\|CULLAVO_LIB_AB" $OUT/prev_$r.txt; done
bash tools/ab.sh $TAG/step 3 "c3=|" "c3prev=CULLAVO_LIB_AB=$PREV|"
