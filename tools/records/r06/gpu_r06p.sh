#!/bin/bash
# Round-6: the direct epilogue's residual chunks all loaded before the first store -- GEMM tests,
# per-shape (new vs the previous library, tools/lab/so/prev/), then steps alternating
set -o pipefail
TAG=${1:-r06p}; OUT=gpurun_out/$TAG; mkdir -p $OUT
PREV=tools/lab/so/prev/libcullavo_prev.so
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ops_gpu.py tests/test_accuracy_gpu.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for r in 1 2; do
  timeout -k 10 300 python -u tools/epi_ab.py --rounds 3 --modes direct --cases o_fwd,down_fwd,vit_o,vit_fc2,qkv_fwd > $OUT/new_$r.txt 2>&1 || { tail -20 $OUT/new_$r.txt; exit 1; }
  CULLAVO_LIB_AB=$PREV timeout -k 10 300 python -u tools/epi_ab.py --rounds 3 --modes direct --cases o_fwd,down_fwd,vit_o,vit_fc2,qkv_fwd > $OUT/prev_$r.txt 2>&1 || { tail -20 $OUT/prev_$r.txt; exit 1; }
done
for r in 1 2; do echo "new $r"; grep -v "amdgpu.ids\|CULLAVO_LIB_AB" $OUT/new_$r.txt; echo "prev $r"; grep -v "amdgpu.ids\|CULLAVO_LIB_AB\|notice" $OUT/prev_$r.txt; done
bash tools/ab.sh $TAG/step 3 "c3=|" "c3prev=CULLAVO_LIB_AB=$PREV|" "vit=|--workload vit" "vitprev=CULLAVO_LIB_AB=$PREV|--workload vit"
