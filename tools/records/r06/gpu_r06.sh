#!/bin/bash
# Round-6 GPU pass: targeted tests of the changed kernels first, A/B benches, then the full suite and the
# default bench line.  bash tools/records/r06/gpu_r06.sh <tag> [full]
set -o pipefail
TAG=${1:-r06}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_ops_gpu.py -k "direct_epilogue or swiglu or epilogue_paths or msplit" tests/test_accuracy_gpu.py \
  tests/test_lora.py -k "direct_epilogue or swiglu or epilogue_paths or msplit or accuracy or attention_against or lora_fused" \
  > $OUT/targeted.log 2>&1 || { echo "targeted tests failed"; tail -40 $OUT/targeted.log; exit 1; }
tail -2 $OUT/targeted.log
timeout -k 10 300 python -u tools/swiglu_dx_bench.py > $OUT/swiglu_dx.txt 2>&1 || { tail -20 $OUT/swiglu_dx.txt; exit 1; }
cat $OUT/swiglu_dx.txt | grep -v amdgpu.ids
timeout -k 10 300 env SHAPES=vit_fc1,vit_qkv,vit_o,gate_up,lm_head VARIANTS=0,2 python -u tools/lab/gemm_lab.py \
  --lib tools/lab/so/libgemm_hc.so --prod --variants 0,2,7,8 --shapes vit_fc1,vit_qkv,vit_o,gate_up,lm_head --rounds 3 \
  > $OUT/lab_vs_prod.txt 2>&1 || { tail -20 $OUT/lab_vs_prod.txt; exit 1; }
grep -v amdgpu.ids $OUT/lab_vs_prod.txt
if [ "$2" = "full" ]; then
  bash tools/gpu_pass.sh $TAG/pass || exit 1
fi
