#!/bin/bash
# Round-6 ViT plan A/B: 288-row tiles at K < 2048 (epilogue bit 9) per shape, then whole ViT steps alternating
set -o pipefail
TAG=${1:-r06e}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 python -u tools/epi_ab.py --rounds 5 --modes direct,short288,short288p \
  --cases vit_fc1,vit_qkv,vit_o,vit_fc2 > $OUT/vit_plan_ab.txt 2>&1 || { tail -20 $OUT/vit_plan_ab.txt; exit 1; }
grep -v amdgpu.ids $OUT/vit_plan_ab.txt
bash tools/ab.sh $TAG/step 3 "vdirect=|--workload vit" "vshort=CULLAVO_GEMM_EPILOGUE=513|--workload vit" "vshortp=CULLAVO_GEMM_EPILOGUE=769|--workload vit"
