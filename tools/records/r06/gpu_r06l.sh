#!/bin/bash
# Round-6: 288-row persistent tiles at short K on top of the eager M-split (epilogue bits 8 + 9) --
# ViT per shape and whole ViT steps alternating; then the ViT PMC record under the current names
set -o pipefail
TAG=${1:-r06l}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 python -u tools/epi_ab.py --rounds 5 --modes direct,short288p --cases vit_fc1,vit_qkv,vit_o,vit_fc2 > $OUT/ab.txt 2>&1 || { tail -20 $OUT/ab.txt; exit 1; }
grep -v amdgpu.ids $OUT/ab.txt
bash tools/ab.sh $TAG/step 3 "vit=|--workload vit" "vit288=CULLAVO_GEMM_EPILOGUE=769|--workload vit" || exit 1
bash tools/profile_all.sh $TAG/prof config2-vit
