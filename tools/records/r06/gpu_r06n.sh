#!/bin/bash
# Round-6: ViT steps alternating, 5 rounds: default / bit 9 (no 288 at short K) / + bit 8 (persistent 288 at long K too)
set -o pipefail
TAG=${1:-r06n}; OUT=gpurun_out/$TAG; mkdir -p $OUT
bash tools/ab.sh $TAG/step 5 "vit=|--workload vit" "vit_no288=CULLAVO_GEMM_EPILOGUE=513|--workload vit" "vit_p288=CULLAVO_GEMM_EPILOGUE=257|--workload vit"
