#!/bin/bash
# Round-6: the split-K block target (cullavo_gemm_set_splitk_target, default 512) on the ViT step, whose
# M-split tails (64 rows) run split over K on the 4-wave kernel; and on config 3 (its small-grid products)
set -o pipefail
TAG=${1:-r06t}; OUT=gpurun_out/$TAG; mkdir -p $OUT
bash tools/ab.sh $TAG/step 3 "v512=|--workload vit" "v256=CULLAVO_SPLITK_TARGET=256|--workload vit" "v128=CULLAVO_SPLITK_TARGET=128|--workload vit" "v1024=CULLAVO_SPLITK_TARGET=1024|--workload vit"
