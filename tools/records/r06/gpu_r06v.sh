#!/bin/bash
# Round-6: tile order (cullavo_gemm_set_group, default -4 = groups of 4 N-tiles sweeping the M-tiles) on
# the config-3 step with the round-6 kernels
set -o pipefail
TAG=${1:-r06v}; [ $# -ge 2 ] || set -- "$TAG" "g-4=|" "g-8=CULLAVO_GEMM_GROUP=-8|" "g-16=CULLAVO_GEMM_GROUP=-16|" "g4=CULLAVO_GEMM_GROUP=4|" "g8=CULLAVO_GEMM_GROUP=8|"; OUT=gpurun_out/$TAG; mkdir -p $OUT
bash tools/ab.sh $TAG/step 2 "${@:2}"
