#!/bin/bash
# Round-6 epilogue A/B on one box: per-shape (tools/epi_ab.py), then whole steps alternating (tools/ab.sh)
set -o pipefail
TAG=${1:-r06ab}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 400 python -u tools/epi_ab.py --rounds 5 > $OUT/epi_ab.txt 2>&1 || { tail -20 $OUT/epi_ab.txt; exit 1; }
grep -v amdgpu.ids $OUT/epi_ab.txt
bash tools/ab.sh $TAG/step 3 "direct=|" "lds=CULLAVO_GEMM_EPILOGUE=129|" "vdirect=|--workload vit" "vlds=CULLAVO_GEMM_EPILOGUE=129|--workload vit"
