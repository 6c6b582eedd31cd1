#!/bin/bash
set -o pipefail
OUT=gpurun_out/r04ze
mkdir -p $OUT
timeout -k 10 300 python -u tools/lab/mall_warm_gemv.py > $OUT/mall.txt 2>&1 || { tail -5 $OUT/mall.txt; exit 1; }
grep -v amdgpu.ids $OUT/mall.txt
