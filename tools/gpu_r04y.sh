#!/bin/bash
# decode GEMV: 16-wave workgroups (variants 8 / 9) against the defaults (4, 6)
set -o pipefail
OUT=gpurun_out/r04y
mkdir -p $OUT
for v in 4 6 8 9 4 8; do
  CULLAVO_GEMV=$v timeout -k 10 120 python -u tools/gemv_variant_bench.py >> $OUT/gemv_variants16.txt 2>&1 || { tail -5 $OUT/gemv_variants16.txt; exit 1; }
done
grep -v amdgpu.ids $OUT/gemv_variants16.txt
