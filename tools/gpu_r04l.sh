#!/bin/bash
# decode GEMV variants: occupancy (8- / 4-load batches) against the 16-load default
set -o pipefail
OUT=gpurun_out/r04l
mkdir -p $OUT
for v in 1 4 5 6 7 1; do
  CULLAVO_GEMV=$v timeout -k 10 120 python -u tools/gemv_variant_bench.py >> $OUT/gemv_variants.txt 2>&1 || { tail -5 $OUT/gemv_variants.txt; exit 1; }
done
cat $OUT/gemv_variants.txt
# attention forward without its in-loop K/V loads (stage 6, lab: wrong results) against stage 4
ATTN_STAGE_AB=4,6,4,6 timeout -k 10 300 python -u tools/attn_bench.py > $OUT/attn_stage6.txt 2>&1 || { tail -5 $OUT/attn_stage6.txt; exit 1; }
cat $OUT/attn_stage6.txt
bash tools/gpu_r04m.sh
