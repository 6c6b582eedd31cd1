#!/bin/bash
# Tile-order A/B on the other BASELINE workloads: config 2 (ViT-L bs64) and config 5 (13B), new
# default (groups of 4 N-tiles) against the old order (CULLAVO_GEMM_GROUP=4), alternating.
set -o pipefail
OUT=gpurun_out/grp3
mkdir -p $OUT
for i in 1 2; do
  for g in -4 4; do
    CULLAVO_GEMM_GROUP=$g timeout -k 10 200 python bench.py --workload vit --no-cpu-baseline > $OUT/vit_g${g}_$i.txt 2>&1 || exit 2
    CULLAVO_GEMM_GROUP=$g timeout -k 10 300 python bench.py --config llava-1.5-13b --batch 4 --text-len 1025 --no-cpu-baseline > $OUT/13b_g${g}_$i.txt 2>&1 || exit 3
  done
done
for f in $OUT/*.txt; do echo $f $(tail -1 $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"); done
