#!/bin/bash
# kernel traces of the ViT workload and the config-3 step at the current head
set -o pipefail
OUT=gpurun_out/r05k
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $OUT/vit -o vit --output-format csv -- python bench.py --workload vit --no-sub --no-cpu-baseline --steps 3 --warmup 1 --detail-out $OUT/vit.json > $OUT/vit.log 2>&1 || { tail -5 $OUT/vit.log; exit 1; }
python tools/prof_summary.py $OUT/vit/vit_kernel_trace.csv > $OUT/vit_summary.txt 2>&1 || true
head -25 $OUT/vit_summary.txt
