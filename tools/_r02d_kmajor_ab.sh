#!/bin/bash
# K-major weight copies for the decoder dX GEMMs (CULLAVO_KMAJOR) under the round's final GEMM
# defaults: config-3 step, alternating off / side / sync.
set -o pipefail
OUT=gpurun_out/kmajor
mkdir -p $OUT
for i in 1 2; do
  for mode in off side sync; do
    CULLAVO_KMAJOR=$mode timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_${mode}_$i.txt 2>&1 || { tail -20 $OUT/bench_${mode}_$i.txt; exit 2; }
  done
done
for f in $OUT/bench_*.txt; do echo $f $(tail -1 $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['loss'])"); done
