#!/bin/bash
# Tile-order A/B on the GPU box: bitwise test, the GEMM group sweep, then the config-3 step with
# the new default order (groups of 4 N-tiles) against the old one (groups of 4 M-tiles), alternating.
set -o pipefail
OUT=gpurun_out/grp2
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/ops_tests.log 2>&1 || { tail -30 $OUT/ops_tests.log; exit 1; }
tail -2 $OUT/ops_tests.log
timeout -k 10 400 python tools/gemm_bench.py --modes=-1 --groups=-4,4,-3,-6,-8,-4,4 --iters 20 > $OUT/sweep.txt 2>&1 || { tail $OUT/sweep.txt; exit 2; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_new_$i.txt 2>&1 || exit 3
  CULLAVO_GEMM_GROUP=4 timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_old_$i.txt 2>&1 || exit 4
done
for f in $OUT/bench_*.txt; do echo $f $(tail -1 $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"); done
