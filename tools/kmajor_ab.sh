#!/bin/bash
# K-major dX A/B on the GPU box: parity tests, then the headline bench under each refresh mode.
set -o pipefail
OUT=gpurun_out/kmajor
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
for mode in side off sync; do
  CULLAVO_KMAJOR=$mode timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_$mode.log 2>&1 || { echo "bench $mode failed"; tail -20 $OUT/bench_$mode.log; exit 1; }
  echo "$mode: $(grep -o '"value": [0-9.]*' $OUT/bench_$mode.log) $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_$mode.log)"
done
