#!/bin/bash
# Fused SwiGLU-backward epilogue: its bitwise tests, then the config-3 step fused vs unfused, alternating.
set -o pipefail
OUT=gpurun_out/swiglu
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py tests/test_model_gpu.py -x -q -m gpu -k "swiglu" --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_fused_$i.txt 2>&1 || { tail -20 $OUT/bench_fused_$i.txt; exit 2; }
  CULLAVO_FUSED_SWIGLU_BWD=0 timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_sep_$i.txt 2>&1 || exit 3
done
for f in $OUT/bench_*.txt; do echo $f $(tail -1 $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['loss'])"); done
