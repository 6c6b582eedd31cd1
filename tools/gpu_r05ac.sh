#!/bin/bash
# GEMM epilogue: lean activation and SwiGLU-backward paths -- the whole GPU suite, then one-box A/B
# (1 = all lean paths, 17 = without the activation / SwiGLU-backward ones)
set -o pipefail
OUT=gpurun_out/r05ac
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for e in 1 17 1 17; do
  CULLAVO_GEMM_EPILOGUE=$e timeout -k 10 600 python -u bench.py --no-cpu-baseline --detail-out $OUT/bench_e$e.json > $OUT/bench_e$e.log 2>&1 || { tail -20 $OUT/bench_e$e.log; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/bench_e$e.json')); print('epi=$e', d['value'], d['ms_per_step'], ' '.join(f'{k}={v[\"value\"]}' for k,v in d['workloads'].items()))"
done
