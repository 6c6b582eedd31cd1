#!/bin/bash
# GEMM epilogue paths A/B on one box: all lean paths (1), no bias/residual path (5), no lean path (13)
set -o pipefail
OUT=gpurun_out/r05ab
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_oob_guard.py tests/test_lora.py -x -q -k "gemm or linear or lora" --timeout 300 --timeout-method thread > $OUT/gemm_tests.log 2>&1
rc=$?; tail -3 $OUT/gemm_tests.log; [ $rc -eq 0 ] || exit $rc
for e in 1 5 13 1; do
  CULLAVO_GEMM_EPILOGUE=$e timeout -k 10 600 python -u bench.py --no-cpu-baseline --detail-out $OUT/bench_e$e.json > $OUT/bench_e$e.log 2>&1 || { tail -20 $OUT/bench_e$e.log; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/bench_e$e.json')); print('epi=$e', d['value'], d['ms_per_step'], ' '.join(f'{k}={v[\"value\"]}' for k,v in d['workloads'].items()))"
done
