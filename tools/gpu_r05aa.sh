#!/bin/bash
# GEMM epilogue: lean plain-bf16 store path in lds_epilogue -- GEMM tests, per-shape lab (production
# path), then the default bench
set -o pipefail
OUT=gpurun_out/r05aa
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_oob_guard.py -x -q -k "gemm or linear" --timeout 300 --timeout-method thread > $OUT/gemm_tests.log 2>&1
rc=$?; tail -3 $OUT/gemm_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/lab/gemm_lab.py --lib tools/lab/bin/libgemm256p_lab.so --prod \
  --variants 1000 --shapes vit_fc1,vit_qkv,vit_o,gate_up,qkv,o,down,lm_head --rounds 3 > $OUT/lab.txt 2>&1 || { tail -5 $OUT/lab.txt; exit 1; }
grep -v amdgpu.ids $OUT/lab.txt
timeout -k 10 600 python -u bench.py --no-cpu-baseline --detail-out $OUT/bench.json > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
python -c "
import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['achieved'])
for k,v in d['workloads'].items(): print(' ', k, v['value'], v['ms_per_step'])"
