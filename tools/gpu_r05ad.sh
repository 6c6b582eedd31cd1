#!/bin/bash
# persistent forward kernel (gemm256p_k, layout (0,0), 256x256): GPU suite, per-shape lab, one-box A/B
# (1 = on, 33 = off via cullavo_gemm_set_epilogue bit 5)
set -o pipefail
OUT=gpurun_out/r05ad
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for e in 1 33; do
  CULLAVO_GEMM_EPILOGUE=$e timeout -k 10 300 python -u tools/lab/gemm_lab.py --lib tools/lab/bin/libgemm256p_lab.so --prod \
    --variants 1000 --shapes vit_fc1,vit_qkv,vit_o,lm_head --rounds 3 > $OUT/lab_e$e.txt 2>&1 || { tail -5 $OUT/lab_e$e.txt; exit 1; }
  echo "epi=$e"; grep -v amdgpu.ids $OUT/lab_e$e.txt
done
for e in 1 33 1 33; do
  CULLAVO_GEMM_EPILOGUE=$e timeout -k 10 600 python -u bench.py --no-cpu-baseline --detail-out $OUT/bench_e$e.json > $OUT/bench_e$e.log 2>&1 || { tail -20 $OUT/bench_e$e.log; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/bench_e$e.json')); print('epi=$e', d['value'], d['ms_per_step'], ' '.join(f'{k}={v[\"value\"]}' for k,v in d['workloads'].items()))"
done
