#!/bin/bash
# GEMM C stores with the non-temporal policy (CULLAVO_GEMM_EPILOGUE=3) against the default: per-shape
# lab (production path) and the whole default bench (config 3 + sub-workloads)
set -o pipefail
OUT=gpurun_out/r05z
mkdir -p $OUT
export TMPDIR=/tmp
for e in 1 3; do
  CULLAVO_GEMM_EPILOGUE=$e timeout -k 10 300 python -u tools/lab/gemm_lab.py --lib tools/lab/bin/libgemm256p_lab.so --prod \
    --variants 1000 --shapes vit_fc1,vit_qkv,vit_o,gate_up,qkv,o,down,lm_head --rounds 3 > $OUT/lab_epi$e.txt 2>&1 || { tail -5 $OUT/lab_epi$e.txt; exit 1; }
  echo "epilogue=$e"; cat $OUT/lab_epi$e.txt | grep -v amdgpu.ids
done
for e in 3 1; do
  CULLAVO_GEMM_EPILOGUE=$e timeout -k 10 600 python -u bench.py --no-cpu-baseline --detail-out $OUT/bench_epi$e.json > $OUT/bench_epi$e.log 2>&1 || { tail -20 $OUT/bench_epi$e.log; exit 1; }
  echo "bench epilogue=$e"; python -c "
import json; d=json.load(open('$OUT/bench_epi$e.json')); print(d['value'], d['ms_per_step'])
for k,v in d['workloads'].items(): print(' ', k, v['value'], v['ms_per_step'])"
done
