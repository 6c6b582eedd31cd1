#!/bin/bash
# persistent 256x256 GEMM lab (tools/lab/gemm256p_lab.hip) against production and hipBLASLt
set -o pipefail
OUT=gpurun_out/r05o
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/lab/gemm_lab.py --lib tools/lab/bin/libgemm256p_lab.so --prod \
  --variants 1000,1008,1512,2024,3048 --shapes vit_fc1,vit_qkv,gate_up,qkv --rounds 3 > $OUT/lab.txt 2>&1
rc=$?; cat $OUT/lab.txt; exit $rc
