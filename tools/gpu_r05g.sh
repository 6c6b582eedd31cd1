#!/bin/bash
# ablations of the 4-wave GEMM (tools/lab/gemm4w_lab.hip)
set -o pipefail
OUT=gpurun_out/r05g
mkdir -p $OUT
timeout -k 10 300 python -u tools/lab/gemm_lab.py --lib tools/lab/bin/libgemm4w_lab.so --variants 2001,2000,2001,2000 --shapes gate_up,lm_head,qkv,o,down --prod > $OUT/abl.txt 2>&1; rc=$?
cat $OUT/abl.txt; exit $rc
