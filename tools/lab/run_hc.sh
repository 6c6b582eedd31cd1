#!/bin/bash
# GPU box: the held-C GEMM lab (tools/lab/gemm_hc_lab.hip) against the production kernel and hipBLASLt
set -o pipefail
OUT=gpurun_out/${1:-hc}
mkdir -p $OUT
timeout -k 10 500 python -u tools/lab/gemm_lab.py --lib tools/lab/so/libgemm_hc.so --prod \
  --variants ${VARIANTS:-0,1,2,3,4,101,102,103,104,201} \
  --shapes ${SHAPES:-vit_fc1,vit_qkv,vit_o,gate_up,qkv,lm_head} --rounds 3 > $OUT/lab.txt 2>&1
rc=$?
cat $OUT/lab.txt | tail -20
exit $rc
