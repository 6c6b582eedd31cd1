#!/bin/bash
set -o pipefail
OUT=gpurun_out/r04za
mkdir -p $OUT
timeout -k 10 300 python -u tools/attn_fwd_ab.py 6 4 7 > $OUT/ab.txt 2>&1 || { tail -5 $OUT/ab.txt; exit 1; }
grep -v amdgpu.ids $OUT/ab.txt
