#!/bin/bash
# ping-pong GEMM lab: one process per ablation (CULLAVO_PP_ABL bits, see gemm_pp.hip), tile mode 12
set -o pipefail
OUT=gpurun_out/${1:-r04c}
mkdir -p $OUT
for abl in 0 1 2 4 8 16 9 25 32 64 3; do
  echo "== abl $abl" >> $OUT/pp_ablate.txt
  CULLAVO_PP_ABL=$abl timeout -k 10 120 python -u tools/gemm_bench.py --modes=12 --iters 10 --only gate_up,o,qkv \
    --kinds fwd,dx,dw >> $OUT/pp_ablate.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $OUT/pp_ablate.txt | sed 's/T=8704 //; s/err [0-9.e+-]*//g' | cut -c1-120
