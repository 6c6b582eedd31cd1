#!/bin/bash
# one box: 32x32x16 ping-pong GEMM (parity + race screen + 7B shapes), decode bench b1/b8,
# ViT GEMM tiles, GEMM PMC (production vs ping-pong)
set -o pipefail
OUT=gpurun_out/r04f
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "pipelined_repeatable" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/gemm_bench.py --modes=-1,15,16,12 --iters 20 > $OUT/gemm_bench.txt 2>&1 || exit 1
grep -v amdgpu.ids $OUT/gemm_bench.txt | sed 's/T=8704 //; s/err [0-9.e+-]*//g' | cut -c1-170
for b in 1 8; do
  timeout -k 10 300 python -u bench.py --workload decode --batch $b --steps 8 --warmup 1 > $OUT/decode_b$b.json 2> $OUT/decode_b$b.err || { tail -20 $OUT/decode_b$b.err; exit 1; }
  cut -c1-1500 $OUT/decode_b$b.json
done
timeout -k 10 300 python -u tools/vit_gemm_bench.py --modes=-1,1,2,15 > $OUT/vit_gemm.txt 2>&1 || exit 1
grep -v amdgpu.ids $OUT/vit_gemm.txt | cut -c1-220
bash tools/gemm_pmc.sh r04f/pmc -1,12,15
