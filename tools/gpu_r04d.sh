#!/bin/bash
# decode GEMV + graph: tests, decode bench b1/b8; ViT GEMM tiles; GEMM PMC (production vs ping-pong)
set -o pipefail
OUT=gpurun_out/r04d
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_generation.py tests/test_ops_gpu.py -m gpu -x -q --timeout 200 \
  --timeout-method thread -k "generation or gemv or decode or eos or gemm_layouts" > $OUT/tests.log 2>&1
rc=$?; tail -5 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for b in 1 8; do
  timeout -k 10 300 python -u bench.py --workload decode --batch $b --steps 8 --warmup 1 > $OUT/decode_b$b.json 2> $OUT/decode_b$b.err || { tail -20 $OUT/decode_b$b.err; exit 1; }
  cut -c1-1200 $OUT/decode_b$b.json
done
timeout -k 10 300 python -u tools/vit_gemm_bench.py --modes=-1,1,2,12,13 > $OUT/vit_gemm.txt 2>&1 || exit 1
cat $OUT/vit_gemm.txt | grep -v amdgpu.ids | cut -c1-220
bash tools/gemm_pmc.sh r04d/pmc -1,12
