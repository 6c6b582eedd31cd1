#!/bin/bash
# M-tail split: GEMM tests, then the ViT workload with the split on / off
set -o pipefail
OUT=gpurun_out/r05i
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q -k "gemm or linear" --timeout 120 --timeout-method thread > $OUT/gemm_tests.log 2>&1
rc=$?; tail -3 $OUT/gemm_tests.log; [ $rc -eq 0 ] || exit $rc
for ms in 1 0 1; do
  CULLAVO_GEMM_MSPLIT=$ms timeout -k 10 300 python -u bench.py --workload vit --no-sub --no-cpu-baseline --detail-out $OUT/vit_ms$ms.json > $OUT/vit_ms$ms.log 2>&1 || { tail -20 $OUT/vit_ms$ms.log; exit 1; }
  echo "msplit=$ms"; tail -c 600 $OUT/vit_ms$ms.log; echo
done
