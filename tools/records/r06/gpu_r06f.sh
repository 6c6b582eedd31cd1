#!/bin/bash
# Round-6 decode A/B: non-temporal weight loads in the GEMV (cullavo_gemv_set_nt) per shape, the
# generation tests with them on, then whole decode steps alternating at batch 1 and 8
set -o pipefail
TAG=${1:-r06f}; OUT=gpurun_out/$TAG; mkdir -p $OUT
for nt in 0 1 0 1; do
  CULLAVO_GEMV_NT=$nt timeout -k 10 200 python -u tools/gemv_variant_bench.py >> $OUT/gemv_nt$nt.txt 2>&1 || { tail -20 $OUT/gemv_nt$nt.txt; exit 1; }
done
grep -h "gemv" $OUT/gemv_nt0.txt $OUT/gemv_nt1.txt
CULLAVO_GEMV_NT=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_generation.py > $OUT/gen_tests_nt.log 2>&1 || { tail -30 $OUT/gen_tests_nt.log; exit 1; }
tail -2 $OUT/gen_tests_nt.log
bash tools/ab.sh $TAG/step 3 "b1=|--workload decode --batch 1" "b1nt=CULLAVO_GEMV_NT=1|--workload decode --batch 1" \
  "b8=|--workload decode --batch 8" "b8nt=CULLAVO_GEMV_NT=1|--workload decode --batch 8"
