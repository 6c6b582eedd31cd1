#!/bin/bash
# One GPU-box pass: GPU parity tests, smoke, the headline bench line (+ LoRA, ViT and 13B lines),
# then the round profile of the headline step. Usage (repo root, on the box):
#   bash tools/gpu_check.sh <tag> [skip-tests]
set -o pipefail
TAG=${1:-check}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
  tail -3 $OUT/gpu_tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
timeout -k 10 400 python -u bench.py > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
timeout -k 10 300 python -u bench.py --trainable lora --no-cpu-baseline > $OUT/bench_lora.log 2>&1 && tail -1 $OUT/bench_lora.log
timeout -k 10 300 python -u bench.py --workload vit --steps 10 --warmup 2 > $OUT/bench_vit.log 2>&1 && tail -1 $OUT/bench_vit.log
timeout -k 10 400 python -u bench.py --config llava-1.5-13b --text-len 1025 --batch 4 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_13b.log 2>&1 && tail -1 $OUT/bench_13b.log
bash tools/profile_round.sh $TAG/prof || { echo "profile failed"; exit 1; }
head -30 $OUT/prof/summary.txt
cat $OUT/prof/roofline_traffic.json
