#!/bin/bash
# One GPU-box pass: GPU parity tests, the headline bench line, then the round profile.
# Usage (from the repo root, on the box): bash tools/gpu_check.sh <tag> [skip-tests]
set -o pipefail
TAG=${1:-check}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
  tail -3 $OUT/gpu_tests.log
fi
timeout -k 10 400 python -u bench.py > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
bash tools/profile_round.sh $TAG/prof || { echo "profile failed"; exit 1; }
head -25 $OUT/prof/summary.txt
cat $OUT/prof/roofline_traffic.json
