#!/bin/bash
# GPU parity suite on the box: bash tools/gpu_tests.sh <tag> [pytest selection...]
set -o pipefail
TAG=${1:-tests}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest ${@:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|SKIPPED" $OUT/gpu_tests.log | grep -v "^tests.*PASSED" | tail -30
tail -40 $OUT/gpu_tests.log | grep -v PASSED | tail -30
exit $rc
