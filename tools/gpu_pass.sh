#!/bin/bash
# One validation pass on the GPU box: GPU parity suite, smoke(), the default bench line.
#   bash tools/gpu_pass.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-pass}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python -u bench.py --detail-out $OUT/bench_detail.json "$@" > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
