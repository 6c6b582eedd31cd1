#!/bin/bash
# Round-5 closing validation after the GEMM epilogue work: GPU suite, smoke(), default bench
set -o pipefail
OUT=gpurun_out/r05af
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; tail -2 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --detail-out $OUT/bench_detail.json > $OUT/bench.log 2>$OUT/bench.err
rc=$?; tail -c 4200 $OUT/bench.log; echo; [ $rc -eq 0 ] || { tail -20 $OUT/bench.err; exit $rc; }
