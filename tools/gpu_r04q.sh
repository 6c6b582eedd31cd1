#!/bin/bash
set -o pipefail
OUT=gpurun_out/r04q
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_ops_gpu.py -k "pipelined_rescale" > $OUT/t.log 2>&1; grep -E "^E  |passed|failed" $OUT/t.log | head -20
