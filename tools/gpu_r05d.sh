#!/bin/bash
# stripped library: GPU suite, then the r05c lab profile (4-wave AGPR kernel vs production vs hipBLASLt)
set -o pipefail
OUT=gpurun_out/r05d
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $OUT/gpu_tests.log | head; exit $rc; }
bash tools/gpu_r05c.sh
