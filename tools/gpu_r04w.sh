#!/bin/bash
set -o pipefail
OUT=gpurun_out/r04w
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_ops_gpu.py tests/test_oob_guard.py tests/test_full_size.py -k "attention or attn or decoder_layer" > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/tests.log | head -20; exit $rc; }
ATTN_STAGE_AB=7,7 timeout -k 10 300 python -u tools/attn_bench.py > $OUT/attn.txt 2>&1 || { tail -5 $OUT/attn.txt; exit 1; }
grep -v amdgpu.ids $OUT/attn.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
REPS=4 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 tools/attn_one.py 7 > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
python3 - $OUT/prof/run_kernel_stats.csv <<'PY'
import csv, sys
for r in sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: -float(r["TotalDurationNs"]))[:6]:
    print(f'{r["Name"][:80]:80s} n={r["Calls"]:>4s} avg={float(r["AverageNs"])/1e3:8.1f} us')
PY
