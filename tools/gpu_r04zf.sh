#!/bin/bash
# decode attention: 64-key chunks (576 workgroups at batch 1)
set -o pipefail
OUT=gpurun_out/r04zf
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_generation.py > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/tests.log | head -20; exit $rc; }
for b in 1 8 1 8; do
  timeout -k 10 300 python -u bench.py --workload decode --batch $b --no-sub --no-cpu-baseline > $OUT/decode_b$b.json 2> $OUT/decode_b$b.err || { tail -5 $OUT/decode_b$b.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/decode_b$b.json').read().strip().splitlines()[-1]);print('b$b', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -- python3 $GRAFT_REPO_ROOT/tools/decode_bench.py --batch 1 > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$OUT/prof.log; exit 1; }
f=$(find $GRAFT_REPO_ROOT/$OUT/prof -name "*kernel_stats.csv" | head -1)
grep -E "attn_decode|gemv_k|rmsnorm|rope|swiglu" "$f" | cut -c1-220
