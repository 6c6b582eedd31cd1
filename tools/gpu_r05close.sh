#!/bin/bash
# closing check of the committed tree: smoke() and the default bench line
set -o pipefail
mkdir -p gpurun_out/r05close
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05close/smoke.log 2>&1 || { tail -5 gpurun_out/r05close/smoke.log; exit 1; }
tail -2 gpurun_out/r05close/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r05close/bench.log 2>&1 || { tail -5 gpurun_out/r05close/bench.log; exit 1; }
tail -1 gpurun_out/r05close/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['unit'], d['roofline']['kernel'][:80], d['roofline']['frac'], len(json.dumps(d)))"
echo all done
