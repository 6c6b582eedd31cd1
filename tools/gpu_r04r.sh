#!/bin/bash
# per-kernel times of backward modes 7 and 8 (7B layer shape), forward stage 4 / 7
set -o pipefail
OUT=gpurun_out/r04r
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
REPS=4 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 tools/attn_one.py 7 8 > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print(f'{r["Name"][:90]:90s} n={r["Calls"]:>4s} avg={float(r["AverageNs"])/1e3:8.1f} us')
PY
