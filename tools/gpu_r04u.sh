#!/bin/bash
# decode step kernel breakdown (kernel trace of the decode-b1 workload)
set -o pipefail
OUT=gpurun_out/r04u
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python bench.py --workload decode --batch 1 --steps 4 --warmup 1 --no-cpu-baseline > $OUT/b1.log 2>&1 || { tail -5 $OUT/b1.log; exit 1; }
python tools/prof_summary.py $OUT/trace/run_kernel_trace.csv --top 40 > $OUT/summary.txt
cat $OUT/summary.txt
