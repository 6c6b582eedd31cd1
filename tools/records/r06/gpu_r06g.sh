#!/bin/bash
# Round-6 attention dQ ring A/B: staging tests (bitwise), per-layer bwd A/B (tools/attn_bench.py),
# a kernel trace of the ring, then whole config-3 steps alternating (bwd stage 1 vs 5)
set -o pipefail
TAG=${1:-r06g}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ops_gpu.py -k attention tests/test_oob_guard.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
ATTN_STAGE_AB=17,57,17,57 timeout -k 10 300 python -u tools/attn_bench.py > $OUT/attn_ab.txt 2>&1 || { tail -20 $OUT/attn_ab.txt; exit 1; }
grep -v amdgpu.ids $OUT/attn_ab.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ATTN_STAGE_AB=57 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python tools/attn_bench.py > $OUT/attn_traced.log 2>&1 || { tail -20 $OUT/attn_traced.log; exit 1; }
python tools/prof_summary.py $OUT/trace/run_kernel_trace.csv --top 12 > $OUT/attn_summary.txt && cat $OUT/attn_summary.txt | cut -c1-160
bash tools/ab.sh $TAG/step 3 "s1=|" "s5=CULLAVO_ATTN_BWD_STAGE=5|"
