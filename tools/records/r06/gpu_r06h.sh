#!/bin/bash
# Round-6 attention backward staging profile: for each bwd stage (cullavo_attn_set_bwd_stage) a kernel
# trace of tools/attn_bench.py plus one FETCH_SIZE and one SQ pass over the dQ / dK-dV kernels
#   bash tools/records/r06/gpu_r06h.sh <tag> [stages...]   (default: 1 5 9 13; optional TESTS=1 first runs the staging tests)
set -o pipefail
TAG=${1:-r06h}; shift || true
STAGES=${*:-1 5 9 13}
OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ops_gpu.py -k attention tests/test_oob_guard.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
  tail -2 $OUT/tests.log
fi
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for st in $STAGES; do
  CULLAVO_ATTN_BWD_STAGE=$st timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace$st -o run --output-format csv -- python tools/attn_bench.py > $OUT/attn_traced$st.log 2>&1 || { tail -20 $OUT/attn_traced$st.log; exit 1; }
  python tools/prof_summary.py $OUT/trace$st/run_kernel_trace.csv --top 40 > $OUT/attn_summary$st.txt && echo "stage $st" && grep "dq_ring\|dq_ds_k<128\|dkdv8_k<128, true, true" $OUT/attn_summary$st.txt | cut -c1-140
  grep "LM causal" $OUT/attn_traced$st.log | cut -c1-120
  CULLAVO_ATTN_BWD_STAGE=$st timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "attn_bwd_dq|dkdv8" -d $OUT/pmc_f$st -o p --output-format csv -- python tools/attn_bench.py > $OUT/pmc_f$st.log 2>&1 || { tail -5 $OUT/pmc_f$st.log; exit 1; }
  CULLAVO_ATTN_BWD_STAGE=$st timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "attn_bwd_dq|dkdv8" -d $OUT/pmc_w$st -o p --output-format csv -- python tools/attn_bench.py > $OUT/pmc_w$st.log 2>&1 || { tail -5 $OUT/pmc_w$st.log; exit 1; }
  CULLAVO_ATTN_BWD_STAGE=$st timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES --kernel-include-regex "attn_bwd_dq|dkdv8" -d $OUT/pmc_s$st -o p --output-format csv -- python tools/attn_bench.py > $OUT/pmc_s$st.log 2>&1 || { tail -5 $OUT/pmc_s$st.log; exit 1; }
done
echo done
