#!/bin/bash
# round-5 closing profiles (after the GEMM epilogue work): per-workload kernel traces + PMC records (tools/profile_all.sh), and the
# decode GEMV's HBM traffic (two PMC passes over the decode-b1 / decode-b8 runs)
set -o pipefail
TAG=r05final3
bash tools/profile_all.sh $TAG || exit 1
OUT=gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for b in 1 8; do
  for pass in "FETCH_SIZE:fetch" "WRITE_SIZE:write" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY:sq"; do
    CNT=${pass%%:*}; T=${pass##*:}
    timeout -s KILL 300 rocprofv3 --pmc $CNT --kernel-include-regex gemv -d $OUT/decode_b$b/pmc_$T -o p --output-format csv -- python bench.py --workload decode --batch $b --steps 2 --warmup 1 --no-cpu-baseline > $OUT/decode_b$b.$T.log 2>&1 || { tail -3 $OUT/decode_b$b.$T.log; exit 1; }
  done
  python tools/pmc_family.py $OUT/decode_b$b/pmc_fetch/p_counter_collection.csv $OUT/decode_b$b/pmc_write/p_counter_collection.csv $OUT/decode_b$b/pmc_sq/p_counter_collection.csv "gemv_k<" decode-b$b > $OUT/decode_b$b/roofline_traffic.json
  cat $OUT/decode_b$b/roofline_traffic.json
done
echo all done
