#!/bin/bash
# Round 5, first GPU pass: GPU parity suite, the default bench (compact line + sidecar), then this
# library's GEMM against hipBLASLt under a kernel trace and PMC passes (same process, same operands).
set -o pipefail
OUT=gpurun_out/r05a
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --detail-out $OUT/bench_detail.json > $OUT/bench.log 2>$OUT/bench.err
rc=$?; tail -c 4200 $OUT/bench.log; echo; [ $rc -eq 0 ] || { tail -20 $OUT/bench.err; exit $rc; }
timeout -k 10 120 python -u tools/gemm_vs_lib.py > $OUT/gemm_vs_lib.txt 2>&1 || exit 1
cat $OUT/gemm_vs_lib.txt
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python tools/gemm_vs_lib.py --rounds 1 > $OUT/kt.log 2>&1 || { tail -5 $OUT/kt.log; exit 1; }
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
P3="FETCH_SIZE GRBM_GUI_ACTIVE"
P4="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
i=0
for CNT in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CNT --kernel-include-regex "gemm|Cijk" -d $OUT/p$i -o p --output-format csv -- python tools/gemm_vs_lib.py --rounds 1 --reps 3 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
echo done
