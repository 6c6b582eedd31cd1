#!/bin/bash
# Round profile on the GPU box: kernel trace + stats of the bench command, then two PMC passes
# (FETCH_SIZE, WRITE_SIZE) for the roofline kernel's HBM traffic. Outputs under gpurun_out/$1.
set -e
OUT=gpurun_out/${1:-prof}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_traced.log 2>&1
python tools/prof_summary.py $OUT/trace/run_kernel_trace.csv --top 60 > $OUT/summary.txt
KERNEL=$(python -c "import bench; print(bench.gemm_kernel_name(8704, 22016, 4096)[0])")
GRID=$(python -c "import bench; print(bench.gemm_kernel_name(8704, 22016, 4096)[1])")
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex gemm256 -d $OUT/pmc_fetch -o p --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/pmc_fetch.log 2>&1
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex gemm256 -d $OUT/pmc_write -o p --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/pmc_write.log 2>&1
python tools/pmc_traffic.py $OUT/pmc_fetch/p_counter_collection.csv $OUT/pmc_write/p_counter_collection.csv "$KERNEL" $GRID > $OUT/roofline_traffic.json
echo done
