#!/bin/bash
# Round-2 closing GPU pass on the restored tree: GPU tests, smoke, the bench lines of every
# BASELINE workload, and a kernel-trace profile of the default bench command.
set -o pipefail
OUT=gpurun_out/${1:-r02d}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 3; }
tail -2 $OUT/smoke.log
timeout -k 10 400 python bench.py > $OUT/bench.txt 2>&1 || { tail -20 $OUT/bench.txt; exit 4; }
tail -1 $OUT/bench.txt
timeout -k 10 300 python bench.py --trainable lora --no-cpu-baseline > $OUT/bench_lora.txt 2>&1 || { tail -20 $OUT/bench_lora.txt; exit 5; }
timeout -k 10 300 python bench.py --workload vit --batch 64 --no-cpu-baseline > $OUT/bench_vit.txt 2>&1 || { tail -20 $OUT/bench_vit.txt; exit 6; }
timeout -k 10 300 python bench.py --config llava-1.5-13b --batch 4 --text-len 1025 --no-cpu-baseline > $OUT/bench_13b.txt 2>&1 || { tail -20 $OUT/bench_13b.txt; exit 7; }
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_traced.log 2>&1 || { tail -20 $OUT/bench_traced.log; exit 8; }
python tools/prof_summary.py $OUT/trace/run_kernel_trace.csv --top 60 > $OUT/kernel_trace_summary.txt
echo done
