# kernel traces of the LoRA recipe and the full fine-tune step (round 2, late session)
set -e
OUT=gpurun_out/r02c
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace_lora -o run --output-format csv -- python bench.py --trainable lora --steps 3 --warmup 2 --no-cpu-baseline > $OUT/bench_lora_traced.log 2>&1
python tools/prof_summary.py $OUT/trace_lora/run_kernel_trace.csv --top 70 > $OUT/summary_lora.txt
timeout -k 10 400 python bench.py --trainable lora --no-cpu-baseline > $OUT/bench_lora.log 2>&1
tail -1 $OUT/bench_lora.log
head -40 $OUT/summary_lora.txt
