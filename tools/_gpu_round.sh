set -o pipefail
mkdir -p gpurun_out
for t in full lora; do
timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --trainable $t > gpurun_out/loss0_$t.log 2>&1 || exit 1
done
