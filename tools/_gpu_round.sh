set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "attn or attention" > gpurun_out/ops_tests.log 2>&1 || exit 1
timeout -k 10 200 python tools/attn_bench.py > gpurun_out/attn_bench.log 2>&1 || exit 2
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || exit 3
cat gpurun_out/attn_bench.log; tail -1 gpurun_out/bench.log
