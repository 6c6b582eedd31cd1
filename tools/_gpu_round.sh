set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_ops_gpu.py -x -q > gpurun_out/ops_tests.log 2>&1 || exit 1
timeout -k 10 300 python -m pytest tests/test_model_gpu.py tests/test_generation.py -x -q > gpurun_out/model_tests.log 2>&1 || exit 1
timeout -k 10 200 python tools/attn_bench.py > gpurun_out/attn_bench.log 2>&1 || exit 2
timeout -k 10 400 python bench.py --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/bench_full.log 2>&1 || exit 3
echo "== before (previous attention build)" >> gpurun_out/attn_bench.log
cp causal-unified-language-vision_amd/libcullavo_hip.so /tmp/lib_after.so && cp causal-unified-language-vision_amd/build/lib_before.so causal-unified-language-vision_amd/libcullavo_hip.so && timeout -k 10 200 python tools/attn_bench.py >> gpurun_out/attn_bench.log 2>&1
cp /tmp/lib_after.so causal-unified-language-vision_amd/libcullavo_hip.so
