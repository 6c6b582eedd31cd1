set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_ops_gpu.py -x -q -k "attn or attention" > gpurun_out/ops_tests.log 2>&1 || exit 1
timeout -k 10 300 python -m pytest tests/test_model_gpu.py -x -q > gpurun_out/model_tests.log 2>&1 || exit 1
timeout -k 10 200 python tools/attn_bench.py > gpurun_out/attn_bench.log 2>&1 || exit 2
echo "== before" >> gpurun_out/attn_bench.log
cp causal-unified-language-vision_amd/libcullavo_hip.so /tmp/lib_after.so && cp causal-unified-language-vision_amd/build/lib_before.so causal-unified-language-vision_amd/libcullavo_hip.so && timeout -k 10 200 python tools/attn_bench.py >> gpurun_out/attn_bench.log 2>&1
cp /tmp/lib_after.so causal-unified-language-vision_amd/libcullavo_hip.so
