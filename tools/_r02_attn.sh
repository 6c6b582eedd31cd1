set -o pipefail
mkdir -p gpurun_out/r02_attn
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_parity_modes.py -m gpu -x -q -k "attention or attn" --timeout 300 --timeout-method thread > gpurun_out/r02_attn/tests.log 2>&1; rc=$?; tail -3 gpurun_out/r02_attn/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r02_attn/tests.log | head -20; exit 1; }
timeout -k 10 300 python -u tools/attn_bench.py > gpurun_out/r02_attn/bench.log 2>&1; grep -v amdgpu.ids gpurun_out/r02_attn/bench.log
