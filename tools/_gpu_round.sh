set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_generation.py tests/test_lora.py -x -q -m gpu > gpurun_out/gen_tests.log 2>&1 || exit 1
timeout -k 10 400 python tools/decode_bench.py --batch 1 --new 32 > gpurun_out/decode_b1.log 2>&1 || exit 2
timeout -k 10 400 python tools/decode_bench.py --batch 8 --new 32 > gpurun_out/decode_b8.log 2>&1 || exit 3
