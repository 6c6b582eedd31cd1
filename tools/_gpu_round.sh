set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_generation.py -x -q -m gpu > gpurun_out/gen_tests.log 2>&1
echo "rc=$?" >> gpurun_out/gen_tests.log
