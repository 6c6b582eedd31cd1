set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_ops_gpu.py -x -q -k "gemm or linear or rmsnorm or layernorm" > gpurun_out/gemm_tests.log 2>&1 || exit 1
timeout -k 10 300 python -m pytest tests/test_model_gpu.py -x -q > gpurun_out/model_tests.log 2>&1 || exit 1
timeout -k 10 120 python tools/norm_bench.py > gpurun_out/norm_bench.log 2>&1 || exit 2
rm -f gpurun_out/spread.log
for sp in 0 1 0 1; do
  echo "== spread $sp" >> gpurun_out/spread.log
  CULLAVO_GEMM_SPREAD=$sp timeout -k 10 300 python tools/gemm_bench.py --modes 2,3 --iters 10 >> gpurun_out/spread.log 2>&1 || exit 3
done
