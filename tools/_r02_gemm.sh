set -o pipefail
mkdir -p gpurun_out/r02_gemm
true
timeout -k 10 600 python -u tools/gemm_bench.py --iters 10 --modes=-1,-1N,-1,-1N > gpurun_out/r02_gemm/bench.log 2>&1; cat gpurun_out/r02_gemm/bench.log | grep -v amdgpu.ids
