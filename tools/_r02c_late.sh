set -e
mkdir -p gpurun_out/late
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q -m gpu -k "epilogue" --timeout 200 --timeout-method thread > gpurun_out/late/epi_tests.log 2>&1 || { tail -30 gpurun_out/late/epi_tests.log; exit 1; }
tail -2 gpurun_out/late/epi_tests.log
timeout -k 10 200 python tools/vit_gemm_bench.py --modes=-1 > gpurun_out/late/vit_gemm.log 2>&1
cat gpurun_out/late/vit_gemm.log
timeout -k 10 200 python bench.py --workload vit --no-cpu-baseline > gpurun_out/late/bench_vit.log 2>&1
tail -1 gpurun_out/late/bench_vit.log | cut -c1-300
bash tools/_prio_ab.sh
bash tools/_dp_rehearsal.sh
