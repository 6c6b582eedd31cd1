set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 200 python tools/imageprep_bench.py > gpurun_out/imageprep_bench.log 2>&1 || { cat gpurun_out/imageprep_bench.log; exit 2; }
cat gpurun_out/imageprep_bench.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 3; }
tail -2 gpurun_out/smoke.log
