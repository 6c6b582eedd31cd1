set -o pipefail
mkdir -p gpurun_out/r02c
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r02c/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r02c/gpu_tests.log; exit 1; }
tail -3 gpurun_out/r02c/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02c/smoke.log 2>&1 || { tail -20 gpurun_out/r02c/smoke.log; exit 3; }
tail -2 gpurun_out/r02c/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r02c/bench.log 2>&1 || { tail -20 gpurun_out/r02c/bench.log; exit 4; }
tail -1 gpurun_out/r02c/bench.log
