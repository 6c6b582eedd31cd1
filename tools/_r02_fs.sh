set -o pipefail
mkdir -p gpurun_out/r02_fs
timeout -k 10 600 python -u -m pytest tests/test_full_size.py -m gpu -x -v --timeout 500 --timeout-method thread > gpurun_out/r02_fs/tests.log 2>&1; echo "tests rc=$?"; tail -5 gpurun_out/r02_fs/tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r02_fs/bench.log 2>&1 && tail -1 gpurun_out/r02_fs/bench.log &&
timeout -k 10 300 python -u bench.py --workload vit --steps 10 --warmup 2 > gpurun_out/r02_fs/vit.log 2>&1 && tail -1 gpurun_out/r02_fs/vit.log &&
timeout -k 10 400 python -u bench.py --config llava-1.5-13b --text-len 1025 --batch 4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r02_fs/b13.log 2>&1 && tail -1 gpurun_out/r02_fs/b13.log
