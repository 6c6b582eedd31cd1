# bench.py's N>1 path rehearsed on ONE GPU: two ranks sharing the card over gloo (the driver's
# 8-GPU scaling run uses RCCL, one rank per GPU; this checks the launcher/env/timing/JSON path)
set -e
mkdir -p gpurun_out/dp2
CULLAVO_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 2 --warmup 1 --batch 4 --no-cpu-baseline \
  > gpurun_out/dp2/bench_dp2_gloo.log 2>&1
tail -1 gpurun_out/dp2/bench_dp2_gloo.log | cut -c1-600
