"""Probe: can two ranks share one GPU over RCCL (torch.distributed "nccl")? Launched as
python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 tools/probe/rccl_two_ranks_one_gpu.py
Prints the all-reduced value per rank or the error."""
import os

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
try:
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    x = torch.full((4,), float(rank + 1), device="cuda")
    dist.all_reduce(x)
    torch.cuda.synchronize()
    print(f"rank {rank}: all_reduce -> {x.tolist()}", flush=True)
    dist.destroy_process_group()
except Exception as e:  # noqa: BLE001
    print(f"rank {rank}: {type(e).__name__}: {str(e)[:300]}", flush=True)
