"""How much of the data-parallel gradient exchange the backward can hide, from a 1-GPU step
(BASELINE config 3 / 4 payload): the production GradReducer runs on a world-1
RCCL group (its all-reduces are no-ops there), and a timing event is recorded on the compute
stream when each bucket's last gradient is enqueued. For each bucket: the time from its ready
point to the end of the backward (the window an all-reduce issued then can run under), and a
ring all-reduce model at N GPUs, t = 2 (N-1)/N x bytes / bus_bw. Buckets are issued in order on
one comm stream, so the exposed time is what the serialised ring finishes after the backward.

  python tools/dp_overlap.py [--gpus 8] [--bus-gbs 300] [--bucket-mb 256] [--trainable full]
"""
import argparse
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--bus-gbs", type=float, nargs="+", default=[150.0, 300.0, 600.0],
                    help="RCCL all-reduce bus bandwidth(s) to model (GB/s)")
    ap.add_argument("--bucket-mb", type=int, default=256)
    ap.add_argument("--trainable", default="full")
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    from cullavo_amd.dist import GradReducer
    from cullavo_amd.trainer import CuLLaVO_Trainer
    opt = {"MODEL": {"CONFIG": "llava-1.5-7b"}, "LLM": {"TRAINABLE": a.trainable},
           "DATA": {"BATCH_SIZE_PER_GPU": 8, "TEXT_LEN": 513, "IMAGE_COL": 35, "STEPS": a.steps + 1}}
    tr = CuLLaVO_Trainer(opt)
    tr.init_train()
    cm = tr.model.cullavo_model
    order = ["head", "layers", "lora", "embed", "projector", "vision"]
    arenas = sorted([x for x in cm.arenas.values() if x.trainable], key=lambda x: order.index(x.name))
    red = GradReducer(arenas, bucket_bytes=a.bucket_mb << 20, enabled=True)
    tr.accel.reducer = red
    batch = next(iter(tr.train_dataloaders))
    res = None
    for step in range(a.steps + 1):
        red.timing = [] if step == a.steps else None
        t0 = torch.cuda.Event(enable_timing=True)
        t_bwd0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t0.record()
        with tr.accel.accumulate(tr.model):
            red.enabled = True  # accumulate() re-derives it from the world size (1 here)
            loss = tr.model(batch, tr.accel)["loss_llm"]
            t_bwd0.record()
            loss.backward()  # no finish(): the end of the backward is the overlap window's end
            t1.record()
            red.finish()
            for ar in cm.arenas.values():
                ar.finalize_grads()
            tr.optimizer.clip_grad_norm_(10.0)
            tr.optimizer.step()
            tr.optimizer.zero_grad()
        torch.cuda.synchronize()
        if step == a.steps:
            res = (t0.elapsed_time(t_bwd0), t_bwd0.elapsed_time(t1),
                   [(bi, nb, ev.elapsed_time(t1)) for bi, nb, ev in red.timing])
    fwd_ms, bwd_ms, buckets = res
    total = sum(nb for _, nb, _ in buckets)
    out = {"workload": f"config 3 ({a.trainable} fine-tune), bucket {a.bucket_mb} MiB", "forward_ms": round(fwd_ms, 1),
           "backward_ms": round(bwd_ms, 1), "buckets": len(buckets), "payload_gb": round(total / 1e9, 3),
           "ready_before_backward_end_ms": [round(w, 1) for _, _, w in buckets], "model": []}
    N = a.gpus
    for bw in a.bus_gbs:
        t_free = 0.0  # comm stream time, ms from the backward's start
        for _, nb, window in buckets:
            ready = bwd_ms - window
            t_free = max(t_free, ready) + 2 * (N - 1) / N * nb / (bw * 1e9) * 1e3
        exposed = max(0.0, t_free - bwd_ms)
        out["model"].append({"gpus": N, "bus_gbs": bw, "comm_ms": round(2 * (N - 1) / N * total / (bw * 1e9) * 1e3, 1),
                             "exposed_ms": round(exposed, 1)})
    print(json.dumps(out, indent=1))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
