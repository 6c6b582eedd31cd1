"""BASELINE config 2: CLIP ViT-L/14-336 encoder forward at bs=64 on one MI355X (SURVEY.md §8(d):
366.0 GFLOP/img for the 23 layers hidden_states[-2] needs plus the patch embedding; 60 % of the
bf16 roofline = 4100 img/s). Synthetic N(0,1) pixels, random-init weights. One JSON line.

  python tools/vit_bench.py [--batch 64] [--steps 10] [--warmup 3]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args()
    from cullavo_amd.arch_cullavo import CuLLaVOModel
    from cullavo_amd.config import llava_1_5_7b
    from cullavo_amd.perf import flops_per_sample
    cfg = llava_1_5_7b()
    m = CuLLaVOModel(cfg, device="cuda", trainable="none", init="random", seed=0)
    m.eval()
    v = cfg.vision_config
    g = torch.Generator(device="cuda").manual_seed(1234)
    pix = torch.randn(a.batch, 3, v.image_size, v.image_size, generator=g, device="cuda").to(torch.bfloat16)
    vt = m.vision_tower.vision_model
    n = v.num_hidden_layers + 1 + cfg.vision_feature_layer  # hidden_states[-2]: 23 layers
    with torch.no_grad():
        for _ in range(a.warmup):
            feats = vt.hidden_state(pix, n)[:, 1:]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            feats = vt.hidden_state(pix, n)[:, 1:]
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
    gf = flops_per_sample(cfg, 513)["vit"]
    print(json.dumps({"metric": "ViT-L/14-336 encoder forward images/sec (BASELINE config 2)",
                      "value": round(a.batch / dt, 1), "unit": "img/s", "batch": a.batch,
                      "ms_per_batch": round(dt * 1e3, 3), "gflop_per_img": round(gf / 1e9, 1),
                      "tflops": round(gf * a.batch / dt / 1e12, 1), "frac_of_2.5PF": round(gf * a.batch / dt / 2.5e15, 4),
                      "out_shape": list(feats.shape), "dtype": "bf16", "data": "synthetic"}))


if __name__ == "__main__":
    main()
