"""Is the frozen vision tower of the config-3 step launch-bound? Times the 23-layer CLIP ViT-L/14-336
forward at B images (default 8, the step's batch) eagerly (wall clock with a sync, and the host
time to enqueue it) and as one captured HIP graph replay. Random-init weights, random pixels.

  python tools/vit_graph_probe.py [--batch 8] [--iters 20]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cullavo_amd.arena import ParamArena  # noqa: E402
from cullavo_amd.config import CLIPVisionConfig, CuLLaVOConfig  # noqa: E402
from cullavo_amd.modeling import CLIPVisionTransformer, clip_specs, init_random_  # noqa: E402
from cullavo_amd.perf import needed_vision_layers  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    vc = CLIPVisionConfig()
    cfg = CuLLaVOConfig(vision_config=vc)
    ar = ParamArena("vision", clip_specs(vc, "vision_tower.vision_model."), device="cuda")
    init_random_({"vision": ar}, seed=0)
    vt = CLIPVisionTransformer(vc, ar.params, "vision_tower.vision_model.", ar)
    n = needed_vision_layers(cfg)
    g = torch.Generator(device="cuda").manual_seed(1)
    pix = torch.randn(a.batch, 3, vc.image_size, vc.image_size, device="cuda", generator=g)
    with torch.no_grad():
        for _ in range(3):
            ref = vt.hidden_state(pix, n)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        enq = 0.0
        for _ in range(a.iters):
            t1 = time.perf_counter()
            vt.hidden_state(pix, n)
            enq += time.perf_counter() - t1
            torch.cuda.synchronize()
        eager = (time.perf_counter() - t0) / a.iters
        # back-to-back (queue kept full by the previous iterations)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            vt.hidden_state(pix, n)
        torch.cuda.synchronize()
        b2b = (time.perf_counter() - t0) / a.iters

        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                vt.hidden_state(pix, n)
        torch.cuda.current_stream().wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            out = vt.hidden_state(pix, n)
        graph.replay()
        torch.cuda.synchronize()
        same = torch.equal(out, ref)
        t0 = time.perf_counter()
        for _ in range(a.iters):
            graph.replay()
            torch.cuda.synchronize()
        replay = (time.perf_counter() - t0) / a.iters
    print(f"ViT-L/14-336 x{n} layers, B={a.batch}: eager {eager * 1e3:.3f} ms (host enqueue {enq / a.iters * 1e3:.3f} ms), "
          f"back-to-back {b2b * 1e3:.3f} ms, graph replay {replay * 1e3:.3f} ms, graph output bitwise equal: {same}",
          flush=True)


if __name__ == "__main__":
    main()
