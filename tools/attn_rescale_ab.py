"""A/B of the attention forward's deferred rescale (cullavo_attn_set_rescale): threshold 0 (the
plain online softmax: rescale whenever a row max grows) vs 8 (default), interleaved rounds in
one process, random bf16 inputs, on the 7B layer (B 8, H 32, L 1088, D 128, causal) and the
ViT-L layer at bs 64 (H 16, L 577, D 64, non-causal). Prints us per call and TFLOP/s.

  python tools/attn_rescale_ab.py [--iters 20] [--rounds 3]
"""
import argparse
import ctypes
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cullavo_amd import _lib, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    L_ = _lib.lib()
    g = torch.Generator(device="cuda").manual_seed(0)
    for name, B, H, L, D, causal in (("7B layer", 8, 32, 1088, 128, True), ("ViT-L bs64", 64, 16, 577, 64, False)):
        q, k, v = (torch.randn(B * L, H * D, device="cuda", generator=g).bfloat16() for _ in range(3))
        kw = dict(B=B, H=H, Lq=L, Lk=L, D=D, scale=D ** -0.5, causal=causal)
        fl = 4.0 * B * H * L * L * D * (0.5 if causal else 1.0)
        res = {0.0: [], 8.0: []}
        for _ in range(200):  # clocks up to the sustained level before timing
            ops.attn_fwd(q, k, v, **kw)
        for _ in range(a.rounds):
            for thr in res:
                L_.cullavo_attn_set_rescale(ctypes.c_float(thr), None)
                ops.attn_fwd(q, k, v, **kw)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(a.iters):
                    ops.attn_fwd(q, k, v, **kw)
                e.record()
                e.synchronize()
                res[thr].append(s.elapsed_time(e) / a.iters * 1e3)
        L_.cullavo_attn_set_rescale(ctypes.c_float(8.0), None)
        line = f"{name:11s}"
        for thr, us in res.items():
            m = statistics.median(us)
            line += f" | threshold {thr:4.1f}: {m:7.1f} us {fl / (m * 1e-6) / 1e12:6.1f} TF/s"
        print(line, flush=True)


if __name__ == "__main__":
    main()
