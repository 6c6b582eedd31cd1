"""Decode-row Linears of the 7B step at batch B: the fused input transforms of cullavo_decode_linear
(RMSNorm -> q|k|v and gate|up, SwiGLU -> down) against the unfused kernels (rmsnorm_fwd / swiglu_fwd,
then the GEMV), HIP-event timed over back-to-back launches, random bf16 operands.

  python tools/decode_linear_bench.py [--batch 1]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cullavo_amd import ops  # noqa: E402


def timeit(fn, iters=50):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1)
    a = ap.parse_args()
    B, d, F = a.batch, 4096, 11008
    g = torch.Generator(device="cuda").manual_seed(0)
    r = lambda *s: torch.randn(*s, device="cuda", generator=g).bfloat16()
    h = r(B, d)
    nw = r(d)
    gu = r(B, 2 * F)
    for name, W, mode in (("qkv", r(3 * d, d), 1), ("gate_up", r(2 * F, d), 1), ("down", r(d, F), 2)):
        nbytes = W.numel() * 2
        if mode == 1:
            unf = lambda: ops.decode_linear(ops.rmsnorm_fwd(h, nw, 1e-5)[0], W)
            fus = lambda: ops.decode_linear(h, W, transform=1, norm_w=nw, eps=1e-5)
        else:
            unf = lambda: ops.decode_linear(ops.swiglu_fwd(gu), W)
            fus = lambda: ops.decode_linear(gu, W, transform=2)
        plain = lambda: ops.decode_linear(h if mode == 1 else gu[:, :F].contiguous(), W)
        for tag, fn in (("unfused", unf), ("fused", fus), ("gemv only", plain), ("unfused", unf), ("fused", fus)):
            us = timeit(fn)
            print(f"{name:8s} B={B} {tag:9s} {us:8.2f} us  {nbytes / us / 1e3:7.1f} GB/s (weights)", flush=True)


if __name__ == "__main__":
    main()
