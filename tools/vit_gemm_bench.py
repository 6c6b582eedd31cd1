"""The CLIP ViT-L/14-336 encoder's GEMMs at config 2 (bs 64: M = 64 x 577 = 36928 tokens, d 1024,
ffn 4096) with their fused epilogues, per tile mode and epilogue path. HIP-event timing, random
bf16 operands.

  python tools/vit_gemm_bench.py [--modes -1,2,3,0] [--tokens 36928]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cullavo_amd import _lib, ops  # noqa: E402
from cullavo_amd.ops import ACT_QUICK_GELU  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="-1,2,3,0")
    ap.add_argument("--tokens", type=int, default=64 * 577)
    a = ap.parse_args()
    T = a.tokens
    g = torch.Generator(device="cuda").manual_seed(0)
    L = _lib.lib()

    def rnd(*s, scale=1.0):
        return (torch.randn(*s, device="cuda", generator=g) * scale).bfloat16()
    x1k, x4k = rnd(T, 1024), rnd(T, 4096)
    wq, wo, w1, w2 = rnd(3072, 1024, scale=1 / 32), rnd(1024, 1024, scale=1 / 32), rnd(4096, 1024, scale=1 / 32), \
        rnd(1024, 4096, scale=1 / 64)
    bq, bo, b1, b2 = rnd(3072), rnd(1024), rnd(4096), rnd(1024)
    res = rnd(T, 1024)
    cases = [
        ("qkv+bias", 3072, 1024, lambda: ops.linear(x1k, wq, bq)),
        ("out+bias+res", 1024, 1024, lambda: ops.linear(x1k, wo, bo, residual=res)),
        ("fc1 plain", 4096, 1024, lambda: ops.linear(x1k, w1)),
        ("fc1+bias", 4096, 1024, lambda: ops.linear(x1k, w1, b1)),
        ("fc1+bias+qgelu", 4096, 1024, lambda: ops.linear(x1k, w1, b1, act=ACT_QUICK_GELU)),
        ("fc2+bias+res", 1024, 4096, lambda: ops.linear(x4k, w2, b2, residual=res)),
    ]
    for name, N, K, fn in cases:
        fl = 2.0 * T * N * K
        line = f"{name:16s} {T}x{N}x{K}"
        for mode in [int(m) for m in a.modes.split(",")]:
            prev = L.cullavo_gemm_set_tile(mode)
            for epi in (1, 0):
                pe = L.cullavo_gemm_set_epilogue(epi)
                ms = timeit(fn)
                L.cullavo_gemm_set_epilogue(pe)
                line += f" | m{mode}{'' if epi else 'L'} {fl / ms / 1e9:6.1f}"
            L.cullavo_gemm_set_tile(prev)
        print(line, flush=True)


if __name__ == "__main__":
    main()
