"""Decode GEMV variants (CULLAVO_GEMV, read once per process) on the 7B decode step's Linear shapes:
Y[B, N] = X[B, K] W[N, K]^T through ops.linear (gemm plan 14), HIP-event timed over back-to-back
launches of a rotating set of weight copies (total > 256 MB, so the MALL does not hold them).

  CULLAVO_GEMV=4 python tools/gemv_variant_bench.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cullavo_amd import ops  # noqa: E402


def main():
    v = os.environ.get("CULLAVO_GEMV", "default")
    g = torch.Generator(device="cuda").manual_seed(0)
    for B in (1, 8):
        for name, N, K in (("qkv", 12288, 4096), ("o", 4096, 4096), ("gate_up", 22016, 4096),
                           ("down", 4096, 11008), ("lm_head", 32064, 4096)):
            copies = max(2, -(-600_000_000 // (N * K * 2)))
            Ws = [torch.randn(N, K, device="cuda", generator=g).bfloat16() for _ in range(copies)]
            x = torch.randn(B, K, device="cuda", generator=g).bfloat16()
            for w in Ws[:2]:
                ops.linear(x, w)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            it = 6 * copies
            s.record()
            for i in range(it):
                ops.linear(x, Ws[i % copies])
            e.record()
            e.synchronize()
            us = s.elapsed_time(e) / it * 1e3
            print(f"gemv {v:7s} B={B} {name:8s} {us:8.2f} us  {N * K * 2 / us / 1e3:7.1f} GB/s", flush=True)
            del Ws


if __name__ == "__main__":
    main()
