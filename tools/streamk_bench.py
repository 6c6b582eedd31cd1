"""The 7B step's GEMM shapes with the stream-K tail off (0) and forced (2), HIP-event timing,
interleaved rounds in one process, random bf16 operands.

  python tools/streamk_bench.py [--rounds 3] [--iters 10]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cullavo_amd import _lib, ops  # noqa: E402

T = 8704
SHAPES = []
for name, n, k in (("qkv", 12288, 4096), ("o", 4096, 4096), ("gate_up", 22016, 4096), ("down", 4096, 11008),
                   ("lm_head", 32064, 4096)):
    SHAPES += [(f"{name} fwd", T, n, k, 0, 0), (f"{name} dX", T, k, n, 0, 1), (f"{name} dW", n, k, T, 1, 1)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    g = torch.Generator(device="cuda").manual_seed(0)
    L = _lib.lib()
    for name, M, N, K, al, bl in SHAPES:
        A = torch.randn((K, M) if al else (M, K), device="cuda", generator=g).bfloat16()
        B = torch.randn((K, N) if bl else (N, K), device="cuda", generator=g).bfloat16()
        C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        grid = ctypes_grid = None
        best = {0: 0.0, 2: 0.0}
        for _ in range(a.rounds):
            for mode in (0, 2):
                prev = L.cullavo_gemm_set_streamk(mode)
                ops.gemm(al, bl, M, N, K, A, A.stride(0), B, B.stride(0), C, N)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(a.iters):
                    ops.gemm(al, bl, M, N, K, A, A.stride(0), B, B.stride(0), C, N)
                e.record()
                e.synchronize()
                L.cullavo_gemm_set_streamk(prev)
                best[mode] = max(best[mode], 2.0 * M * N * K / (s.elapsed_time(e) / a.iters * 1e-3) / 1e12)
        del A, B, C, grid, ctypes_grid
        print(f"{name:14s} {M}x{N}x{K} ({al},{bl})  dp {best[0]:7.1f}  sk {best[2]:7.1f} TF/s  {100 * (best[2] / best[0] - 1):+5.1f} %",
              flush=True)


if __name__ == "__main__":
    main()
