"""Small-grid GEMMs (the ViT at 4 / 8 images, patch embedding, projector weight gradient): the
automatic plan (split-K on the 8-wave kernel where cullavo_gemm_plan says 9) against the forced
unsplit kernels (tile modes 0 / 2 / 3) and hipBLASLt, random bf16 operands, TFLOP/s.

  python tools/small_gemm_bench.py [--iters 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cullavo_amd import _lib, ops  # noqa: E402

SHAPES = [  # (name, M, N, K, a_layout, b_layout)
    ("vit4 qkv", 2308, 3072, 1024, 0, 0), ("vit4 out", 2308, 1024, 1024, 0, 0), ("vit4 fc1", 2308, 4096, 1024, 0, 0),
    ("vit4 fc2", 2308, 1024, 4096, 0, 0), ("patch4", 2304, 1024, 640, 0, 0), ("vit8 out", 4616, 1024, 1024, 0, 0),
    ("vit8 fc2", 4616, 1024, 4096, 0, 0), ("patch8", 4608, 1024, 640, 0, 0), ("dW proj1 b4", 5120, 1024, 2304, 1, 1),
    ("dW proj1 b8", 4096, 1024, 4608, 1, 1), ("dW proj2 b8", 4096, 4096, 4608, 1, 1)]


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    L = _lib.lib()
    g = torch.Generator(device="cuda").manual_seed(0)
    for name, M, N, K, al, bl in SHAPES:
        A = torch.randn((K, M) if al else (M, K), device="cuda", generator=g).bfloat16()
        B = torch.randn((K, N) if bl else (N, K), device="cuda", generator=g).bfloat16()
        C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        fl = 2.0 * M * N * K
        Am, Bm = (A.t() if al else A), (B if bl else B.t())
        line = f"{name:12s} {M}x{N}x{K} ({al},{bl}) plan {L.cullavo_gemm_plan(M, N, K, al, bl, None)}:"
        line += f" hipBLASLt {fl / timeit(lambda: torch.matmul(Am, Bm, out=C), a.iters) / 1e9:7.1f}"
        for mode in (-1, 0, 2, 3):
            prev = L.cullavo_gemm_set_tile(mode)
            try:
                ms = timeit(lambda: ops.gemm(al, bl, M, N, K, A, A.stride(0), B, B.stride(0), C, N), a.iters)
            finally:
                L.cullavo_gemm_set_tile(prev)
            line += f" | {'auto' if mode < 0 else 'tile' + str(mode)} {fl / ms / 1e9:7.1f}"
        print(line, flush=True)


if __name__ == "__main__":
    main()
