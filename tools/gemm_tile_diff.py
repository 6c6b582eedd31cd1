"""Bitwise comparison of the GEMM kernel shapes (cullavo_gemm_set_tile) on the ViT-L / 7B shapes
with the production epilogues (bias + quick_gelu, bias + residual): prints max |diff| between
each forced tile mode and the 256x256 kernel (0 = bitwise equal)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cullavo_amd import _lib, ops  # noqa: E402

L = _lib.lib()
g = torch.Generator(device="cuda").manual_seed(0)
for (M, N, K, epi) in [(36928, 4096, 1024, "qg"), (36928, 1024, 4096, "res"), (36928, 3072, 1024, "b"),
                       (1154, 4096, 1024, "qg"), (8704, 4096, 4096, "res"), (2000, 4096, 1024, "qg")]:
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) * 0.03).bfloat16()
    b = torch.randn(N, device="cuda", generator=g).bfloat16()
    r = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    outs = {}
    for tile in (2, 10, 3, 0, -1):
        prev = L.cullavo_gemm_set_tile(tile)
        if epi == "qg":
            y = ops.linear(x, w, b, act=ops.ACT_QUICK_GELU)
        elif epi == "res":
            y = ops.linear(x, w, b, residual=r)
        else:
            y = ops.linear(x, w, b)
        torch.cuda.synchronize()
        L.cullavo_gemm_set_tile(prev)
        outs[tile] = y
    ref = outs[2].float()
    print(f"{M}x{N}x{K} {epi}: plan {L.cullavo_gemm_plan(M, N, K, 0, 0, None)} | " +
          " | ".join(f"t{t} {(o.float() - ref).abs().max().item():.3e}" for t, o in outs.items()), flush=True)
