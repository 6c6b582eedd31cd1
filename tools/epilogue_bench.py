"""Cost of the fused epilogues on the decoder's N=4096 forward GEMMs (o_proj K=4096, down
K=11008; M = 8704 tokens): plain vs + residual (the step's form) vs + residual + LoRA addend.
HIP-event timing, random bf16 operands.

  python tools/epilogue_bench.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cullavo_amd import _lib, ops  # noqa: E402


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


T = 8704
g = torch.Generator(device="cuda").manual_seed(0)
for name, N, K in (("o_proj", 4096, 4096), ("down", 4096, 11008), ("qkv", 12288, 4096)):
    x = torch.randn(T, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).bfloat16()
    r = torch.randn(T, N, device="cuda", generator=g).bfloat16()
    t = torch.randn(T, N, device="cuda", generator=g).bfloat16()
    y = torch.empty(T, N, device="cuda", dtype=torch.bfloat16)
    fl = 2.0 * T * N * K
    line = f"{name:7s} {T}x{N}x{K}"
    for label, fn in (("plain", lambda: ops.linear(x, w, out=y)),
                      ("+res", lambda: ops.linear(x, w, residual=r, out=y)),
                      ("+res+add", lambda: ops.linear(x, w, residual=r, addend=t, out=y))):
        for epi in (1, 0):
            prev = _lib.lib().cullavo_gemm_set_epilogue(epi)
            ms = timeit(fn)
            _lib.lib().cullavo_gemm_set_epilogue(prev)
            line += f" | {label}{'' if epi else '(lane)'} {fl / ms / 1e9:7.1f} TF"
    print(line, flush=True)
