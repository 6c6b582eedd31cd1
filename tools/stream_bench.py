"""The step's streaming elementwise kernels at config-3 shapes (T = 8704 tokens, F = 11008):
SwiGLU fwd / bwd, RoPE, AdamW on a 1.6 G-element slice; HIP-event timing, HBM GB/s.

  python tools/stream_bench.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cullavo_amd import ops  # noqa: E402


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


T, d, F = 8704, 4096, 11008
gu = torch.randn(T, 2 * F, device="cuda").bfloat16()
da = torch.randn(T, F, device="cuda").bfloat16()
q = torch.randn(T, d, device="cuda").bfloat16()
k = torch.randn(T, d, device="cuda").bfloat16()
pos = torch.arange(1088, device="cuda").repeat(8)
n = 1536 * 1024 * 1024
p, g, m, v = (torch.randn(n, device="cuda", dtype=torch.bfloat16) * 0.01 for _ in range(4))
v.abs_()
sc = torch.ones(1, device="cuda")
for name, fn, nbytes in [
    ("swiglu_fwd", lambda: ops.swiglu_fwd(gu), 3 * T * F * 2),
    ("swiglu_bwd", lambda: ops.swiglu_bwd(da, gu), 5 * T * F * 2),
    ("rope", lambda: ops.rope(q, k, pos, hq=32, hk=32, head_dim=128, theta=10000.0), 4 * T * d * 2),
    ("adamw", lambda: ops.adamw(p, g, m, v, lr=1e-5, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0, step=1,
                                grad_scale=sc), 14 * n),
]:
    ms = timeit(fn, 10 if name == "adamw" else 20)
    print(f"{name:11s} {ms * 1e3:8.1f} us {nbytes / ms / 1e6:7.0f} GB/s", flush=True)
