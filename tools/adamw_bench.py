"""AdamW kernel bandwidth (bf16 p, g, m, v: 14 B per element) on a 1.5 G-element arena slice,
HIP-event timing.

  python tools/adamw_bench.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cullavo_amd import ops  # noqa: E402

n = 1536 * 1024 * 1024
p, g, m, v = (torch.randn(n, device="cuda", dtype=torch.bfloat16) * 0.01 for _ in range(4))
v.abs_()
sc = torch.ones(1, device="cuda")
for _ in range(2):
    ops.adamw(p, g, m, v, lr=1e-5, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0, step=1, grad_scale=sc)
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(10):
    ops.adamw(p, g, m, v, lr=1e-5, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0, step=1, grad_scale=sc)
e.record()
e.synchronize()
ms = s.elapsed_time(e) / 10
print(f"adamw n={n} {ms:.3f} ms {14 * n / ms / 1e6:.0f} GB/s", flush=True)
