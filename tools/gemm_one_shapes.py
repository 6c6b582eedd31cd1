"""Launch the 7B step's GEMM families once each (a few repeats) for PMC passes:
fwd gate|up (0,0), dX o-proj-in (0,1, N=4096), dW qkv (1,1). Random bf16 operands.

  rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -- python tools/gemm_one_shapes.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cullavo_amd import ops  # noqa: E402

T, d, F = 8704, 4096, 11008
g = torch.Generator(device="cuda").manual_seed(0)
x = torch.randn(T, d, device="cuda", generator=g).bfloat16()
w_gu = torch.randn(2 * F, d, device="cuda", generator=g).bfloat16()
dy_gu = torch.randn(T, 2 * F, device="cuda", generator=g).bfloat16()
dy_qkv = torch.randn(T, 3 * d, device="cuda", generator=g).bfloat16()
dw = torch.empty(3 * d, d, device="cuda", dtype=torch.bfloat16)
for _ in range(int(os.environ.get("REPS", "3"))):
    ops.linear(x, w_gu)                 # fwd  gemm256_k<0, 0, 1, 256, 256, 1>
    ops.linear_dx(dy_gu, w_gu)          # dX   gemm256_k<0, 1, 1, 192, 256, 1>
    ops.linear_dw(dy_qkv, x, dw)        # dW   gemm256_k<1, 1, 1, 256, 256, 0>
torch.cuda.synchronize()
print("ok")
