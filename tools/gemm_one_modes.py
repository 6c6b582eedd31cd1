"""Launch a few 7B-step GEMM shapes under the given tile modes (a few repeats each) for PMC passes:
dW qkv (1,1), fwd gate|up (0,0), dX gate|up (0,1). Random N(0,1) bf16 operands.

  rocprofv3 --pmc ... -- python tools/gemm_one_modes.py [modes, default -1,12]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cullavo_amd import _lib, ops  # noqa: E402

T, d, F = 8704, 4096, 11008
modes = [int(m) for m in (sys.argv[1] if len(sys.argv) > 1 else "-1,12").split(",")]
g = torch.Generator(device="cuda").manual_seed(0)
x = torch.randn(T, d, device="cuda", generator=g).bfloat16()
w_gu = torch.randn(2 * F, d, device="cuda", generator=g).bfloat16()
dy_gu = torch.randn(T, 2 * F, device="cuda", generator=g).bfloat16()
dy_qkv = torch.randn(T, 3 * d, device="cuda", generator=g).bfloat16()
dw = torch.empty(3 * d, d, device="cuda", dtype=torch.bfloat16)
lib = _lib.lib()
for mode in modes:
    prev = lib.cullavo_gemm_set_tile(mode)
    for _ in range(int(os.environ.get("REPS", "2"))):
        ops.linear_dw(dy_qkv, x, dw)
        ops.linear(x, w_gu)
        ops.linear_dx(dy_gu, w_gu)
    torch.cuda.synchronize()
    lib.cullavo_gemm_set_tile(prev)
print("ok")
