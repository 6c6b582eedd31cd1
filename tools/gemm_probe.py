"""Run one GEMM shape in the three layouts (fwd / dx / dw) under a forced kernel shape, for
PMC-counter comparison under rocprofv3 (one dispatch kind per layout)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cullavo_amd import _lib, ops  # noqa: E402

T, out_f, in_f = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
mode = int(sys.argv[4]) if len(sys.argv) > 4 else 2
_lib.lib().cullavo_gemm_set_tile(mode)
g = torch.Generator(device="cuda").manual_seed(0)
x = torch.randn(T, in_f, device="cuda", generator=g).bfloat16()
w = torch.randn(out_f, in_f, device="cuda", generator=g).bfloat16()
dy = torch.randn(T, out_f, device="cuda", generator=g).bfloat16()
dw = torch.empty(out_f, in_f, device="cuda", dtype=torch.bfloat16)
for _ in range(5):
    ops.linear(x, w)
    ops.linear_dx(dy, w)
    ops.linear_dw(dy, x, dw)
torch.cuda.synchronize()
wT = w.T.contiguous()
for _ in range(5):
    ops.linear(dy, wT)  # dx through the K-contiguous (0,0) path on a transposed weight copy
torch.cuda.synchronize()
