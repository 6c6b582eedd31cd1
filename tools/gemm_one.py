"""One GEMM kind (fwd / dx / dw of a Linear) under a forced kernel shape, repeated, for PMC
comparison of kernel variants: python tools/gemm_one.py T out in mode kind [reps]."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cullavo_amd import _lib, ops  # noqa: E402

T, out_f, in_f, mode = (int(v) for v in sys.argv[1:5])
kind = sys.argv[5]
reps = int(sys.argv[6]) if len(sys.argv) > 6 else 5
_lib.lib().cullavo_gemm_set_tile(mode)
g = torch.Generator(device="cuda").manual_seed(0)
x = torch.randn(T, in_f, device="cuda", generator=g).bfloat16()
w = torch.randn(out_f, in_f, device="cuda", generator=g).bfloat16()
dy = torch.randn(T, out_f, device="cuda", generator=g).bfloat16()
dw = torch.empty(out_f, in_f, device="cuda", dtype=torch.bfloat16)
run = {"fwd": lambda: ops.linear(x, w), "dx": lambda: ops.linear_dx(dy, w),
       "dw": lambda: ops.linear_dw(dy, x, dw)}[kind]
for _ in range(reps):
    run()
torch.cuda.synchronize()
