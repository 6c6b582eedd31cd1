"""Cost of the LoRA dropout mask (counter hash per element) in the three GEMMs that apply it, at
the 7B q-module shapes (M = 8704 tokens, in = 4096, r = 64) and the down module (in = 11008):
u = drop(x) A^T (mask on the A operand), dA = du^T drop(x) (mask on B), dx += drop(du A) (mask in
the epilogue); p = 0.05 against p = 0 on the same launch. HIP-event timing, random bf16.

  python tools/lora_drop_bench.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cullavo_amd import ops  # noqa: E402


def timeit(fn, iters=30):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    M, r = 8704, 64
    for inf in (4096, 11008):
        x = torch.randn(M, inf, device="cuda").bfloat16()
        A = (torch.randn(r, inf, device="cuda") * 0.02).bfloat16()
        du = torch.randn(M, r, device="cuda").bfloat16()
        u = torch.empty(M, r, device="cuda", dtype=torch.bfloat16)
        gA = torch.empty(r, inf, device="cuda", dtype=torch.bfloat16)
        dx = torch.randn(M, inf, device="cuda").bfloat16()
        line = f"in={inf:5d}"
        for name, fn in [
            ("u", lambda p: ops.gemm_ex(0, 0, M, r, inf, x, inf, A, inf, u, r, drop_operand=1 if p else 0, drop_p=p, drop_seed=7)),
            ("dA", lambda p: ops.gemm_ex(1, 1, r, inf, M, du, r, x, inf, gA, inf, drop_operand=2 if p else 0, drop_p=p, drop_seed=7)),
            ("dx", lambda p: ops.gemm_ex(0, 1, M, inf, r, du, r, A, inf, dx, inf, beta=1.0, drop_operand=3 if p else 0, drop_p=p, drop_seed=7)),
        ]:
            t0 = timeit(lambda: fn(0.0))
            t1 = timeit(lambda: fn(0.05))
            line += f" | {name}: p=0 {t0:6.1f} us, p=0.05 {t1:6.1f} us"
        print(line, flush=True)


if __name__ == "__main__":
    main()
