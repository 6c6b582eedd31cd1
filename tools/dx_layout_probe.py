"""dX layout study: dx = dy @ W with W [N,K] read N-contiguous (gemm mode (0,1), today's
linear_dx) against the same product from a transposed copy Wt [K,N] (mode (0,0), both operands
reduction-contiguous), plus the cost of producing Wt. Prints TF/s and bitwise equality."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cullavo_amd import ops  # noqa: E402

SHAPES = [("qkv", 8704, 12288, 4096), ("o", 8704, 4096, 4096), ("gate_up", 8704, 22016, 4096),
          ("down", 8704, 4096, 11008), ("lm_head", 8704, 32064, 4096)]


def timeit(fn, reps=10):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


g = torch.Generator(device="cuda").manual_seed(0)
for name, T, N, K in SHAPES:
    w = torch.randn(N, K, device="cuda", generator=g).bfloat16()
    dy = torch.randn(T, N, device="cuda", generator=g).bfloat16()
    wt = torch.empty(K, N, device="cuda", dtype=torch.bfloat16)
    a = torch.empty(T, K, device="cuda", dtype=torch.bfloat16)
    b = torch.empty(T, K, device="cuda", dtype=torch.bfloat16)
    tr = getattr(ops, "transpose2d", None)
    mk = (lambda: tr(w, wt)) if tr else (lambda: wt.copy_(w.t()))
    mk()
    t01 = timeit(lambda: ops.gemm(0, 1, T, K, N, dy, N, w, K, a, K))
    t00 = timeit(lambda: ops.gemm(0, 0, T, K, N, dy, N, wt, N, b, K))
    ttr = timeit(mk)
    fl = 2.0 * T * N * K
    print(f"{name:8s} dx (0,1) {t01 * 1e3:8.1f} us {fl / t01 / 1e9:7.1f} TF | (0,0)+Wt {t00 * 1e3:8.1f} us "
          f"{fl / t00 / 1e9:7.1f} TF | transpose {ttr * 1e3:7.1f} us {4.0 * N * K / ttr / 1e6:6.0f} GB/s | "
          f"bitwise {torch.equal(a, b)}", flush=True)
