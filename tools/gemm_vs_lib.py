"""This library's GEMM and hipBLASLt (torch.matmul) on the same problem, same layouts, same random
bf16 operands, alternating in one process: the workload for a PMC / kernel-trace comparison of the
two kernels (VERDICT r04 "Next round" item 2, step 1).

  python tools/gemm_vs_lib.py [shape ...] [--reps N]
  shape = fwd:M:N:K (Y = X W^T, both K-contiguous) | dw:M:N:K (dW = dY^T X) | dx:M:N:K (dX = dY W)
Prints per shape and kernel the mean time and TFLOP/s over the timed launches (HIP events).
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cullavo_amd import _lib, ops  # noqa: E402

DEFAULT = ["fwd:8704:22016:4096", "fwd:8704:32064:4096", "dw:22016:4096:8704", "dx:8704:4096:11008"]


def problem(kind, M, N, K, g):
    """(ours, lib) closures computing the same M x N product"""
    if kind == "fwd":  # x [M, K], w [N, K]
        x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
        w = torch.randn(N, K, device="cuda", generator=g).bfloat16()
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        return (lambda: ops.gemm(0, 0, M, N, K, x, K, w, K, c, N)), (lambda: torch.matmul(x, w.t(), out=c)), c
    if kind == "dw":  # dy [K, M] (tokens x out), x [K, N] -> dW [M, N]
        dy = torch.randn(K, M, device="cuda", generator=g).bfloat16()
        x = torch.randn(K, N, device="cuda", generator=g).bfloat16()
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        return (lambda: ops.gemm(1, 1, M, N, K, dy, M, x, N, c, N)), (lambda: torch.matmul(dy.t(), x, out=c)), c
    if kind == "dx":  # dy [M, K], w [K, N] -> dX [M, N]
        dy = torch.randn(M, K, device="cuda", generator=g).bfloat16()
        w = torch.randn(K, N, device="cuda", generator=g).bfloat16()
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        return (lambda: ops.gemm(0, 1, M, N, K, dy, K, w, N, c, N)), (lambda: torch.matmul(dy, w, out=c)), c
    raise ValueError(kind)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("shapes", nargs="*", default=DEFAULT)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--modes", default="-1", help="this library's tile modes to time (cullavo_gemm_set_tile)")
    a = ap.parse_args()
    g = torch.Generator(device="cuda").manual_seed(0)
    for spec in a.shapes:
        kind, M, N, K = spec.split(":")
        M, N, K = int(M), int(N), int(K)
        ours, lib, c = problem(kind, M, N, K, g)
        L = _lib.lib()
        modes = [int(m) for m in a.modes.split(",")]

        def forced(mode):
            def run():
                prev = L.cullavo_gemm_set_tile(mode)
                ours()
                L.cullavo_gemm_set_tile(prev)
            return run
        runs = [(f"t{m}", forced(m)) for m in modes] + [("hipblaslt", lib)]
        res = {name: [] for name, _ in runs}
        for _ in range(a.rounds):
            for name, fn in runs:
                fn()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(a.reps):
                    fn()
                e.record()
                e.synchronize()
                res[name].append(s.elapsed_time(e) / a.reps)
        lib()
        ref = c.float().clone()
        errs = {}
        for name, fn in runs[:-1]:
            c.fill_(float("nan"))
            fn()
            errs[name] = ((c.float() - ref).norm() / ref.norm()).item()
        fl = 2.0 * M * N * K
        print(f"{spec:24s} err vs hipBLASLt " + " ".join(f"{n} {e:.1e}" for n, e in errs.items()), flush=True)
        print(f"{spec:24s} " + " | ".join(
            f"{n} {min(v) * 1e3:8.1f} us {fl / (min(v) * 1e-3) / 1e12:7.1f} TF/s" for n, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
