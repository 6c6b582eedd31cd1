"""The down-projection dX GEMM with the SwiGLU backward in its epilogue (8704 x 11008 x 4096,
layouts (0,1), act 3) against the same product plain, and the prefetching
SwiGLU instantiation (default) against the general rolled path (cullavo_gemm_set_epilogue bit 6).
Interleaved rounds in one process, HIP-event timing, random bf16 operands; also checks the two
SwiGLU paths bitwise.

  python tools/swiglu_dx_bench.py [--rounds 5]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cullavo_amd import _lib, ops  # noqa: E402


def timeit(fn, iters=20):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    T, F, d = 8704, 11008, 4096
    g = torch.Generator(device="cuda").manual_seed(0)
    dy = torch.randn(T, d, device="cuda", generator=g).bfloat16()
    w = (torch.randn(d, F, device="cuda", generator=g) * d ** -0.5).bfloat16()  # down_proj.weight [d, F]
    gu = torch.randn(T, 2 * F, device="cuda", generator=g).bfloat16()
    L = _lib.lib()
    fl = 2.0 * T * F * d
    base = L.cullavo_gemm_set_epilogue(1)
    L.cullavo_gemm_set_epilogue(base)

    def swg():
        return ops.linear_dx(dy, w, swiglu_gu=gu)

    def plain():
        return ops.linear_dx(dy, w)

    outs = {}
    res = {"swiglu_prefetch": [], "swiglu_general": [], "plain": []}
    for r in range(a.rounds):
        for name in res:
            L.cullavo_gemm_set_epilogue(base | 64 if name == "swiglu_general" else base)
            fn = plain if name == "plain" else swg
            if r == 0:
                outs[name] = fn().clone()
            res[name].append(fl / (timeit(fn) * 1e-3) / 1e12)
    L.cullavo_gemm_set_epilogue(base)
    same = torch.equal(outs["swiglu_prefetch"], outs["swiglu_general"])
    for name, v in res.items():
        print(f"{name:16s} {T}x{F}x{d}: median {statistics.median(v):7.1f} TF/s  (min {min(v):7.1f}, max {max(v):7.1f})")
    print(f"prefetch == general bitwise: {same}")


if __name__ == "__main__":
    main()
