"""The small-grid GEMMs of the config-3 step (CLIP ViT-L/14-336 forward at B = 8 images:
M = 8 x 577 = 4616 tokens, d 1024, ffn 4096; projector M = 8 x 576) with their fused epilogues,
through each dispatch the library offers: the default tile choice, split-K (gemm_ex with a
workspace), and the 256x256 / 192x256 kernels with a stream-K tail. HIP-event timing, random bf16.

  python tools/vit_step_gemm_bench.py [--tokens 4616]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cullavo_amd import _lib, ops  # noqa: E402
from cullavo_amd.ops import ACT_GELU, ACT_QUICK_GELU  # noqa: E402


def timeit(fn, iters=30):
    for _ in range(3):
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
    ap.add_argument("--tokens", type=int, default=8 * 577)
    a = ap.parse_args()
    T = a.tokens
    P = T - T // 577  # projector rows: the CLS rows dropped
    g = torch.Generator(device="cuda").manual_seed(0)
    L = _lib.lib()

    def rnd(*s, scale=1.0):
        return (torch.randn(*s, device="cuda", generator=g) * scale).bfloat16()
    x1k, x4k = rnd(T, 1024), rnd(T, 4096)
    p1k, p4k = rnd(P, 1024), rnd(P, 4096)
    wq, wo, w1, w2 = rnd(3072, 1024, scale=1 / 32), rnd(1024, 1024, scale=1 / 32), rnd(4096, 1024, scale=1 / 32), \
        rnd(1024, 4096, scale=1 / 64)
    wp1, wp2 = rnd(4096, 1024, scale=1 / 32), rnd(4096, 4096, scale=1 / 64)
    bq, bo, b1, b2, bp = rnd(3072), rnd(1024), rnd(4096), rnd(1024), rnd(4096)
    res = rnd(T, 1024)
    cases = [
        ("qkv+bias", x1k, wq, dict(bias=bq)),
        ("out+bias+res", x1k, wo, dict(bias=bo, residual=res)),
        ("fc1+bias+qgelu", x1k, w1, dict(bias=b1, act=ACT_QUICK_GELU)),
        ("fc2+bias+res", x4k, w2, dict(bias=b2, residual=res)),
        ("proj1+bias+gelu", p1k, wp1, dict(bias=bp, act=ACT_GELU)),
        ("proj2+bias", p4k, wp2, dict(bias=bp)),
    ]

    def run(x, w, kw, split):
        M, K = x.shape
        N = w.shape[0]
        y = torch.empty(M, N, dtype=x.dtype, device=x.device)
        r = kw.get("residual")
        fn = ops.gemm_ex if split else ops.gemm
        extra = dict(split_k=True) if split else {}
        return lambda: fn(0, 0, M, N, K, x, K, w, K, y, N, bias=kw.get("bias"), act=kw.get("act", 0),
                          residual=r, ldr=r.stride(0) if r is not None else 0, **extra), y

    for name, x, w, kw in cases:
        M, K = x.shape
        N = w.shape[0]
        fl = 2.0 * M * N * K
        grid = ctypes_grid(L, M, N, K)
        line = f"{name:16s} {M}x{N}x{K} (default tile {grid})"
        ref_fn, ref_y = run(x, w, kw, False)
        ref_fn()
        ref = ref_y.float().clone()
        for label, tile, sk, split in (("default", -1, 0, False), ("splitK", -1, 0, True),
                                       ("256+sk", 2, 2, False), ("192+sk", 3, 2, False),
                                       ("256", 2, 0, False), ("192", 3, 0, False), ("128", 0, 0, False)):
            pt = L.cullavo_gemm_set_tile(tile)
            ps = L.cullavo_gemm_set_streamk(sk)
            fn, y = run(x, w, kw, split)
            ms = timeit(fn)
            err = ((y.float() - ref).norm() / ref.norm()).item()
            L.cullavo_gemm_set_tile(pt)
            L.cullavo_gemm_set_streamk(ps)
            line += f" | {label} {fl / ms / 1e9:6.1f} TF {ms * 1e3:6.1f} us (d {err:.0e})"
        print(line, flush=True)


def ctypes_grid(L, M, N, K):
    import ctypes
    g = ctypes.c_int64(0)
    t = L.cullavo_gemm_plan(M, N, K, 0, 0, ctypes.addressof(g))
    return f"{t}, {g.value} blocks"


if __name__ == "__main__":
    main()
