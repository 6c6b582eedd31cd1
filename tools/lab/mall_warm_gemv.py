"""Lab: does a decode GEMV run faster when its weights were just read by another kernel (the MALL,
MI355X's 256 MB memory-side cache, holding them)? Per shape, each timed GEMV follows either a read
of its own weight matrix ("warm") or of an unrelated buffer of the same size ("cold"); only the
GEMV is inside the HIP events.

  python tools/lab/mall_warm_gemv.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from cullavo_amd import ops  # noqa: E402


def main():
    g = torch.Generator(device="cuda").manual_seed(0)
    for name, N, K in (("qkv", 12288, 4096), ("o", 4096, 4096), ("down", 4096, 11008)):
        copies = max(2, -(-600_000_000 // (N * K * 2)))
        Ws = [torch.randn(N, K, device="cuda", generator=g).bfloat16() for _ in range(copies)]
        junk = [torch.randn(N, K, device="cuda", generator=g).bfloat16() for _ in range(2)]
        x = torch.randn(1, K, device="cuda", generator=g).bfloat16()
        for w in Ws[:2]:
            ops.linear(x, w)
        res = {}
        for mode in ("cold", "warm", "cold", "warm"):
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(4 * copies)]
            for i, (s, e) in enumerate(ev):
                w = Ws[i % copies]
                (w if mode == "warm" else junk[i % 2]).view(torch.int16).amax()
                s.record()
                ops.linear(x, w)
                e.record()
            torch.cuda.synchronize()
            us = sum(s.elapsed_time(e) for s, e in ev) / len(ev) * 1e3
            res.setdefault(mode, []).append(us)
        pre_us = []
        for _ in range(3):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record(); junk[0].view(torch.int16).amax(); e.record(); torch.cuda.synchronize()
            pre_us.append(s.elapsed_time(e) * 1e3)
        print(f"{name:5s} {N*K*2/1e6:6.1f} MB  cold {min(res['cold']):7.2f} us  warm {min(res['warm']):7.2f} us"
              f"  (read kernel {min(pre_us):6.1f} us)", flush=True)
        del Ws, junk


if __name__ == "__main__":
    main()
