"""GEMM tuning bench on the MI355X: every GEMM shape of the 7B train step, each kernel shape
(cullavo_gemm_set_tile 0/1/2 and auto), against torch.matmul (hipBLASLt) as a measured ceiling.
Random N(0,1) bf16 operands (guide §5.4 rule 25). Prints one line per (shape, kernel).

  python tools/gemm_bench.py [--T 8704] [--iters 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cullavo_amd import _lib, ops  # noqa: E402


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=8704)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--modes", default="-1,0,2,3")
    ap.add_argument("--groups", default="-4", help="tile orders to sweep (cullavo_gemm_set_group)")
    ap.add_argument("--kinds", default="fwd,dx,dw")
    ap.add_argument("--only", default="", help="comma list of shape names")
    a = ap.parse_args()
    T, d, F, V = a.T, 4096, 11008, 32064
    # (name, kind, rows, out, inner): fwd y[T,out]=x[T,in] w[out,in]^T; dx: dy[T,out] w[out,in];
    # dw: dW[out,in] = dy[T,out]^T x[T,in]
    shapes = [("qkv", 3 * d, d), ("o", d, d), ("gate_up", 2 * F, d), ("down", d, F), ("lm_head", V, d)]
    lib = _lib.lib()
    g = torch.Generator(device="cuda").manual_seed(0)
    for name, out_f, in_f in shapes:
        if a.only and name not in a.only.split(","):
            continue
        x = torch.randn(T, in_f, device="cuda", generator=g).bfloat16()
        w = torch.randn(out_f, in_f, device="cuda", generator=g).bfloat16()
        dy = torch.randn(T, out_f, device="cuda", generator=g).bfloat16()
        dw = torch.empty(out_f, in_f, device="cuda", dtype=torch.bfloat16)
        fl = 2.0 * T * out_f * in_f
        ref = {"fwd": lambda: x @ w.T, "dx": lambda: dy @ w, "dw": lambda: dy.T @ x}
        ours = {"fwd": lambda: ops.linear(x, w), "dx": lambda: ops.linear_dx(dy, w),
                "dw": lambda: ops.linear_dw(dy, x, dw)}
        for kind in a.kinds.split(","):
            r = ref[kind]()
            tb = timeit(ref[kind], a.iters)
            line = f"{name:8s} {kind:3s} T={T} out={out_f} in={in_f}  hipBLASLt {fl / tb / 1e9:7.1f} TF"
            for mode, grp in [(m.strip(), int(gg)) for m in a.modes.split(",") for gg in a.groups.split(",")]:
                lib.cullavo_gemm_set_group(grp)
                lane_epi = "L" in mode  # e.g. "-1L": same kernel, per-lane epilogue
                nt = "N" in mode        # e.g. "-1N": non-temporal C stores
                lib.cullavo_gemm_set_dma(0 if "D" in mode else 1)  # "-1D": per-K-tile DMA offsets
                lib.cullavo_gemm_set_tile(int(mode.rstrip("LND")))
                lib.cullavo_gemm_set_epilogue((0 if lane_epi else 1) | (2 if nt else 0))
                o = ours[kind]()
                err = ((o.float() - r.float()).norm() / r.float().norm()).item()
                t = timeit(ours[kind], a.iters)
                line += f" | m{mode}g{grp} {fl / t / 1e9:7.1f} TF err {err:.1e}"
            lib.cullavo_gemm_set_tile(-1)
            lib.cullavo_gemm_set_epilogue(1)
            lib.cullavo_gemm_set_dma(1)
            lib.cullavo_gemm_set_group(-4)
            print(line, flush=True)


if __name__ == "__main__":
    main()
