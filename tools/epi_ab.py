"""Per-shape A/B of the GEMM epilogue modes (cullavo_gemm_set_epilogue) on the config-3 / ViT
shapes, interleaved rounds in one process (guide §5.4 rule 24), random bf16 operands, HIP events:
  direct : the default (direct register epilogue, persistent 256 / 288-row forward kernels)
  lds    : bit 7 (the LDS-staged epilogue and the round-5 persistent kernel)
  nopers : bit 5 (no persistent forward kernel; direct epilogue in the data-parallel kernels)
  eager    : cullavo_gemm_set_msplit(2) (the M-tail split wherever the plan estimates a gain; the default
             since round 6), msplit5: set_msplit(1) (only >= 5 %, round 5)
  no288    : bit 9 (no 288-row tiles at K < 2048: round 5's plan; since round 6 the default takes them,
             on the persistent 288-row kernel). short288 / short288p (bits 9 / 9 + 8) were the round-6
             A/B names while bit 9 meant "allow"; with the flipped bit they now mean no288 / no288 + bit 8
Each case runs with the epilogue it has in the step (plain, residual, bias, quick_gelu).

  python tools/epi_ab.py [--rounds 5]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cullavo_amd import _lib, ops  # noqa: E402

CASES = [  # name, M, N, K, a_layout, b_layout, epilogue
    ("qkv_fwd", 8704, 12288, 4096, 0, 0, "plain"), ("o_fwd", 8704, 4096, 4096, 0, 0, "res"),
    ("gateup_fwd", 8704, 22016, 4096, 0, 0, "plain"), ("down_fwd", 8704, 4096, 11008, 0, 0, "res"),
    ("lmhead_fwd", 8704, 32064, 4096, 0, 0, "plain"),
    ("qkv_dx", 8704, 4096, 12288, 0, 1, "plain"), ("gateup_dx", 8704, 4096, 22016, 0, 1, "res"),
    ("o_dx", 8704, 4096, 4096, 0, 1, "plain"),
    ("gateup_dw", 22016, 4096, 8704, 1, 1, "plain"), ("down_dw", 4096, 11008, 8704, 1, 1, "plain"),
    ("lmhead_dw", 32064, 4096, 8704, 1, 1, "plain"),
    ("vit_fc1", 36928, 4096, 1024, 0, 0, "qgelu"), ("vit_qkv", 36928, 3072, 1024, 0, 0, "bias"),
    ("vit_o", 36928, 1024, 1024, 0, 0, "bias_res"), ("vit_fc2", 36928, 1024, 4096, 0, 0, "bias_res"),
]
MSPLIT = {"eager": 2, "msplit5": 1}  # modes that set cullavo_gemm_set_msplit (default 2) besides the epilogue bits
ALL_MODES = {"no288": 1 | 512, "eager": 1, "msplit5": 1, "direct": 1, "lds": 1 | 128, "nopers": 1 | 32, "short288": 1 | 512, "short288p": 1 | 512 | 256}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--cases", default="")
    ap.add_argument("--modes", default="direct,lds,nopers")
    a = ap.parse_args()
    MODES = {m: ALL_MODES[m] for m in a.modes.split(",")}
    L = _lib.lib()
    base = L.cullavo_gemm_set_epilogue(1)
    g = torch.Generator(device="cuda").manual_seed(0)
    sel = [c for c in CASES if not a.cases or c[0] in a.cases.split(",")]
    for name, M, N, K, al, bl, epi in sel:
        A = torch.randn((K, M) if al else (M, K), device="cuda", generator=g).bfloat16()
        B = (torch.randn((K, N) if bl else (N, K), device="cuda", generator=g) * K ** -0.5).bfloat16()
        bias = torch.randn(N, device="cuda", generator=g).bfloat16() if epi in ("bias", "bias_res", "qgelu") else None
        res = torch.randn(M, N, device="cuda", generator=g).bfloat16() if epi in ("res", "bias_res") else None
        act = ops.ACT_QUICK_GELU if epi == "qgelu" else ops.ACT_NONE
        C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)

        def run():
            ops.gemm_ex(al, bl, M, N, K, A, A.stride(0), B, B.stride(0), C, N, bias=bias, act=act, residual=res,
                        ldr=N if res is not None else 0)

        fl = 2.0 * M * N * K
        res_t = {m: [] for m in MODES}
        outs = {}
        for r in range(a.rounds):
            for m, bits in MODES.items():
                L.cullavo_gemm_set_epilogue(bits)
                L.cullavo_gemm_set_msplit(MSPLIT.get(m, 2))
                run()
                if r == 0:
                    torch.cuda.synchronize()
                    outs[m] = C.clone()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(a.iters):
                    run()
                e.record()
                e.synchronize()
                res_t[m].append(fl / (s.elapsed_time(e) / a.iters * 1e-3) / 1e12)
        L.cullavo_gemm_set_epilogue(base)
        same = all(torch.equal(next(iter(outs.values())), o) for o in outs.values())
        line = f"{name:11s} {M}x{N}x{K} ({al},{bl}) {epi:8s}"
        for m, bits in MODES.items():
            L.cullavo_gemm_set_epilogue(bits)
            L.cullavo_gemm_set_msplit(MSPLIT.get(m, 2))
            line += f" | {m} [{L.cullavo_gemm_plan(M, N, K, al, bl, None)}] {statistics.median(res_t[m]):7.1f}"
        L.cullavo_gemm_set_epilogue(base)
        L.cullavo_gemm_set_msplit(2)
        print(line + f" | bitwise {'equal' if same else 'DIFFERENT'}", flush=True)
        del A, B, C, bias, res


if __name__ == "__main__":
    main()
