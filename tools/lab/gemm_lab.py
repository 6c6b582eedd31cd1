"""Run the GEMM lab variants (tools/lab/gemm_lab.hip) on the GPU box: interleaved rounds in one
process (guide §5.4 rule 24), random N(0,1) bf16 operands, median TFLOP/s per variant.

  python tools/lab/gemm_lab.py [--variants 0,1,2,...] [--shapes gate_up,o,...] [--rounds 3]
"""
import argparse
import ctypes
import os
import statistics

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SHAPES = {"qkv": (8704, 12288, 4096), "o": (8704, 4096, 4096), "gate_up": (8704, 22016, 4096),
          "down": (8704, 4096, 11008), "lm_head": (8704, 32064, 4096),
          "vit_fc1": (36928, 4096, 1024), "vit_qkv": (36928, 3072, 1024), "vit_o": (36928, 1024, 1024),
          "vit_fc2": (36928, 1024, 4096)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,1,2,4,8")
    ap.add_argument("--shapes", default="gate_up,o,lm_head")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--lib", default=os.path.join(HERE, "libgemm_lab.so"))
    ap.add_argument("--prod", action="store_true", help="also time the production kernel (cullavo_amd.ops.linear)")
    a = ap.parse_args()
    prod = None
    if a.prod:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
        from cullavo_amd import ops as prod
    lib = ctypes.CDLL(a.lib)
    lib.lab_gemm.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    variants = [int(v) for v in a.variants.split(",")]
    g = torch.Generator(device="cuda").manual_seed(0)
    for name in a.shapes.split(","):
        M, N, K = SHAPES[name]
        A = torch.randn(M, K, device="cuda", generator=g).bfloat16()
        B = torch.randn(N, K, device="cuda", generator=g).bfloat16()
        C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        ref = (A @ B.T).float()
        stream = torch.cuda.current_stream().cuda_stream
        fl = 2.0 * M * N * K
        res = {v: [] for v in variants}
        errs = {}
        first = None
        same = {}
        for v in variants:
            C.fill_(float("nan"))
            rc = lib.lab_gemm(v, M, N, K, A.data_ptr(), B.data_ptr(), C.data_ptr(), stream)
            assert rc == 0, (v, rc)
            torch.cuda.synchronize()
            errs[v] = ((C.float() - ref).norm() / ref.norm()).item()
            if first is None:
                first = C.clone()
            same[v] = bool(torch.equal(C, first))
        tb, tp = [], []
        if prod is not None:
            yp = prod.linear(A, B)
            torch.cuda.synchronize()
            errs["prod"] = ((yp.float() - ref).norm() / ref.norm()).item()
        for _ in range(a.rounds):
            if prod is not None:
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(a.iters):
                    prod.linear(A, B, out=yp)
                e.record()
                e.synchronize()
                tp.append(fl / (s.elapsed_time(e) / a.iters) / 1e9)
            for v in variants:
                lib.lab_gemm(v, M, N, K, A.data_ptr(), B.data_ptr(), C.data_ptr(), stream)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(a.iters):
                    lib.lab_gemm(v, M, N, K, A.data_ptr(), B.data_ptr(), C.data_ptr(), stream)
                e.record()
                e.synchronize()
                res[v].append(fl / (s.elapsed_time(e) / a.iters) / 1e9)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.iters):
                A @ B.T
            e.record()
            e.synchronize()
            tb.append(fl / (s.elapsed_time(e) / a.iters) / 1e9)
        line = f"{name:8s} M={M} N={N} K={K} hipBLASLt {statistics.median(tb):7.1f}"
        if tp:
            line += f" | prod {statistics.median(tp):7.1f} (err {errs['prod']:.1e})"
        for v in variants:
            line += f" | v{v} {statistics.median(res[v]):7.1f} (err {errs[v]:.1e}{'' if same[v] else ' DIFF'})"
        print(line, flush=True)


if __name__ == "__main__":
    main()
