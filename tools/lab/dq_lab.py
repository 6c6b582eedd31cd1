"""dQ ring lab (tools/lab/dq_lab.hip): the production dQ kernels (cullavo_attn_bwd_ws, mode 7, via the
staging switch) and the lab ring variants (stages x left-out parts) on the 7B layer's shapes,
random K / dS^T, HIP-event timed, interleaved rounds.

  python tools/lab/dq_lab.py [--rounds 3]
"""
import argparse
import ctypes
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from cullavo_amd import _lib  # noqa: E402

B, H, L, D = 8, 32, 1088, 128


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    ctypes.CDLL(_lib.LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    lab = ctypes.CDLL(os.path.join(ROOT, "tools", "lab", "so", "libdq.so"))
    lab.dq_lab.restype = ctypes.c_int
    lab.dq_lab.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                           ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64,
                           ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_void_p]
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = (torch.randn(B * L, 3 * H * D, device="cuda", generator=g) * 0.5).bfloat16()
    K = qkv[:, H * D:2 * H * D]
    LkP = LqP = -(-L // 128) * 128
    ds = (torch.randn(B * H * LkP * LqP, device="cuda", generator=g) * 0.01).bfloat16()
    dq = torch.empty(B * L, H * D, device="cuda", dtype=torch.bfloat16)
    stream = torch.cuda.current_stream().cuda_stream
    fl = 2.0 * B * H * L * L * D / 2
    cases = {}
    for blk in (0, 1):
        ldst, st_blk = (128, LkP * 128) if blk else (LqP, 128)
        for v in (40, 30, 20, 41, 31, 21, 42, 32, 43):
            cases[f"ring NST {v // 10} lab {v % 10} {'blocked' if blk else 'rows'}"] = (
                lambda v=v, ldst=ldst, st_blk=st_blk: lab.dq_lab(v, K.data_ptr(), K.stride(0), ds.data_ptr(), ldst,
                                                                 LkP * LqP, st_blk, LkP, dq.data_ptr(), dq.stride(0),
                                                                 B, H, L, D ** -0.5, stream))
    res = {k: [] for k in cases}
    for _ in range(a.rounds):
        for k, fn in cases.items():
            assert fn() == 0
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.iters):
                fn()
            e.record()
            e.synchronize()
            res[k].append(s.elapsed_time(e) / a.iters * 1e3)
    dsb = B * H * sum(min(L, 128 * (qb + 1)) for qb in range(LqP // 128)) * 256
    for k, ts in res.items():
        us = statistics.median(ts)
        print(f"{k:34s} {us:8.1f} us  dS^T {dsb / us / 1e3:7.1f} GB/s  {fl / us / 1e6:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
