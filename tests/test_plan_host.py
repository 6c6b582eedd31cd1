"""The GEMM plan's switches, host-only (cullavo_gemm_plan needs no GPU): the round-6 defaults
(eager M-tail split, 288-row tiles at K < 2048, the round split) and the A/B bits that restore
round 5's plans, with the setters returning the previous setting."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cullavo_amd import _lib  # noqa: E402


def plan(L, M, N, K, al=0, bl=0):
    g = ctypes.c_int64(0)
    return L.cullavo_gemm_plan(M, N, K, al, bl, ctypes.byref(g)), g.value


def test_round6_plan_defaults_and_switches():
    L = _lib.lib()
    prev_e = L.cullavo_gemm_set_epilogue(1)
    prev_m = L.cullavo_gemm_set_msplit(2)
    try:
        assert prev_e == 1 and prev_m == 2  # the defaults
        # ViT fc1 (M = 64 x 577): 288-row M-split, 128 M-tiles x 16 = 8 whole rounds
        assert plan(L, 36928, 4096, 1024) == (110, 2048)
        # bit 9: round 5's short-K rule (no 288 rows at K < 2048) -> the 256-row eager M-split
        assert L.cullavo_gemm_set_epilogue(1 | 512) == 1
        assert plan(L, 36928, 4096, 1024) == (102, 2304)
        # and msplit 1 (>= 5 % only): fc1 unsplit on 256 rows
        assert L.cullavo_gemm_set_msplit(1) == 2
        assert plan(L, 36928, 4096, 1024) == (2, 2320)
        assert L.cullavo_gemm_set_epilogue(1) == 1 | 512
        assert L.cullavo_gemm_set_msplit(2) == 1
        # the round split of the gate|up weight gradient: 5 whole rounds of 256x256 tiles
        assert plan(L, 22016, 4096, 8704, 1, 1) == (102, 1280)
        # a split never leaves a tail of <= 16 rows: 16 x 288 + 8 rows
        p, grid = plan(L, 16 * 288 + 8, 4096, 4096)
        if p >= 100:
            bm = {2: 256, 3: 192, 10: 288}[p - 100]
            assert 16 * 288 + 8 - grid // 16 * bm > 16
    finally:
        L.cullavo_gemm_set_epilogue(prev_e)
        L.cullavo_gemm_set_msplit(prev_m)
