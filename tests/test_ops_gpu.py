"""Per-kernel parity: every C-ABI kernel on the MI355X against the CPU oracle / an fp32 torch
restatement of the same op on the same (bf16-rounded) inputs.

Tolerances (stated per test): bf16 storage has a relative step of 2^-8 = 3.9e-3, so kernels
whose output is bf16 are checked at max|err| <= c * 2^-8 * scale with c small, and integer /
index work (merge plan, targets, gathers, embedding rows) bit-exactly.
"""
import math

import ctypes

import pytest
import torch
import torch.nn.functional as F

from oracle import cullavo_oracle as O

pytestmark = pytest.mark.gpu

DEV = "cuda"
BF = torch.bfloat16


def ops():
    from cullavo_amd import ops as _ops
    return _ops


def rnd(shape, seed, scale=1.0, dtype=BF):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(shape, generator=g) * scale).to(dtype)


def close(out, ref, tol, what=""):
    out = out.float().cpu()
    ref = ref.float().cpu()
    err = (out - ref).abs().max().item()
    scale = ref.abs().max().item() + 1e-12
    assert err <= tol * scale, f"{what}: max|err| {err:.3e} > {tol:.1e} * {scale:.3e}"


# ---------------------------------------------------------------------------------------------
# GEMM
# ---------------------------------------------------------------------------------------------
GEMM_SHAPES = [(128, 128, 64), (256, 384, 512), (200, 136, 72), (77, 520, 1000), (1024, 1024, 1024)]


@pytest.fixture(params=[0, 2, 3, 10, -1], ids=["t128", "t256x256", "t192x256", "t288x256", "auto"])
def tile_mode(request):
    from cullavo_amd import _lib
    prev = _lib.lib().cullavo_gemm_set_tile(request.param)
    yield request.param
    _lib.lib().cullavo_gemm_set_tile(prev)


@pytest.mark.parametrize("M,N,K", GEMM_SHAPES + [(520, 264, 8704), (8, 1032, 136)])
@pytest.mark.parametrize("al,bl", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_gemm_layouts(M, N, K, al, bl, tile_mode):
    if al == 1 and M % 8:  # unsupported shape: rejected on the host with the reference-style error
        A = torch.empty((K, M), dtype=BF, device=DEV)
        B = torch.empty((N, K) if bl == 0 else (K, N), dtype=BF, device=DEV)
        C = torch.empty((M, N), dtype=BF, device=DEV)
        with pytest.raises(ValueError, match="M must be a multiple of 8"):
            ops().gemm(al, bl, M, N, K, A, A.stride(0), B, B.stride(0), C, N)
        return
    A = rnd((M, K), 1)
    B = rnd((N, K), 2)
    ref = A.float() @ B.float().T
    Ad = (A if al == 0 else A.T.contiguous()).to(DEV)
    Bd = (B if bl == 0 else B.T.contiguous()).to(DEV)
    C = torch.empty((M, N), dtype=BF, device=DEV)
    ops().gemm(al, bl, M, N, K, Ad, Ad.stride(0), Bd, Bd.stride(0), C, N)
    close(C, ref, 8e-3, f"gemm {al}{bl} {M}x{N}x{K}")


@pytest.fixture(params=[1, 0], ids=["lds_epi", "lane_epi"])
def epi_mode(request):
    from cullavo_amd import _lib
    prev = _lib.lib().cullavo_gemm_set_epilogue(request.param)
    yield request.param
    _lib.lib().cullavo_gemm_set_epilogue(prev)


@pytest.mark.parametrize("act", [0, 1, 2])
def test_gemm_epilogues(act, tile_mode, epi_mode):
    M, N, K = 300, 264, 192
    x, w, b = rnd((M, K), 3), rnd((N, K), 4, 0.1), rnd((N,), 5, 0.1)
    r = rnd((M, N), 6)
    y, pre = ops().linear(x.to(DEV), w.to(DEV), b.to(DEV), act=act, residual=r.to(DEV), want_preact=True)
    p = (x.float() @ w.float().T + b.float()).to(BF).float()
    a = {0: p, 1: F.gelu(p), 2: O.quick_gelu(p)}[act]
    close(pre, p, 8e-3, "preact")
    close(y, a.to(BF).float() + r.float(), 8e-3, "epilogue")


@pytest.mark.parametrize("M,N,K,act", [(36928, 1024, 4096, "none"), (18496, 2048, 4096, "quick_gelu"),
                                         (18496, 1024, 4096, "none"), (36928, 4096, 1024, "quick_gelu")])
def test_gemm_msplit(M, N, K, act):
    """M-tail split (cullavo_gemm_set_msplit; the ViT's M = 64 x 577 = 36928): the head rows run in
    whole rounds of the planned tile and the rest as a thin split-K product. Head rows are
    bit-identical to the same tile run over all of M (cullavo_gemm_set_tile), the tail rows match
    the fp32 product (bias, quick_gelu and residual in the epilogue of both parts)."""
    from cullavo_amd import _lib
    L = _lib.lib()
    plan = L.cullavo_gemm_plan(M, N, K, 0, 0, None)
    assert plan >= 100, plan
    tile = plan - 100
    bm = {2: 256, 3: 192, 10: 288}[tile]
    mm = M // bm * bm
    g = torch.Generator(device=DEV).manual_seed(7)
    x = torch.randn(M, K, device=DEV, generator=g).to(BF)
    w = (torch.randn(N, K, device=DEV, generator=g) * K ** -0.5).to(BF)
    b = (torch.randn(N, device=DEV, generator=g) * 0.1).to(BF)
    r = torch.randn(M, N, device=DEV, generator=g).to(BF)
    code = ops().ACT_QUICK_GELU if act == "quick_gelu" else ops().ACT_NONE
    y = ops().linear(x, w, b, act=code, residual=r)
    prev = L.cullavo_gemm_set_tile(tile)
    try:
        y_tile = ops().linear(x, w, b, act=code, residual=r)
    finally:
        L.cullavo_gemm_set_tile(prev)
    assert torch.equal(y[:mm], y_tile[:mm])
    p = (x[mm:].float() @ w.float().T + b.float()).to(BF).float()
    a = O.quick_gelu(p) if act == "quick_gelu" else p
    close(y[mm:], a.to(BF).float() + r[mm:].float(), 8e-3, "tail rows")
    close(y[:mm][::97], y_tile[:mm][::97], 0.0, "head rows")


def test_gemm_round_split_weight_gradient():
    """The round split (round 6; cullavo_gemm_plan 100 + tile with the head on whole rounds): the
    gate|up weight gradient 22016 x 4096 x 8704 is 5.375 rounds of 256x256 tiles, so the plan runs
    5 rounds (20480 rows) on the 8-wave kernel and the last 1536 rows split over K on the same
    kernel (f32 partials reduced in split order). Head rows are bitwise the unsplit product's,
    tail rows match the fp32 product."""
    from cullavo_amd import _lib
    L = _lib.lib()
    T, Fo, d = 8704, 22016, 4096
    plan = L.cullavo_gemm_plan(Fo, d, T, 1, 1, None)
    assert plan == 102, plan
    g = torch.Generator(device=DEV).manual_seed(5)
    dy = torch.randn(T, Fo, device=DEV, generator=g).to(BF)
    x = torch.randn(T, d, device=DEV, generator=g).to(BF)
    dw = torch.empty(Fo, d, dtype=BF, device=DEV)
    ops().linear_dw(dy, x, dw)
    prev = L.cullavo_gemm_set_tile(2)
    try:
        dw_whole = torch.empty(Fo, d, dtype=BF, device=DEV)
        ops().linear_dw(dy, x, dw_whole)
    finally:
        L.cullavo_gemm_set_tile(prev)
    mm = 20480
    assert torch.equal(dw[:mm], dw_whole[:mm])
    ref = dy[:, mm:].float().T @ x.float()  # dW rows = dy columns
    close(dw[mm:], ref, 8e-3, "round-split tail rows")


@pytest.mark.parametrize("act", ["gelu", "quick_gelu"])
def test_gemm_epilogue_paths_bit_identical(tile_mode, act):
    """The LDS-staged 16-B epilogue (packed quick_gelu) and the per-lane one compute the same
    roundings in the same order, so every output (bias, LoRA addend, residual, preact, activation,
    accumulate) is bit-identical."""
    from cullavo_amd import _lib
    M, N, K = 520, 776, 320
    x, w, b = rnd((M, K), 31).to(DEV), rnd((N, K), 32, 0.1).to(DEV), rnd((N,), 33, 0.1).to(DEV)
    r, t = rnd((M, N), 34).to(DEV), rnd((M, N), 35, 0.05).to(DEV)
    code = ops().ACT_GELU if act == "gelu" else ops().ACT_QUICK_GELU
    outs = []
    for epi in (1, 0):
        prev = _lib.lib().cullavo_gemm_set_epilogue(epi)
        try:
            y, pre = ops().linear(x, w, b, act=code, residual=r, want_preact=True, addend=t)
            acc = rnd((N, K), 36, dtype=torch.float32).to(DEV)
            ops().linear_dw(y, x, acc, beta=1.0)
            outs.append((y, pre, acc))
        finally:
            _lib.lib().cullavo_gemm_set_epilogue(prev)
    for a, c in zip(outs[0], outs[1]):
        assert torch.equal(a, c)


@pytest.mark.parametrize("M,N,K,al,bl,tile,epi", [
    (2000, 1032, 1024, 0, 0, 2, "plain"), (2000, 1032, 1024, 0, 0, 2, "bias"), (2000, 1032, 1024, 0, 0, 2, "bias_res"),
    (2000, 1032, 1024, 0, 0, 2, "qgelu"), (2000, 1032, 1024, 0, 0, 2, "gelu"), (300, 264, 192, 0, 0, 2, "res"),
    (2000, 1032, 4096, 0, 0, 10, "plain"), (2000, 1032, 4096, 0, 0, 10, "res"), (8704 + 37, 4096, 4096, 0, 0, 10, "res"),
    (2000, 1032, 4096, 0, 1, 10, "plain"), (2000, 1032, 4096, 0, 1, 10, "res"), (2000, 1032, 1000, 0, 1, 2, "plain"),
    (2000, 1032, 1000, 0, 1, 2, "res"), (1032, 2056, 2000, 1, 1, 2, "plain"), (1032, 2056, 2000, 1, 1, 2, "res"),
    # > 256 tiles: the persistent kernel walks several tiles per CU (early K-tile 1 DMA, counted vmcnt)
    (8704 + 37, 4104, 1024, 0, 0, 2, "bias_res"), (8704 + 37, 2056, 192, 0, 0, 2, "plain"),
    (8704, 4096, 64, 0, 0, 2, "qgelu"), (8704 + 37, 4104, 1024, 0, 0, 2, "res")])
def test_gemm_direct_epilogue_bitwise(M, N, K, al, bl, tile, epi):
    """The direct epilogue (round 6: accumulators packed, permlane16-swapped and stored as 16-B buffer
    stores, no LDS round trip; the persistent forward kernel with the next tile's K-tile 1 issued
    before the stores, and the data-parallel 288- / 256-row kernels) against the LDS-staged epilogue
    (cullavo_gemm_set_epilogue bit 7) and the per-lane epilogue (bit 0 off): bitwise equal for every
    lean case (plain, bias, residual, bias + residual, quick_gelu / erf-GELU after a bias), ragged M
    and N tiles included, and within bf16 noise of the fp32 product."""
    from cullavo_amd import _lib
    L = _lib.lib()
    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    A = torch.randn((K, M) if al else (M, K), device=DEV, generator=g).to(BF)
    B = (torch.randn((K, N) if bl else (N, K), device=DEV, generator=g) * K ** -0.5).to(BF)
    bias = (torch.randn(N, device=DEV, generator=g) * 0.5).to(BF) if epi in ("bias", "bias_res", "qgelu", "gelu") else None
    res = torch.randn(M, N, device=DEV, generator=g).to(BF) if epi in ("res", "bias_res") else None
    act = {"qgelu": ops().ACT_QUICK_GELU, "gelu": ops().ACT_GELU}.get(epi, ops().ACT_NONE)
    prev_t, prev_e = L.cullavo_gemm_set_tile(tile), L.cullavo_gemm_set_epilogue(1)
    outs = []
    try:
        for mode in (1, 1 | 128, 0, 1 | 256):  # default, LDS-staged, per-lane, persistent 288-row opt-in
            L.cullavo_gemm_set_epilogue(mode)
            C = torch.full((M, N), float("nan"), dtype=BF, device=DEV)
            ops().gemm(al, bl, M, N, K, A, A.stride(0), B, B.stride(0), C, N, bias=bias, act=act, residual=res,
                       ldr=N if res is not None else 0)
            outs.append(C)
    finally:
        L.cullavo_gemm_set_tile(prev_t)
        L.cullavo_gemm_set_epilogue(prev_e)
    Ad = A.t() if al else A
    Bd = B if bl else B.t()
    ref = (Ad.float() @ Bd.float()) + (bias.float() if bias is not None else 0)
    if act:
        ref = ref.to(BF).float()
        ref = O.quick_gelu(ref) if epi == "qgelu" else F.gelu(ref)
    if res is not None:
        ref = ref.to(BF).float() + res.float()
    close(outs[0], ref, 8e-3, f"direct epilogue {epi}")
    assert torch.equal(outs[0], outs[1]), "direct vs LDS-staged epilogue"
    assert torch.equal(outs[0], outs[2]), "direct vs per-lane epilogue"
    assert torch.equal(outs[0], outs[3]), "direct vs the persistent 288-row direct kernel (opt-in)"


@pytest.mark.parametrize("M,N,K,al,bl", [(2304, 8192, 1024, 0, 0), (1032, 2056, 4104, 1, 1), (2000, 1544, 520, 0, 1),
                                          (1000, 4104, 1032, 1, 0)])
def test_gemm_tile_order_bitwise(M, N, K, al, bl):
    """The 8-wave kernels' tile order (cullavo_gemm_set_group: groups of M-tiles sweeping N, or of
    N-tiles sweeping M, ragged last groups included) only moves tiles between CUs: every order
    gives bitwise the same C."""
    from cullavo_amd import _lib
    A = rnd((M, K), 61)
    B = rnd((N, K), 62)
    Ad = (A if al == 0 else A.T.contiguous()).to(DEV)
    Bd = (B if bl == 0 else B.T.contiguous()).to(DEV)
    L = _lib.lib()
    prev = L.cullavo_gemm_set_group(-4)
    outs = []
    try:
        for g in (-4, 4, 1, 3, -1, -3, 8, -64):
            L.cullavo_gemm_set_group(g)
            C = torch.full((M, N), float("nan"), dtype=BF, device=DEV)
            ops().gemm(al, bl, M, N, K, Ad, Ad.stride(0), Bd, Bd.stride(0), C, N)
            outs.append((g, C))
    finally:
        L.cullavo_gemm_set_group(prev)
    close(outs[0][1], A.float() @ B.float().T, 8e-3, f"group -4 {al}{bl} {M}x{N}x{K}")
    for g, C in outs:
        assert torch.equal(C, outs[0][1]), f"tile order {g} changed C"


def test_gemm_f32_accumulate_beta(tile_mode):
    M, N, K = 128, 192, 256
    dy, x = rnd((M, N), 7), rnd((M, K), 8)
    out = rnd((N, K), 9, dtype=torch.float32).to(DEV)
    base = out.clone()
    ops().linear_dw(dy.to(DEV), x.to(DEV), out, beta=1.0)
    ref = dy.float().T @ x.float() + base.cpu()
    close(out, ref, 1e-5, "dw beta f32")


def test_linear_dx_dw_bf16(tile_mode):
    M, N, K = 520, 384, 264
    dy, w, x = rnd((M, N), 10), rnd((N, K), 11), rnd((M, K), 12)
    dx = ops().linear_dx(dy.to(DEV), w.to(DEV))
    close(dx, dy.float() @ w.float(), 8e-3, "dx")
    dw = torch.empty((N, K), dtype=BF, device=DEV)
    ops().linear_dw(dy.to(DEV), x.to(DEV), dw)
    close(dw, dy.float().T @ x.float(), 8e-3, "dw")


def test_gemm_strided_operands(tile_mode):
    # q|k|v fused projection output consumed as strided views (ld > K)
    M, K, N = 96, 128, 64
    big = rnd((M, 3 * K), 13)
    w = rnd((N, K), 14)
    xv = big.to(DEV)[:, K:2 * K]
    y = ops().linear(xv, w.to(DEV))
    close(y, big[:, K:2 * K].float() @ w.float().T, 8e-3, "strided")


@pytest.mark.parametrize("al,bl", [(0, 0), (0, 1), (1, 1)])
def test_gemm_pipelined_repeatable(al, bl):
    """Race screen for the counted-vmcnt kernels: the same product, launched many times
    back to back at sizes with K tails and several K-tiles, must be bit-identical every time
    (a read racing its LDS-DMA shows up as rare wrong tiles) and match the fp32 product."""
    from cullavo_amd import _lib
    for mode in (2, 3, 10):
        prev = _lib.lib().cullavo_gemm_set_tile(mode)
        try:
            for (M, N, K) in [(768, 1024, 4160), (520, 264, 200), (2048, 2048, 1024)]:
                A, B = rnd((M, K), 21), rnd((N, K), 22)
                Ad = (A if al == 0 else A.T.contiguous()).to(DEV)
                Bd = (B if bl == 0 else B.T.contiguous()).to(DEV)
                outs = []
                for _ in range(12):
                    C = torch.empty((M, N), dtype=BF, device=DEV)
                    ops().gemm(al, bl, M, N, K, Ad, Ad.stride(0), Bd, Bd.stride(0), C, N)
                    outs.append(C)
                close(outs[0], A.float() @ B.float().T, 8e-3, f"mode {mode} {al}{bl} {M}x{N}x{K}")
                for o in outs[1:]:
                    assert torch.equal(o, outs[0]), (mode, al, bl, M, N, K)
        finally:
            _lib.lib().cullavo_gemm_set_tile(prev)


# ---------------------------------------------------------------------------------------------
# norms
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("rows,cols", [(64, 4096), (37, 1024), (5, 128), (9, 8192), (97, 5120)])
def test_rmsnorm(rows, cols):
    x, w = rnd((rows, cols), 20), (1 + 0.1 * rnd((cols,), 21).float()).to(BF)
    y, rstd = ops().rmsnorm_fwd(x.to(DEV), w.to(DEV), 1e-5)
    xr = x.float().requires_grad_(True)
    wr = w.float().requires_grad_(True)
    yr = O.rmsnorm(xr, wr, 1e-5)
    close(y, yr, 8e-3, "rms fwd")
    dy = rnd((rows, cols), 22)
    dres = rnd((rows, cols), 23)
    dw = torch.empty(cols, dtype=torch.float32, device=DEV)
    dx = ops().rmsnorm_bwd(dy.to(DEV), x.to(DEV), w.to(DEV), rstd, dres=dres.to(DEV), dw=dw)
    yr.backward(dy.float())
    close(dx, xr.grad + dres.float(), 1e-2, "rms dx")
    close(dw, wr.grad, 1e-2, "rms dw")


@pytest.mark.parametrize("rows,cols", [(8704, 4096), (1037, 4096), (3, 4096), (515, 1024), (6400, 5120),
                                       (131, 8192)])
def test_rmsnorm_bwd_modes(rows, cols):
    """Pipelined backward (mode 1, default) vs the round-1 kernels (mode 0) and the oracle, at the
    config-3 and config-5 (d 5120) shapes and ragged row counts (partial last iterations / empty
    workgroups); with and without the weight gradient."""
    from cullavo_amd import _lib
    x, w = rnd((rows, cols), 40), (1 + 0.1 * rnd((cols,), 41).float()).to(BF)
    dy, dres = rnd((rows, cols), 42), rnd((rows, cols), 43)
    _, rstd = ops().rmsnorm_fwd(x.to(DEV), w.to(DEV), 1e-5)
    L = _lib.lib()
    outs = {}
    try:
        for mode in (0, 1):
            L.cullavo_rmsnorm_set_bwd(mode)
            dw = torch.empty(cols, dtype=torch.float32, device=DEV)
            dx = ops().rmsnorm_bwd(dy.to(DEV), x.to(DEV), w.to(DEV), rstd, dres=dres.to(DEV), dw=dw)
            dx2 = ops().rmsnorm_bwd(dy.to(DEV), x.to(DEV), w.to(DEV), rstd, dres=dres.to(DEV), dw=dw)
            assert torch.equal(dx, dx2), "rmsnorm_bwd is not deterministic"
            outs[mode] = (dx.float(), dw.clone())
        for mode in (0, 1):  # no weight gradient (frozen norms: the LoRA recipe)
            L.cullavo_rmsnorm_set_bwd(mode)
            dxn = ops().rmsnorm_bwd(dy.to(DEV), x.to(DEV), w.to(DEV), rstd, dres=dres.to(DEV))
            assert torch.equal(dxn, ops().rmsnorm_bwd(dy.to(DEV), x.to(DEV), w.to(DEV), rstd, dres=dres.to(DEV)))
            outs[("nodw", mode)] = dxn.float()
    finally:
        L.cullavo_rmsnorm_set_bwd(1)
    (dx0, dw0), (dx1, dw1) = outs[0], outs[1]
    # same per-element arithmetic; only the row dot product's partial-sum order differs
    assert (dx1 - dx0).abs().max().item() <= 2 * (dx0.abs().max().item() * 2 ** -7)
    assert (outs[("nodw", 1)] - dx0).abs().max().item() <= 2 * (dx0.abs().max().item() * 2 ** -7)
    assert (outs[("nodw", 0)] - dx0).abs().max().item() <= 2 * (dx0.abs().max().item() * 2 ** -7)
    assert ((dw1 - dw0).norm() / dw0.norm()).item() < 1e-5
    xr = x.float().requires_grad_(True)
    wr = w.float().requires_grad_(True)
    O.rmsnorm(xr, wr, 1e-5).backward(dy.float())
    close(dx1, xr.grad + dres.float(), 1e-2, "rms dx (pipelined)")
    close(dw1, wr.grad, 1e-2, "rms dw (pipelined)")


@pytest.mark.parametrize("rows,cols", [(64, 1024), (577, 128), (3, 64)])
def test_layernorm(rows, cols):
    x = rnd((rows, cols), 30, 2.0)
    w, b = (1 + 0.1 * rnd((cols,), 31).float()).to(BF), rnd((cols,), 32, 0.1)
    y, mean, rstd = ops().layernorm_fwd(x.to(DEV), w.to(DEV), b.to(DEV), 1e-5)
    xr = x.float().requires_grad_(True)
    wr, br = w.float().requires_grad_(True), b.float().requires_grad_(True)
    yr = O.layernorm(xr, wr, br, 1e-5)
    close(y, yr, 8e-3, "ln fwd")
    dy = rnd((rows, cols), 33)
    dw = torch.empty(cols, dtype=torch.float32, device=DEV)
    db = torch.empty(cols, dtype=torch.float32, device=DEV)
    dx = ops().layernorm_bwd(dy.to(DEV), x.to(DEV), w.to(DEV), mean, rstd, dw=dw, db=db)
    yr.backward(dy.float())
    close(dx, xr.grad, 1e-2, "ln dx")
    close(dw, wr.grad, 1e-2, "ln dw")
    close(db, br.grad, 1e-3, "ln db")


# ---------------------------------------------------------------------------------------------
# element-wise
# ---------------------------------------------------------------------------------------------
def test_swiglu():
    rows, Fd = 70, 688
    gu = rnd((rows, 2 * Fd), 40, 2.0)
    out = ops().swiglu_fwd(gu.to(DEV))
    g, u = gu[:, :Fd].float().requires_grad_(True), gu[:, Fd:].float().requires_grad_(True)
    ref = F.silu(g) * u
    close(out, ref, 8e-3, "swiglu")
    d = rnd((rows, Fd), 41)
    dgu = ops().swiglu_bwd(d.to(DEV), gu.to(DEV))
    ref.backward(d.float())
    close(dgu[:, :Fd], g.grad, 1e-2, "dgate")
    close(dgu[:, Fd:], u.grad, 1e-2, "dup")


@pytest.mark.parametrize("M,Fd,d,tile", [(8704, 11008, 4096, -1), (1000, 1376, 520, -1), (520, 688, 264, 0),
                                         (1000, 1376, 520, 2), (1000, 1376, 520, 3), (1000, 1376, 520, 10),
                                         (40, 688, 4104, -1)])
def test_swiglu_bwd_fused_in_dx_gemm(M, Fd, d, tile):
    """The down-projection dX GEMM with the SwiGLU backward in its epilogue (ACT_SWIGLU_BWD) is
    bitwise equal to dh = dy @ W_down then swiglu_bwd(dh, gu): the 7B shape, ragged tiles, the
    4-wave / 256x256 / 192x256 kernels (tile modes 0 / 2 / 3), the split-K small-M launch, and
    both weight layouts (W and its K-major copy)."""
    from cullavo_amd import _lib
    dy = rnd((M, d), 71).to(DEV)
    w = rnd((d, Fd), 72, 0.05).to(DEV)          # down_proj.weight [d, F]
    gu = rnd((M, 2 * Fd), 73, 2.0).to(DEV)
    prev = _lib.lib().cullavo_gemm_set_tile(tile)
    try:
        ref = ops().swiglu_bwd(ops().linear_dx(dy, w), gu)
        fused = ops().linear_dx(dy, w, swiglu_gu=gu)
        fused_t = ops().linear_dx_t(dy, w.t().contiguous(), swiglu_gu=gu)
    finally:
        _lib.lib().cullavo_gemm_set_tile(prev)
    assert torch.equal(fused, ref)
    assert torch.equal(fused_t, ref)
    # the prefetching LDS-staged form (default) against the rolled general path (bit 6)
    L = _lib.lib()
    prev_t, prev_e = L.cullavo_gemm_set_tile(tile), L.cullavo_gemm_set_epilogue(1)
    try:
        for bits in (1 | 64,):
            L.cullavo_gemm_set_epilogue(bits)
            assert torch.equal(ops().linear_dx(dy, w, swiglu_gu=gu), ref), bits
    finally:
        L.cullavo_gemm_set_tile(prev_t)
        L.cullavo_gemm_set_epilogue(prev_e)
    with pytest.raises(Exception):
        ops().linear_dx(dy, w, swiglu_gu=gu[:, :Fd])


@pytest.mark.parametrize("M,N,K,al,bl,epi", [(2308, 1024, 4096, 0, 0, "bias_res"), (1024, 1024, 8192, 0, 0, "quick_gelu"),
                                              (4096, 1024, 4608, 1, 1, "beta"), (2304, 1024, 5120, 0, 1, "none"),
                                              (1032, 520, 8192, 0, 0, "bias")])
def test_gemm_split256_small_grid(M, N, K, al, bl, epi):
    """Small 256x256 grids with a long K (the ViT's fc2 at 4 images, the projector's weight
    gradient at 8 images, ragged edges) run split over K on the 8-wave kernel (cullavo_gemm_plan tile 9) with a torch
    workspace: fp32-product parity with every epilogue it carries, deterministic (bitwise equal
    across launches) and within a bf16 ulp of the unsplit kernel (forced tile 2)."""
    from cullavo_amd import _lib
    L = _lib.lib()
    assert L.cullavo_gemm_plan(M, N, K, al, bl, None) == 9
    A = rnd((K, M) if al else (M, K), 80).to(DEV)
    B = rnd((K, N) if bl else (N, K), 81).to(DEV)
    bias = rnd((N,), 82).to(DEV) if epi in ("bias", "bias_res", "quick_gelu") else None
    res = rnd((M, N), 83).to(DEV) if epi == "bias_res" else None
    act = ops().ACT_QUICK_GELU if epi == "quick_gelu" else ops().ACT_NONE
    beta = 1.0 if epi == "beta" else 0.0
    C0 = rnd((M, N), 84).to(DEV)

    def run():
        C = C0.clone()
        ops().gemm(al, bl, M, N, K, A, A.stride(0), B, B.stride(0), C, N, bias=bias, act=act, residual=res,
                   ldr=N if res is not None else 0, beta=beta)
        return C
    c1, c2 = run(), run()
    assert torch.equal(c1, c2)
    prev = L.cullavo_gemm_set_tile(2)
    try:
        c_ref = run()
    finally:
        L.cullavo_gemm_set_tile(prev)
    Am = (A.float().T if al else A.float())
    Bm = (B.float() if bl else B.float().T)
    z = Am @ Bm
    if bias is not None:
        z = z + bias.float()
    if act == ops().ACT_QUICK_GELU:
        z = O.quick_gelu(z.to(BF).float())
    if res is not None:
        z = z.to(BF).float() + res.float()
    z = z + beta * C0.float()
    close(c1, z, 8e-3, f"split-K {M}x{N}x{K}")
    diff = (c1.float() - c_ref.float()).abs()
    assert diff.max().item() <= 2 ** -6 * c_ref.float().abs().max().item(), diff.max().item()


@pytest.mark.parametrize("tile", [2, 3, 10])
@pytest.mark.parametrize("al,bl,K", [(0, 0, 1024), (0, 1, 576), (1, 0, 640), (1, 1, 1000), (1, 1, 4096), (0, 0, 1000)])
def test_gemm_dma_precomputed_offsets_bitwise(tile, al, bl, K):
    """The precomputed-offset LDS-DMA loop (cullavo_gemm_set_dma(1): per-lane source offsets once
    per tile, K advance in the scalar offset) loads the same bytes as the per-K-tile path, so the
    8-wave kernels' outputs are bitwise equal with it on or off: every layout pair, ragged M/N
    edges (rows past M / N read as zeros), a K tail on layout-1 operands (rows past K lie past the
    buffer), and the fallback when a layout-0 operand has K % 64 != 0 (K 1000 with al = 0)."""
    from cullavo_amd import _lib
    L = _lib.lib()
    if tile in (3, 10) and al == 1:
        pytest.skip("192- and 288-row tiles take a layout-0 A only")
    M, N = 1000, 776
    A = rnd((K, M) if al else (M, K), 90).to(DEV)
    B = rnd((K, N) if bl else (N, K), 91).to(DEV)
    bias = rnd((N,), 92).to(DEV)
    outs = []
    prev_t = L.cullavo_gemm_set_tile(tile)
    try:
        for mode in (0, 1, 0):
            prev = L.cullavo_gemm_set_dma(mode)
            C = torch.empty((M, N), dtype=BF, device=DEV)
            ops().gemm(al, bl, M, N, K, A, A.stride(0), B, B.stride(0), C, N, bias=bias)
            torch.cuda.synchronize()
            L.cullavo_gemm_set_dma(prev)
            outs.append(C)
    finally:
        L.cullavo_gemm_set_tile(prev_t)
    assert torch.equal(outs[0], outs[2])
    assert torch.equal(outs[0], outs[1]), (outs[0].float() - outs[1].float()).abs().max().item()
    Am = (A.float().T if al else A.float())
    Bm = (B.float() if bl else B.float().T)
    close(outs[1], Am @ Bm + bias.float(), 8e-3, f"dma_pre tile {tile} {al}{bl} K={K}")


@pytest.mark.parametrize("act", [1, 2])
def test_act_bwd(act):
    x = rnd((33, 256), 50, 2.0)
    dy = rnd((33, 256), 51)
    xr = x.float().requires_grad_(True)
    (F.gelu(xr) if act == 1 else O.quick_gelu(xr)).backward(dy.float())
    dx = ops().act_bwd(act, dy.to(DEV), x.to(DEV))
    close(dx, xr.grad, 8e-3, "act bwd")


def test_colsum():
    x = rnd((1000, 264), 55)
    out = torch.zeros(264, dtype=torch.float32, device=DEV)
    ops().colsum(x.to(DEV), out)
    close(out, x.float().sum(0), 1e-5, "colsum")


@pytest.mark.parametrize("D,H", [(128, 4), (64, 3)])
def test_rope(D, H):
    T = 50
    q = rnd((T, H * D), 60)
    k = rnd((T, H * D), 61)
    pos = torch.randint(0, 1100, (T,))
    cos, sin = O.rope_cos_sin(pos[None], D, 10000.0)
    cos, sin = cos.to(BF).float(), sin.to(BF).float()
    def ref(x):
        xh = x.float().view(1, T, H, D).transpose(1, 2)
        return O.apply_rope(xh, cos, sin).transpose(1, 2).reshape(T, H * D)
    qd, kd = q.to(DEV), k.to(DEV)
    ops().rope(qd, kd, pos.to(DEV), hq=H, hk=H, head_dim=D, theta=10000.0)
    close(qd, ref(q), 8e-3, "rope q")
    close(kd, ref(k), 8e-3, "rope k")
    ops().rope(qd, kd, pos.to(DEV), hq=H, hk=H, head_dim=D, theta=10000.0, inverse=True)
    close(qd, q.float(), 2e-2, "rope inverse")


# ---------------------------------------------------------------------------------------------
# attention
# ---------------------------------------------------------------------------------------------
ATTN = [
    # B, H, L, D, causal
    (2, 2, 200, 128, True),
    (1, 3, 1088, 128, True),
    (2, 2, 577, 64, False),
    (1, 2, 64, 64, False),
    (1, 1, 33, 128, False),
]


def _attn_ref(q, k, v, B, H, L, D, causal, kv_start=None):
    qf = q.float().view(B, L, H, D).transpose(1, 2).requires_grad_(True)
    kf = k.float().view(B, L, H, D).transpose(1, 2).requires_grad_(True)
    vf = v.float().view(B, L, H, D).transpose(1, 2).requires_grad_(True)
    allowed = None
    if causal:
        m = torch.ones(B, L, dtype=torch.long)
        if kv_start is not None:
            for b, s in enumerate(kv_start):
                m[b, :s] = 0
        allowed = O.causal_allowed(m)
    o = O.attention(qf, kf, vf, D ** -0.5, allowed)
    return qf, kf, vf, o


@pytest.mark.parametrize("B,H,L,D,causal", ATTN)
def test_attention_fwd_bwd(B, H, L, D, causal):
    q, k, v = rnd((B * L, H * D), 70), rnd((B * L, H * D), 71), rnd((B * L, H * D), 72)
    qf, kf, vf, o_ref = _attn_ref(q, k, v, B, H, L, D, causal)
    o, lse = ops().attn_fwd(q.to(DEV), k.to(DEV), v.to(DEV), B=B, H=H, Lq=L, Lk=L, D=D, scale=D ** -0.5,
                            causal=causal)
    o_ref2 = o_ref.transpose(1, 2).reshape(B * L, H * D)
    close(o, o_ref2, 1.2e-2, "attn o")
    s = (qf @ kf.transpose(-1, -2)) * D ** -0.5
    if causal:
        s = s.masked_fill(~torch.ones(L, L, dtype=torch.bool).tril(), float("-inf"))
    close(lse, torch.logsumexp(s, -1), 1e-3, "attn lse")
    do = rnd((B * L, H * D), 73)
    o_ref2.backward(do.float())
    dq, dk, dv = ops().attn_bwd(q.to(DEV), k.to(DEV), v.to(DEV), o, do.to(DEV), lse, B=B, H=H, Lq=L, Lk=L, D=D,
                                scale=D ** -0.5, causal=causal)
    tr = lambda g: g.transpose(1, 2).reshape(B * L, H * D)
    close(dv, tr(vf.grad), 2e-2, "dv")
    close(dk, tr(kf.grad), 2e-2, "dk")
    close(dq, tr(qf.grad), 2e-2, "dq")


def test_attention_config3_batch8_sampled_heads():
    """Attention at config 3's real shape (B = 8, H = 32, L = 1088, D = 128 causal: B*H = 256
    heads, q|k|v as column blocks of the fused [T, 3d] projection output, the production layout)
    against the oracle on sampled (batch, head) pairs incl. the last one (b 7, h 31): O, LSE and
    dQ / dK / dV, same tolerances as test_attention_fwd_bwd (reference path
    /root/reference/cullavo/arch_cullavo.py:638-665 via the LM's FA2 attention)."""
    B, H, L, D = 8, 32, 1088, 128
    hd = H * D
    qkv = rnd((B * L, 3 * hd), 270).to(DEV)
    do = rnd((B * L, hd), 271).to(DEV)
    q, k, v = qkv[:, :hd], qkv[:, hd:2 * hd], qkv[:, 2 * hd:]
    o, lse = ops().attn_fwd(q, k, v, B=B, H=H, Lq=L, Lk=L, D=D, scale=D ** -0.5, causal=True)
    dq, dk, dv = ops().attn_bwd(q, k, v, o, do, lse, B=B, H=H, Lq=L, Lk=L, D=D, scale=D ** -0.5, causal=True)
    torch.cuda.synchronize()
    for t in (o, dq, dk, dv):
        assert torch.isfinite(t.float()).all()
    for b, h in ((0, 0), (3, 17), (7, 31), (5, 2)):
        r, c = slice(b * L, (b + 1) * L), slice(h * D, (h + 1) * D)
        pick = lambda t: t[r, c].float().cpu().view(1, 1, L, D)
        qf, kf, vf = (pick(t).requires_grad_(True) for t in (q, k, v))
        allowed = O.causal_allowed(torch.ones(1, L, dtype=torch.long))
        o_ref = O.attention(qf, kf, vf, D ** -0.5, allowed)
        close(o[r, c], o_ref.view(L, D), 1.2e-2, f"o b{b} h{h}")
        sc = (qf @ kf.transpose(-1, -2)) * D ** -0.5
        sc = sc.masked_fill(~torch.ones(L, L, dtype=torch.bool).tril(), float("-inf"))
        close(lse[b, h], torch.logsumexp(sc, -1).view(L), 1e-3, f"lse b{b} h{h}")
        o_ref.backward(pick(do))
        close(dq[r, c], qf.grad.view(L, D), 2e-2, f"dq b{b} h{h}")
        close(dk[r, c], kf.grad.view(L, D), 2e-2, f"dk b{b} h{h}")
        close(dv[r, c], vf.grad.view(L, D), 2e-2, f"dv b{b} h{h}")


@pytest.mark.parametrize("D,causal", [(128, True), (64, False)])
def test_attention_fwd_deferred_rescale_forced(D, causal):
    """The forward's deferred rescale (cullavo_attn_set_rescale, guide T13 / rule 26): inputs that
    FORCE the rare branch -- a spike key late in the sequence whose score jumps far above every
    earlier one for most queries, so the running max must move by more than the threshold at a
    late tile -- checked against a float64 reference at thresholds 0 (rescale on every growth,
    the plain online softmax), 8 (default) and 16, with LSE agreeing to 1e-5 across them."""
    from cullavo_amd import _lib
    B, H, L = 2, 2, 300
    u = rnd((1, 1, H, D), 78).float()                     # a direction every query shares
    q = (rnd((B, L, H, D), 75).float() + u).reshape(B * L, H * D).to(BF)
    kh = rnd((B, L, H, D), 76).float()
    v = rnd((B * L, H * D), 77)
    spike = 230  # a key in the 4th 64-key tile scoring ~3D / sqrt(D) against every query
    kh[:, spike] = 3.0 * u[0, 0]
    k = kh.reshape(B * L, H * D).to(BF)
    kw = dict(B=B, H=H, Lq=L, Lk=L, D=D, scale=D ** -0.5, causal=causal)
    L_ = _lib.lib()
    outs = {}
    prev = ctypes.c_float(0.0)
    try:
        for thr in (0.0, 8.0, 16.0):
            assert L_.cullavo_attn_set_rescale(ctypes.c_float(thr), ctypes.addressof(prev)) == 0
            outs[thr] = ops().attn_fwd(q.to(DEV), k.to(DEV), v.to(DEV), **kw)
    finally:
        L_.cullavo_attn_set_rescale(ctypes.c_float(8.0), None)
    qd = q.double().view(B, L, H, D).transpose(1, 2)
    kd = k.double().view(B, L, H, D).transpose(1, 2)
    vd = v.double().view(B, L, H, D).transpose(1, 2)
    sc = (qd @ kd.transpose(-1, -2)) * D ** -0.5
    if causal:
        sc = sc.masked_fill(~torch.ones(L, L, dtype=torch.bool).tril(), float("-inf"))
    assert (sc[..., spike:, spike] - sc[..., spike:, :spike].amax(-1)).median() * 1.4427 > 16  # branch forced
    o_ref = (torch.softmax(sc, -1) @ vd).transpose(1, 2).reshape(B * L, H * D)
    for thr, (o, lse) in outs.items():
        close(o, o_ref, 1.2e-2, f"attn o, threshold {thr}")
        close(lse, torch.logsumexp(sc, -1), 1e-4, f"lse, threshold {thr}")
        assert ((lse - outs[0.0][1]).abs() / outs[0.0][1].abs().clamp_min(1.0)).max().item() < 1e-5
    with pytest.raises(ValueError):
        _lib.call("attn_set_rescale", ctypes.c_float(-1.0), None)


@pytest.mark.parametrize("B,H,L,D,causal,ks", [(2, 2, 1088, 128, True, [0, 37]), (3, 2, 200, 128, True, [5, 0, 130]),
                                               (2, 3, 577, 64, False, None), (1, 2, 33, 128, False, None)])
def test_attention_fwd_staging_modes_bitwise(B, H, L, D, causal, ks):
    """The forward's K/V staging variants (cullavo_attn_set_stage: 2 = per-tile scalar descriptor;
    1 = per-chunk range-checked buffer loads; 0 = pointer loads; 3 = 2 with raised
    MFMA priority; 4 = LDS-DMA straight into the swizzled image, the default; 5 = 4 with inline-asm fragment
    reads in counted groups; 7 = the software-pipelined D = 128 kernel, softmax of tile t beside
    the S MFMAs of tile t+1) stage the same bytes
    (rows past the sequence end as zeros), so O and LSE are bitwise equal: ragged last tiles
    (L % 64 != 0), a partial single tile (L = 33), left-padded rows (kv_start), the LM D = 128
    causal and ViT D = 64 shapes; and the default matches the float reference."""
    from cullavo_amd import _lib
    q, k, v = rnd((B * L, H * D), 170), rnd((B * L, H * D), 171), rnd((B * L, H * D), 172)
    kv = torch.tensor(ks, dtype=torch.int32, device=DEV) if ks is not None else None
    kw = dict(B=B, H=H, Lq=L, Lk=L, D=D, scale=D ** -0.5, causal=causal)
    if kv is not None:
        kw["kv_start"] = kv
    L_ = _lib.lib()
    outs = {}
    prev = L_.cullavo_attn_set_stage(2)
    try:
        for mode in (2, 1, 0, 3, 4, 5, 7):
            assert L_.cullavo_attn_set_stage(mode) in (0, 1, 2, 3, 4, 5, 7)
            outs[mode] = ops().attn_fwd(q.to(DEV), k.to(DEV), v.to(DEV), **kw)
    finally:
        L_.cullavo_attn_set_stage(prev)
    for mode in (1, 0, 3, 4, 5, 7):
        assert torch.equal(outs[2][0], outs[mode][0]), f"O differs, stage {mode}"
        assert torch.equal(outs[2][1], outs[mode][1]), f"LSE differs, stage {mode}"
    if ks is None:
        _, _, _, o_ref = _attn_ref(q, k, v, B, H, L, D, causal)
        close(outs[4][0], o_ref.transpose(1, 2).reshape(B * L, H * D), 1.2e-2, "attn o (stage 4)")


@pytest.mark.parametrize("D,causal", [(128, True), (64, False)])
def test_attention_bwd_tile_modes_bitwise(D, causal):
    """Every backward tile shape (cullavo_attn_set_bwd_tiles) sums the same products in the same
    order, so dQ/dK/dV agree bit for bit; ragged L and a left-padded batch row included."""
    from cullavo_amd import _lib
    B, H, L = 2, 3, 200
    q, k, v, do = (rnd((B * L, H * D), s).to(DEV) for s in (91, 92, 93, 94))
    ks = torch.tensor([0, 45], dtype=torch.int32, device=DEV)
    kw = dict(B=B, H=H, Lq=L, Lk=L, D=D, scale=D ** -0.5, causal=causal, kv_start=ks)
    o, lse = ops().attn_fwd(q, k, v, **kw)
    prev = _lib.lib().cullavo_attn_set_bwd_tiles(0)
    try:
        outs = []
        for mode in (0, 1, 2, 3):
            _lib.lib().cullavo_attn_set_bwd_tiles(mode)
            outs.append([t.clone() for t in ops().attn_bwd(q, k, v, o, do, lse, **kw)])
    finally:
        _lib.lib().cullavo_attn_set_bwd_tiles(prev)
    for i, mode in enumerate((1, 2, 3)):
        for name, a, b in zip("qkv", outs[0], outs[i + 1]):
            assert torch.equal(a.view(torch.int16), b.view(torch.int16)), f"d{name} mode {mode}"
    # mode 4 (8-wave kernels: the pair halves of each tile are summed once at the end) adds the
    # same products in another order: bf16-rounding-level differences only, and deterministic
    res8 = {}
    for mode8 in (4, 7):
        _lib.lib().cullavo_attn_set_bwd_tiles(mode8)
        try:
            o4 = [t.clone() for t in ops().attn_bwd(q, k, v, o, do, lse, **kw)]
            o4b = [t.clone() for t in ops().attn_bwd(q, k, v, o, do, lse, **kw)]
        finally:
            _lib.lib().cullavo_attn_set_bwd_tiles(prev)
        res8[mode8] = o4
        for name, a, b, c in zip("qkv", outs[0], o4, o4b):
            assert torch.equal(b.view(torch.int16), c.view(torch.int16)), f"d{name} mode {mode8} not deterministic"
            err = ((a.float() - b.float()).norm() / a.float().norm()).item()
            assert err <= 5e-3, (name, mode8, err)
    # mode 7 runs mode 4's dK/dV kernel (plus the dS^T stores): dK, dV bitwise equal to it
    for name, a, b in zip("kv", res8[4][1:], res8[7][1:]):
        assert torch.equal(a.view(torch.int16), b.view(torch.int16)), f"d{name} mode 7 vs 4"
    # the LDS-DMA staging (cullavo_attn_set_bwd_stage) stages the same bytes (rows past the end as
    # zeros): modes 4 and 7 bitwise equal to the register staging, for the dK/dV kernel's Q / dO
    # (bit 0), the dQ-from-dS kernel's K / dS^T (bit 1), its LDS-DMA ring form (bit 2, D = 128) and
    # the blocked dS^T layout (bit 3)
    prev_st = _lib.lib().cullavo_attn_set_bwd_stage(1)
    try:
        for st in range(1, 16):
            _lib.lib().cullavo_attn_set_bwd_stage(st)
            for mode8 in (4, 7):
                _lib.lib().cullavo_attn_set_bwd_tiles(mode8)
                od = [t.clone() for t in ops().attn_bwd(q, k, v, o, do, lse, **kw)]
                for name, a, b in zip("qkv", res8[mode8], od):
                    assert torch.equal(a.view(torch.int16), b.view(torch.int16)), f"d{name} mode {mode8} DMA staging {st}"
    finally:
        _lib.lib().cullavo_attn_set_bwd_stage(prev_st)
        _lib.lib().cullavo_attn_set_bwd_tiles(prev)


def test_attention_strided_and_kv_start():
    B, H, L, D = 2, 2, 160, 128
    qkv = rnd((B * L, 3 * H * D), 80)
    kv_start = [0, 37]
    q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
    qf, kf, vf, o_ref = _attn_ref(q.contiguous(), k.contiguous(), v.contiguous(), B, H, L, D, True, kv_start)
    d = qkv.to(DEV)
    ks = torch.tensor(kv_start, dtype=torch.int32, device=DEV)
    o, lse = ops().attn_fwd(d[:, :H * D], d[:, H * D:2 * H * D], d[:, 2 * H * D:], B=B, H=H, Lq=L, Lk=L, D=D,
                            scale=D ** -0.5, causal=True, kv_start=ks)
    ref = o_ref.transpose(1, 2).reshape(B * L, H * D)
    valid = torch.ones(B * L, dtype=torch.bool)
    valid[L:L + 37] = False  # fully masked query rows of batch 1
    close(o.cpu()[valid], ref[valid], 1.2e-2, "strided attn")


# ---------------------------------------------------------------------------------------------
# embeddings / merge / loss
# ---------------------------------------------------------------------------------------------
def test_embedding_fwd_bwd_exact():
    V, Dm, n = 500, 256, 300
    table = rnd((V, Dm), 90)
    ids = torch.randint(0, V, (n,))
    ids[::7] = 3  # duplicates
    out = ops().embedding_fwd(ids.to(DEV), table.to(DEV))
    assert torch.equal(out.cpu(), table[ids])
    dout = rnd((n, Dm), 91)
    dt = torch.zeros((V, Dm), dtype=torch.float32, device=DEV)
    ops().embedding_bwd(ids.to(DEV), dout.to(DEV), dt, beta=1.0)
    ref = torch.zeros(V, Dm).index_add_(0, ids, dout.float())
    close(dt, ref, 1e-6, "embedding bwd")


@pytest.mark.parametrize("pad_tail,left", [(None, False), ([0, 5], False), ([0, 6], True)])
def test_merge_plan_bit_exact(pad_tail, left):
    cfg = O.config_small_gpu()
    ids, mask, _, _ = O.make_inputs(cfg, 2, 40, 4, 3, pad_tail=pad_tail)
    if left and pad_tail:  # move padding to the front
        for b, n in enumerate(pad_tail):
            if n:
                ids[b] = torch.cat([ids[b, 40 - n:], ids[b, :40 - n]])
                mask[b] = torch.cat([mask[b, 40 - n:], mask[b, :40 - n]])
    P, D = cfg.vision.num_patches, 16
    emb = rnd((2, 40, D), 95)
    img = rnd((2, P, D), 96)
    r_emb, r_mask, _, r_pos = O.merge(img, emb, ids, mask, cfg)
    L = r_emb.shape[1]
    left_pad = not bool((ids[:, -1] == cfg.pad_token_id).sum())
    td, src, mm, pos = ops().merge_plan(ids.to(DEV), mask.to(DEV), L=L, image_token=cfg.image_token_index,
                                       n_patches=P, left_padding=left_pad)
    out = ops().row_gather2(src.reshape(-1), emb.to(DEV).reshape(-1, D), img.to(DEV).reshape(-1, D))
    assert torch.equal(out.cpu().view(2, L, D), r_emb)
    assert torch.equal(mm.cpu(), r_mask.long())
    assert torch.equal(pos.cpu(), r_pos)
    # backward plan: the text gradient is the merged-row gradient gathered through text_dst
    emb_r = emb.clone().requires_grad_(True)
    G = rnd((2, L, D), 97)
    O.merge(img, emb_r, ids, mask, cfg)[0].backward(G)
    dtext = ops().row_gather2(td.reshape(-1), G.to(DEV).reshape(-1, D), None)
    assert torch.equal(dtext.cpu().view(2, 40, D), emb_r.grad)


def test_ce_fwd_bwd():
    B, L, V = 2, 50, 1000
    logits = rnd((B * L, V), 100, 3.0)
    labels = torch.randint(0, V, (B, L))
    labels[:, :10] = -100
    mask = torch.ones(B, L, dtype=torch.long)
    mask[1, 40:] = 0
    tgt = ops().shift_targets(labels.to(DEV), mask.to(DEV))
    ref_tgt = torch.full((B, L), -100)
    ref_tgt[:, :-1] = torch.where(mask[:, 1:] != 0, labels[:, 1:], torch.tensor(-100))
    assert torch.equal(tgt.cpu(), ref_tgt.reshape(-1))
    lg = logits.to(DEV)
    row_loss, lse = ops().ce_fwd(lg, tgt)
    out = ops().ce_reduce(row_loss, tgt)
    lr = logits.float().requires_grad_(True)
    ref = O.shifted_ce(lr.view(B, L, V), labels, mask)
    assert abs(out[0].item() - ref.item()) < 1e-5 * abs(ref.item()) + 1e-6
    ref.backward()
    d = ops().ce_bwd(lg, tgt, lse, out)
    close(d, lr.grad, 8e-3, "ce bwd")


def test_vision_front_end():
    cfg = O.config_small_gpu().vision
    B = 2
    W = O.make_weights(O.config_small_gpu(), 5)
    vp = "vision_tower.vision_model."
    pix = torch.randn(B, 3, cfg.image_size, cfg.image_size, generator=torch.Generator().manual_seed(7))
    kpad = 640
    patches = ops().im2col_patches(pix.to(DEV), cfg.patch_size, kpad)
    wconv = W[vp + "embeddings.patch_embedding.weight"].reshape(cfg.hidden_size, -1)
    wpad = torch.zeros(cfg.hidden_size, kpad)
    wpad[:, :wconv.shape[1]] = wconv
    x = ops().linear(patches, wpad.to(BF).to(DEV))
    T = cfg.num_patches + 1
    bf = lambda t: t.to(BF).to(DEV)
    h = ops().vision_embed_ln(x, bf(W[vp + "embeddings.class_embedding"]),
                              bf(W[vp + "embeddings.position_embedding.weight"]), bf(W[vp + "pre_layrnorm.weight"]),
                              bf(W[vp + "pre_layrnorm.bias"]), B=B, T=T, eps=cfg.layer_norm_eps)
    ref = O.vision_hidden_states(pix, W, cfg, 0)[0]
    close(h.view(B, T, -1), ref, 2e-2, "vision embed+ln")


def test_adamw_matches_torch():
    n = 4096 + 24
    p0 = rnd((n,), 110, dtype=torch.float32)
    grads = [rnd((n,), 111 + i, dtype=torch.float32) for i in range(3)]
    ref = p0.clone().requires_grad_(True)
    opt = torch.optim.AdamW([ref], lr=1e-2, weight_decay=0.1)
    p = p0.clone().to(DEV)
    m = torch.zeros(n, device=DEV)
    v = torch.zeros(n, device=DEV)
    for step, g in enumerate(grads, 1):
        ref.grad = g.clone()
        opt.step()
        ops().adamw(p, g.to(DEV), m, v, lr=1e-2, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.1, step=step)
    close(p, ref.detach(), 1e-5, "adamw")


def test_clip_coef_and_sumsq():
    a = rnd((1000,), 120, dtype=torch.float32).to(DEV)
    b = rnd((333,), 121).to(DEV)
    acc = torch.zeros(1, device=DEV)
    ops().sumsq(a, acc)
    ops().sumsq(b, acc)
    norm = math.sqrt(a.double().pow(2).sum().item() + b.double().pow(2).sum().item())
    coef = torch.empty(1, device=DEV)
    nrm = torch.empty(1, device=DEV)
    ops().clip_coef(acc, 1.0, coef, nrm)
    assert abs(nrm.item() - norm) < 1e-4 * norm
    assert abs(coef.item() - min(1.0, 1.0 / (norm + 1e-6))) < 1e-6


def test_linear_dw_ragged_token_count():
    # dW reduces over tokens: B*L is arbitrary (590 here), only N % 8 matters
    M, N, K = 590, 1024, 256
    dy, x = rnd((M, N), 130), rnd((M, K), 131)
    dw = torch.empty((N, K), dtype=torch.float32, device=DEV)
    ops().linear_dw(dy.to(DEV), x.to(DEV), dw)
    close(dw, dy.float().T @ x.float(), 1e-5, "dw ragged")


@pytest.mark.parametrize("rows,cols,pad", [(64, 64, 0), (72, 136, 0), (4096, 11008, 0), (200, 96, 24)])
def test_transpose16_exact(rows, cols, pad):
    """cullavo_transpose16 (K-major weight copies for the dX GEMMs) == torch .t(), ragged tiles and
    padded leading dims included"""
    from cullavo_amd import ops
    g = torch.Generator(device="cuda").manual_seed(rows + cols)
    base = torch.randn(rows, cols + pad, device="cuda", generator=g).bfloat16()
    src = base[:, :cols]
    dst = torch.full((cols, rows), 7.0, device="cuda", dtype=torch.bfloat16)
    ops.transpose2d(src, dst)
    assert torch.equal(dst, src.t())
    with pytest.raises(Exception):
        ops.transpose2d(src[:, :cols - 4], torch.empty(cols - 4, rows, device="cuda", dtype=torch.bfloat16))


@pytest.mark.parametrize("M,N,K", [(8704, 4096, 4096), (300, 1024, 640), (8704, 11008, 4096)])
def test_linear_dx_kmajor_bitwise(M, N, K):
    """dx from the K-major copy (gemm mode (0,0)) is bitwise equal to dx = dy @ W read along N
    (mode (0,1)): same K-tile order, same MFMA sequence"""
    from cullavo_amd import ops
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    w = torch.randn(N, K, device="cuda", generator=g).bfloat16()
    dy = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    wt = ops.transpose2d(w, torch.empty(K, N, device="cuda", dtype=torch.bfloat16))
    a = ops.linear_dx(dy, w)
    b = ops.linear_dx_t(dy, wt)
    assert torch.equal(a, b)
    ref = dy.float() @ w.float()
    assert ((b.float() - ref).norm() / ref.norm()).item() < 1e-2


@pytest.mark.parametrize("state_dtype", [torch.bfloat16, torch.float32])
def test_adamw_vector_path_bitwise_equals_scalar_path(state_dtype):
    """The 8-wide AdamW path (16-B aligned buffers) and the element-wise path (a buffer offset
    by one element) give bitwise-equal params and moments; n is ragged so the tail runs too."""
    n = 3 * 65536 + 13
    g0 = torch.Generator(device="cuda").manual_seed(5)
    base = {k: torch.randn(n + 8, device="cuda", generator=g0) * 0.1 for k in ("p", "g")}
    outs = []
    for off in (0, 1):
        p = base["p"].bfloat16()[:n].clone() if off == 0 else _misaligned(base["p"].bfloat16(), n)
        g = base["g"].bfloat16()[:n].clone() if off == 0 else _misaligned(base["g"].bfloat16(), n)
        m = torch.zeros(n + 8, device="cuda", dtype=state_dtype)[off:off + n]
        v = torch.zeros(n + 8, device="cuda", dtype=state_dtype)[off:off + n]
        for step in (1, 2, 3):
            ops().adamw(p, g, m, v, lr=1e-2, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.1, step=step)
        outs.append((p.clone(), m.clone(), v.clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def _misaligned(t, n):
    buf = torch.empty(n + 8, device=t.device, dtype=t.dtype)
    view = buf[1:1 + n]
    view.copy_(t[:n])
    return view


@pytest.mark.parametrize("D,H,inverse", [(128, 32, 0), (128, 32, 1), (64, 3, 0), (16, 5, 1)])
def test_rope_vector_path_bitwise_equals_element_path(D, H, inverse):
    """rope8_k (LDS cos/sin table, 16-B rows) and rope_k (4-wide, taken for rows that are not
    16-B aligned) give bitwise-equal q and k, forward and inverse, on the fused q|k|v layout."""
    T = 70
    g = torch.Generator(device="cuda").manual_seed(D + H)
    qkv = torch.randn(T, 3 * H * D, device="cuda", generator=g).bfloat16()
    pos = torch.randint(0, 1100, (T,), device="cuda", generator=g)
    a = qkv.clone()
    ops().rope(a[:, :H * D], a[:, H * D:2 * H * D], pos, hq=H, hk=H, head_dim=D, theta=10000.0, inverse=inverse)
    buf = torch.empty(T * 3 * H * D + 1, device="cuda", dtype=torch.bfloat16)
    b = buf[1:].view(T, 3 * H * D)  # 2-B offset: not 16-B aligned -> element path
    b.copy_(qkv)
    ops().rope(b[:, :H * D], b[:, H * D:2 * H * D], pos, hq=H, hk=H, head_dim=D, theta=10000.0, inverse=inverse)
    assert torch.equal(a, b)


def test_sumsq_deterministic_and_accurate():
    """the grad-norm sum of squares is bit-identical across repeats (fixed-order partials, no
    float atomics) and matches a float64 sum; ragged n exercises the tail"""
    x = (torch.randn(50_000_003, device=DEV) * 1e-2).bfloat16()
    vals = []
    for _ in range(5):
        acc = torch.zeros(1, device=DEV)
        ops().sumsq(x, acc)
        vals.append(acc.item())
    assert len(set(vals)) == 1
    ref = x.double().pow(2).sum().item()
    assert abs(vals[0] - ref) <= 1e-5 * ref


@pytest.mark.parametrize("left", [False, True])
def test_merge_plan_long_rows_bit_exact(left):
    """rows longer than one 1024-wide scan chunk (S=1300 text ids, 576 patches per image, two
    images in one row, padded rows): the chunk carries of the workgroup scans match the oracle"""
    cfg = O.config_small_gpu()
    B, S, P, D = 3, 1300, 576, 8
    g = torch.Generator().manual_seed(7)
    ids = torch.randint(2, cfg.image_token_index - 1, (B, S), generator=g)
    ids[0, 35] = cfg.image_token_index
    ids[1, 10] = ids[1, 900] = cfg.image_token_index
    ids[2, 1200] = cfg.image_token_index
    mask = torch.ones(B, S, dtype=torch.long)
    for b, n in ((0, 0), (1, 200), (2, 37)):
        if n:
            if left:
                ids[b] = torch.cat([torch.full((n,), cfg.pad_token_id), ids[b, :S - n]])
                mask[b, :n] = 0
            else:
                ids[b, S - n:] = cfg.pad_token_id
                mask[b, S - n:] = 0
    n_img = int((ids == cfg.image_token_index).sum())
    emb = rnd((B, S, D), 97)
    img = rnd((n_img, P, D), 98)
    cfg_p = type("C", (), dict(pad_token_id=cfg.pad_token_id, image_token_index=cfg.image_token_index,
                               ignore_index=-100, vision=type("V", (), dict(num_patches=P))()))()
    r_emb, r_mask, _, r_pos = O.merge(img, emb, ids, mask, cfg_p)
    L = r_emb.shape[1]
    left_pad = not bool((ids[:, -1] == cfg.pad_token_id).sum())
    assert left_pad == left
    td, src, mm, pos = ops().merge_plan(ids.to(DEV), mask.to(DEV), L=L, image_token=cfg.image_token_index,
                                       n_patches=P, left_padding=left_pad)
    out = ops().row_gather2(src.reshape(-1), emb.to(DEV).reshape(-1, D), img.to(DEV).reshape(-1, D))
    assert torch.equal(out.cpu().view(B, L, D), r_emb)
    assert torch.equal(mm.cpu(), r_mask.long())
    assert torch.equal(pos.cpu(), r_pos)


@pytest.mark.parametrize("M,N,K,al,bl,epi", [(8704, 4096, 4096, 0, 1, "none"), (8704, 4096, 11008, 0, 0, "res"),
                                              (1000, 776, 1024, 0, 0, "bias"), (577, 520, 640, 0, 1, "none"),
                                              (300, 264, 4096, 0, 1, "beta"), (8704, 12288, 4096, 0, 0, "none"),
                                              (36928, 1024, 4096, 0, 0, "res")])
def test_gemm_288_rows_bitwise_vs_256(M, N, K, al, bl, epi):
    """The 288x256 tile (mode 10: 9 MFMA rows per wave, 36 A pieces over the loader waves, 144 KiB
    LDS epilogue) accumulates every output element over the same K order as the 256x256 tile, so their outputs
    are bitwise equal: the 7B dX (o_proj) and down-projection forward shapes it is planned for, ragged M (rows past M of the last 288-row tile), K % 64 != 0,
    accumulate (beta = 1), residual and bias epilogues. Also checks the plan picks it for the 7B
    dX shape and not for the ViT's K = 1024 products."""
    from cullavo_amd import _lib
    L = _lib.lib()
    if (M, N, K) == (8704, 4096, 4096):
        assert L.cullavo_gemm_plan(M, N, K, al, bl, None) == 10
    assert L.cullavo_gemm_plan(36928, 4096, 1024, 0, 0, None) != 10
    A = rnd((K, M) if al else (M, K), 95).to(DEV)
    B = rnd((K, N) if bl else (N, K), 96).to(DEV)
    bias = rnd((N,), 97).to(DEV) if epi == "bias" else None
    res = rnd((M, N), 98).to(DEV) if epi == "res" else None
    beta = 1.0 if epi == "beta" else 0.0
    C0 = rnd((M, N), 99).to(DEV)
    outs = {}
    for tile in (10, 2):
        prev = L.cullavo_gemm_set_tile(tile)
        try:
            C = C0.clone()
            ops().gemm(al, bl, M, N, K, A, A.stride(0), B, B.stride(0), C, N, bias=bias, residual=res,
                       ldr=N if res is not None else 0, beta=beta)
            torch.cuda.synchronize()
        finally:
            L.cullavo_gemm_set_tile(prev)
        outs[tile] = C
    assert torch.equal(outs[10], outs[2])
    # fp32 check on sampled rows and columns (every shape, the M = 8,704 ones included): the last
    # 64 rows (the ragged last 288-row tile at M = 8,704), the first rows and random ones
    g = torch.Generator().manual_seed(M + N + K)
    rows = torch.cat([torch.arange(min(64, M)), torch.arange(max(0, M - 64), M),
                      torch.randint(0, M, (128,), generator=g)]).unique()
    cols = torch.cat([torch.arange(min(32, N)), torch.arange(max(0, N - 32), N),
                      torch.randint(0, N, (96,), generator=g)]).unique()
    Ar = (A.T[rows.to(DEV)] if al else A[rows.to(DEV)]).float().cpu()          # [r, K]
    Bc = (B.T[cols.to(DEV)] if bl else B[cols.to(DEV)]).float().cpu()          # [c, K]
    z = Ar @ Bc.T
    if bias is not None:
        z = z + bias.float().cpu()[cols]
    if res is not None:
        z = z.to(BF).float() + res.float().cpu()[rows][:, cols]
    z = z + beta * C0.float().cpu()[rows][:, cols]
    close(outs[10].cpu()[rows][:, cols], z, 8e-3, f"288x256 {M}x{N}x{K} (sampled rows/cols)")


@pytest.mark.gpu
@pytest.mark.parametrize("thr", [0.0, 8.0])
def test_attention_fwd_pipelined_rescale_bitwise(thr):
    """The pipelined forward (stage 7) takes the deferred-rescale branch at the same tiles as stage 4
    and rescales O and l and nothing else: bitwise equal O / LSE at threshold 0 (rescale at every
    max growth) and 8, on a spike key in the 4th tile that moves every later row's max (the
    construction of test_attention_rescale_threshold) and a ragged causal length."""
    from cullavo_amd import _lib
    B, H, L, D = 2, 2, 1000, 128
    u = rnd((1, 1, H, D), 78).float()
    q = (rnd((B, L, H, D), 75).float() + u).reshape(B * L, H * D).to(BF)
    kh = rnd((B, L, H, D), 76).float()
    v = rnd((B * L, H * D), 77)
    kh[:, 230] = 3.0 * u[0, 0]
    kh[:, 700] = 3.5 * u[0, 0]
    k = kh.reshape(B * L, H * D).to(BF)
    kw = dict(B=B, H=H, Lq=L, Lk=L, D=D, scale=D ** -0.5, causal=True)
    L_ = _lib.lib()
    prev = L_.cullavo_attn_set_stage(4)
    try:
        assert L_.cullavo_attn_set_rescale(ctypes.c_float(thr), None) == 0
        o4, lse4 = ops().attn_fwd(q.to(DEV), k.to(DEV), v.to(DEV), **kw)
        L_.cullavo_attn_set_stage(7)
        o7, lse7 = ops().attn_fwd(q.to(DEV), k.to(DEV), v.to(DEV), **kw)
    finally:
        L_.cullavo_attn_set_stage(prev)
        L_.cullavo_attn_set_rescale(ctypes.c_float(8.0), None)
    dl = (lse4 - lse7).abs()
    bad = (lse4 != lse7) & ~(lse4.isnan() & lse7.isnan())
    assert torch.equal(o4, o7), ((o4.float() - o7.float()).abs().max().item())
    assert not bad.any(), (int(bad.sum()), dl[bad].max().item(), bad.nonzero()[:8].tolist(),
                           lse4[bad][:4].tolist(), lse7[bad][:4].tolist())
    _, _, _, o_ref = _attn_ref(q, k, v, B, H, L, D, True)
    close(o7, o_ref.transpose(1, 2).reshape(B * L, H * D), 1.2e-2, "attn o (stage 7)")
