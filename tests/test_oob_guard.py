"""Out-of-range rows and K tails must read as zeros, proven with NaN neighbours.

The LDS-DMA / buffer-load staging of the GEMM and attention kernels relies on the buffer range
check to zero-fill rows past an operand's end (K tails of layout-1 GEMM operands, rows past the
sequence end in attention tiles). Zeroed allocator slack after a tensor cannot tell a real
zero-fill from a read of the neighbouring memory, so here every operand is a view of a larger
tensor whose memory after the operand (and between its rows) holds NaN: a single stray read
turns into NaN in the output (NaN * 0 = NaN). Outputs must be finite, equal across the staging
modes, and match the fp32 restatement (gemm.hip dma_pre, attention.hip StageT).
"""
import pytest
import torch

from oracle import cullavo_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF = torch.bfloat16
NAN = float("nan")


def rnd(shape, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(shape, generator=g).to(BF)


def nan_view(data, extra_rows=128, extra_cols=0):
    """`data` copied into the top-left of a NaN-filled [rows + extra_rows, cols + extra_cols]
    device tensor; returns the view (same shape as data, row stride cols + extra_cols)"""
    r, c = data.shape
    big = torch.full((r + extra_rows, c + extra_cols), NAN, dtype=data.dtype, device=DEV)
    big[:r, :c] = data.to(DEV)
    return big[:r, :c]


def close(out, ref, tol, what):
    out, ref = out.float().cpu(), ref.float().cpu()
    assert torch.isfinite(out).all(), f"{what}: non-finite output (a read past the operand)"
    err = (out - ref).abs().max().item()
    scale = ref.abs().max().item() + 1e-12
    assert err <= tol * scale, f"{what}: max|err| {err:.3e} > {tol:.1e} * {scale:.3e}"


@pytest.mark.parametrize("tile", [-1, 2, 10])
@pytest.mark.parametrize("al,bl", [(1, 1), (1, 0), (0, 1), (0, 0)])
@pytest.mark.parametrize("K", [1000, 1160, 4096])
def test_gemm_k_tail_reads_zeros_next_to_nan(tile, al, bl, K):
    from cullavo_amd import _lib, ops
    L = _lib.lib()
    M, N = 1000, 776
    A = rnd((M, K), 301)
    B = rnd((N, K), 302)
    bias = rnd((N,), 303)
    ref = A.float() @ B.float().T + bias.float()
    # layout 1 stores [K, rows]: NaN rows past K and NaN columns past M / N (row stride + 24);
    # layout 0 stores [rows, K]: NaN columns past K and NaN rows past M / N
    Ad = nan_view(A.T.contiguous(), 128, 24) if al else nan_view(A, 128, 72)
    Bd = nan_view(B.T.contiguous(), 128, 24) if bl else nan_view(B, 128, 72)
    outs = []
    prev_t = L.cullavo_gemm_set_tile(tile)
    try:
        for mode in (1, 0):
            prev = L.cullavo_gemm_set_dma(mode)
            C = torch.empty((M, N), dtype=BF, device=DEV)
            ops.gemm(al, bl, M, N, K, Ad, Ad.stride(0), Bd, Bd.stride(0), C, N, bias=bias.to(DEV))
            torch.cuda.synchronize()
            L.cullavo_gemm_set_dma(prev)
            outs.append(C)
    finally:
        L.cullavo_gemm_set_tile(prev_t)
    close(outs[0], ref, 8e-3, f"dma_pre tile {tile} layouts {al}{bl} K={K}")
    close(outs[1], ref, 8e-3, f"dma per-tile tile {tile} layouts {al}{bl} K={K}")
    assert torch.equal(outs[0], outs[1])


def test_gemm_dw_ragged_token_count_next_to_nan():
    """the weight-gradient product dW = dY^T X at a token count that is not a multiple of 64
    (a ragged B*L): both operands layout 1 with NaN token rows after the last one"""
    from cullavo_amd import ops
    T, N, K_ = 1037, 4096, 1024  # tokens, out features, in features
    dy = rnd((T, N), 311)
    x = rnd((T, K_), 312)
    ref = dy.float().T @ x.float()
    dyd, xd = nan_view(dy, 128), nan_view(x, 128)
    C = torch.empty((N, K_), dtype=BF, device=DEV)
    ops.gemm(1, 1, N, K_, T, dyd, dyd.stride(0), xd, xd.stride(0), C, K_)
    close(C, ref, 8e-3, "dW ragged T")


ATTN = [(2, 2, 200, 128, True), (2, 3, 577, 64, False), (1, 2, 1088 - 5, 128, True)]


def _attn_ref(q, k, v, do, B, H, L, D, causal):
    qf, kf, vf = (t.float().view(B, L, H, D).transpose(1, 2).requires_grad_(True) for t in (q, k, v))
    allowed = O.causal_allowed(torch.ones(B, L, dtype=torch.long)) if causal else None
    o = O.attention(qf, kf, vf, D ** -0.5, allowed)
    o.backward(do.float().view(B, L, H, D).transpose(1, 2))
    tr = lambda t: t.transpose(1, 2).reshape(B * L, H * D)
    return tr(o.detach()), tr(qf.grad), tr(kf.grad), tr(vf.grad)


@pytest.mark.parametrize("B,H,L,D,causal", ATTN)
def test_attention_rows_past_end_next_to_nan(B, H, L, D, causal):
    """q|k|v as column blocks of a fused [T, 3*H*D] buffer followed by NaN rows, dO and O
    followed by NaN rows; L not a multiple of 64, so the last tile of the last sequence reaches
    past the tensor. Every forward staging mode and every backward tile / staging mode."""
    from cullavo_amd import _lib, ops
    Lb = _lib.lib()
    hd = H * D
    T = B * L
    q, k, v, do = (rnd((T, hd), s) for s in (321, 322, 323, 324))
    o_ref, dq_ref, dk_ref, dv_ref = _attn_ref(q, k, v, do, B, H, L, D, causal)
    qkv = nan_view(torch.cat([q, k, v], 1), 128)
    qd, kd, vd = qkv[:, :hd], qkv[:, hd:2 * hd], qkv[:, 2 * hd:]
    dod = nan_view(do, 128)
    kw = dict(B=B, H=H, Lq=L, Lk=L, D=D, scale=D ** -0.5, causal=causal)
    outs = {}
    prev = Lb.cullavo_attn_set_stage(4)
    try:
        for st in (0, 1, 2, 4, 5, 7):
            Lb.cullavo_attn_set_stage(st)
            o, lse = ops.attn_fwd(qd, kd, vd, **kw)
            close(o, o_ref, 1.2e-2, f"attn o stage {st}")
            outs[st] = (o, lse)
    finally:
        Lb.cullavo_attn_set_stage(prev)
    for st in (0, 1, 2, 5, 7):
        assert torch.equal(outs[st][0], outs[4][0]), f"O stage {st} vs 4"
    o, lse = outs[4]
    od = nan_view(o.cpu(), 128)
    lse_d = lse  # [B, H, L] f32, read per row with its own bound
    prev_t = Lb.cullavo_attn_set_bwd_tiles(7)
    prev_s = Lb.cullavo_attn_set_bwd_stage(0)
    try:
        base = None
        for tiles in ((7, 4) if D == 128 else (0, 4)):
            Lb.cullavo_attn_set_bwd_tiles(tiles)
            for st in range(16):  # bit 2: the LDS-DMA ring dQ kernel (D = 128), bit 3: blocked dS^T
                Lb.cullavo_attn_set_bwd_stage(st)
                dq, dk, dv = ops.attn_bwd(qd, kd, vd, od, dod, lse_d, **kw)
                torch.cuda.synchronize()
                tag = f"tiles {tiles} stage {st}"
                close(dq, dq_ref, 2e-2, f"dq {tag}")
                close(dk, dk_ref, 2e-2, f"dk {tag}")
                close(dv, dv_ref, 2e-2, f"dv {tag}")
                if st == 0:
                    base = (dq, dk, dv)
                else:
                    for name, a, b in zip("qkv", base, (dq, dk, dv)):
                        assert torch.equal(a, b), f"d{name} {tag} vs stage 0"
    finally:
        Lb.cullavo_attn_set_bwd_tiles(prev_t)
        Lb.cullavo_attn_set_bwd_stage(prev_s)
