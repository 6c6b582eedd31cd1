"""Production kernels pinned at accumulation accuracy, not at a fraction of
the bf16 output noise.

GEMM (every config-3 shape class of the 7B step, the ViT's K = 1024 products, ragged M / K tails):
  1. the kernel with an f32 output (the same tile plan, main loop and MFMA order as the bf16
     product; only the epilogue's store differs) on bf16-exact operands against the f64 product:
     rel-L2 <= 1e-5 (measured 1.8e-7 at K = 1024 .. 9.5e-7 at K = 22016), and element-wise the
     classical bound of any f32 summation order, |c - ref| <= K * 2^-24 * (|A| |B|^T) (a dropped,
     doubled or mis-placed 64-deep K-slab breaks it by ~10x at K = 4096). The max relative error
     over |ref| > 1e-3 max|ref| (VERDICT r05 asked <= 1e-4) is logged, not gated: f32 accumulation
     alone puts it at 1.4e-4 (K = 1024) .. 6.5e-4 (K = 22016) for a correct kernel, since such small
     outputs are sums of terms ~1000x larger;
  2. the production bf16 output (persistent / 288-row / 256-row / split kernels as the plan picks
     them) BITWISE equal to bf16(that f32 output): the bf16 kernels round the same f32 accumulator
     once, so anything they drop, double-count or mis-order shows up as a bit difference.
Attention (config-3 head shape D = 128 causal at L = 1088, ViT D = 64 non-causal at L = 577):
  the f32 LSE within 1e-5 of the f64 log-sum-exp (measured 1.2e-6); O, dQ, dK, dV (bf16) within
  rel-L2 3e-3 of the f64 reference (measured 2.0-2.5e-3: the FA2 arithmetic rounds P and dS to bf16
  once per element, ~1.1e-3 each, plus the output's own bf16 rounding ~1.1e-3) and element-wise
  within 2^-3 of (|ref| + rms of ref's row) (one head's D values of one token; + 1e-3 of the
  tensor's rms for rows whose exact value is 0; the reference's delta = rowsum(dO * O) uses the
  forward's stored O, as FA2 does): a dropped or
  double-counted key / query tile moves the rows it touches by ~0.3 of their size and fails it.
The f64 references run on the GPU (torch), the checked kernels through the C-ABI (ops.*). Stats of
every case are appended to gpurun_out/accuracy_stats.jsonl on the box.
"""
import json
import os
import zlib

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"
BF = torch.bfloat16
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out", "accuracy_stats.jsonl")


def ops():
    from cullavo_amd import ops as _ops
    return _ops


def _log(rec):
    try:
        os.makedirs(os.path.dirname(OUT), exist_ok=True)
        with open(OUT, "a") as f:
            f.write(json.dumps(rec) + "\n")
    except OSError:
        pass


# (name, M, N, K, a_layout, b_layout): forward Y = X W^T (0,0), dX = dY W (0,1), dW = dY^T X (1,1)
GEMM_CASES = [
    ("qkv_fwd", 8704, 12288, 4096, 0, 0), ("o_fwd", 8704, 4096, 4096, 0, 0),
    ("gateup_fwd", 8704, 22016, 4096, 0, 0), ("down_fwd", 8704, 4096, 11008, 0, 0),
    ("lmhead_fwd", 8704, 32064, 4096, 0, 0),
    ("qkv_dx", 8704, 4096, 12288, 0, 1), ("gateup_dx", 8704, 4096, 22016, 0, 1),
    ("down_dx", 8704, 11008, 4096, 0, 1), ("o_dx", 8704, 4096, 4096, 0, 1),
    ("qkv_dw", 12288, 4096, 8704, 1, 1), ("gateup_dw", 22016, 4096, 8704, 1, 1),
    ("down_dw", 4096, 11008, 8704, 1, 1), ("lmhead_dw", 32064, 4096, 8704, 1, 1),
    ("vit_fc1", 36928, 4096, 1024, 0, 0), ("vit_qkv", 36928, 3072, 1024, 0, 0),
    ("vit_fc2", 36928, 1024, 4096, 0, 0),
    ("ragged_m_fwd", 8704 + 37, 4096, 4096, 0, 0), ("ragged_m_dx", 8704 + 45, 4096, 4096, 0, 1),
    ("ragged_dw", 4104, 4096, 8704 + 40, 1, 1), ("ragged_k_fwd", 2000, 3072, 4096 + 72, 0, 0),
]


@pytest.mark.parametrize("name,M,N,K,al,bl", GEMM_CASES, ids=[c[0] for c in GEMM_CASES])
def test_gemm_f32_accumulation_and_bf16_bitwise(name, M, N, K, al, bl):
    g = torch.Generator(device=DEV).manual_seed(zlib.crc32(name.encode()))
    A = torch.randn((K, M) if al else (M, K), device=DEV, generator=g).to(BF)
    B = torch.randn((K, N) if bl else (N, K), device=DEV, generator=g).to(BF)
    Ad = A.t() if al else A
    Bd = B if bl else B.t()  # [K, N]
    ref = Ad.double() @ Bd.double()
    del Ad, Bd
    c32 = torch.empty((M, N), dtype=torch.float32, device=DEV)
    ops().gemm_ex(al, bl, M, N, K, A, A.stride(0), B, B.stride(0), c32, N)
    c16 = torch.empty((M, N), dtype=BF, device=DEV)
    ops().gemm_ex(al, bl, M, N, K, A, A.stride(0), B, B.stride(0), c16, N)
    torch.cuda.synchronize()
    err = c32.double() - ref
    rel_l2 = (err.norm() / ref.norm()).item()
    big = ref.abs() > 1e-3 * ref.abs().max()
    max_rel = (err.abs()[big] / ref.abs()[big]).max().item()
    del ref, big
    Aa = (A.t() if al else A).double().abs()
    Ba = (B if bl else B.t()).double().abs()
    bound_ratio = (err.abs() / (Aa @ Ba)).max().item() / (K * 2.0 ** -24)
    del Aa, Ba, err
    ndiff = int((c16 != c32.to(BF)).sum().item())
    _log({"test": "gemm", "case": name, "M": M, "N": N, "K": K, "layouts": [al, bl], "rel_l2_f32": rel_l2,
          "max_rel_f32": max_rel, "err_over_f32_bound": bound_ratio, "bf16_bits_differing": ndiff})
    assert rel_l2 <= 1e-5, f"{name}: f32-output rel-L2 {rel_l2:.2e} vs f64"
    assert bound_ratio <= 1.0, f"{name}: f32-output error {bound_ratio:.2f} x the f32 summation bound K u |A||B|"
    assert ndiff == 0, f"{name}: {ndiff} bf16 outputs differ from bf16(f32 output of the same product)"


def _attn_ref(q, k, v, do, B, H, L, D, scale, causal, o_kernel):
    """f64 attention forward + backward of [B*L, H*D] row-major q, k, v, dO. The backward's
    delta = rowsum(dO * O) takes the forward's output as stored (o_kernel, bf16), as FA2 defines it:
    with the exact O instead, rows with few live keys (the causal diagonal's first queries) differ by
    the cancellation in dP - delta, not by anything the backward kernels compute."""
    def heads(x):
        return x.double().view(B, L, H, D).transpose(1, 2)  # [B, H, L, D]
    Q, Kt, V, dO = heads(q), heads(k), heads(v), heads(do)
    S = (Q @ Kt.transpose(-1, -2)) * scale
    if causal:
        S = S.masked_fill(torch.ones(L, L, dtype=torch.bool, device=DEV).triu(1), float("-inf"))
    lse = torch.logsumexp(S, -1)
    P = torch.exp(S - lse[..., None])
    O = P @ V
    dV = P.transpose(-1, -2) @ dO
    dP = dO @ V.transpose(-1, -2)
    delta = (dO * heads(o_kernel)).sum(-1, keepdim=True)
    dS = P * (dP - delta)
    dQ = dS @ Kt * scale
    dK = dS.transpose(-1, -2) @ Q * scale

    def flat(x):
        return x.transpose(1, 2).reshape(B * L, H * D)
    return flat(O), lse, flat(dQ), flat(dK), flat(dV)


ATTN_CASES = [("lm_d128_causal", 2, 4, 1088, 128, True), ("vit_d64", 2, 4, 577, 64, False),
              ("lm_d128_ragged", 1, 3, 1000, 128, True)]


@pytest.mark.parametrize("name,B,H,L,D,causal", ATTN_CASES, ids=[c[0] for c in ATTN_CASES])
def test_attention_against_f64(name, B, H, L, D, causal):
    g = torch.Generator(device=DEV).manual_seed(11)
    q, k, v, do = (torch.randn(B * L, H * D, device=DEV, generator=g).to(BF) for _ in range(4))
    scale = D ** -0.5
    o, lse = ops().attn_fwd(q, k, v, B=B, H=H, Lq=L, Lk=L, D=D, scale=scale, causal=causal)
    dq, dk, dv = ops().attn_bwd(q, k, v, o, do, lse, B=B, H=H, Lq=L, Lk=L, D=D, scale=scale, causal=causal)
    torch.cuda.synchronize()
    O, LSE, dQ, dK, dV = _attn_ref(q, k, v, do, B, H, L, D, scale, causal, o)
    rec = {"test": "attention", "case": name, "B": B, "H": H, "L": L, "D": D, "causal": causal}
    lse_err = (lse.double() - LSE).abs().max().item()
    rec["lse_max_abs"] = lse_err
    fails = []
    if not lse_err <= 1e-5:
        fails.append(f"lse max|err| {lse_err:.2e}")
    for nm, out, ref in (("O", o, O), ("dQ", dq, dQ), ("dK", dk, dK), ("dV", dv, dV)):
        err = out.double() - ref
        rel = (err.norm() / ref.norm()).item()
        row_rms = ref.view(-1, H, D).pow(2).mean(-1, keepdim=True).sqrt().expand(-1, H, D).reshape(ref.shape)
        # (+ 1e-3 of the tensor's rms: rows whose exact value is 0, e.g. dQ of query 0 under the
        # causal mask, where the kernel's f32 dP - delta leaves ~1e-7)
        floor = 1e-3 * ref.pow(2).mean().sqrt()
        worst = (err.abs() / (ref.abs() + row_rms + floor)).max().item()
        rec[f"{nm}_rel_l2"] = rel
        rec[f"{nm}_max_row_scaled"] = worst
        if not rel <= 3e-3:
            fails.append(f"{nm} rel-L2 {rel:.2e}")
        if not worst <= 2 ** -3:
            fails.append(f"{nm} max |err| / (|ref| + row rms) {worst:.2e}")
    _log(rec)
    assert not fails, f"{name}: " + "; ".join(fails)
