"""Parity of the HIP path at the tolerances the north star and SURVEY.md §7 state.

Two modes, two gates (SURVEY.md §7 "Hard parts: parity tolerance"):

* f32 parity mode (CuLLaVOModel(dtype=torch.float32)): every parameter, activation and kernel
  operand is f32 (gemm_f32.hip on v_mfma_f32_16x16x4_f32, attn_generic.hip, the f32 variants
  of the norm / element-wise / loss kernels). Gate against the REFERENCE's own fp32 forward and
  backward (tests/golden/*.npz, made by tests/golden/make_golden.py from
  reference cullavo/arch_cullavo.py:546-677): logits relative-L2 <= 1e-3 (north_star: "logits
  within 1e-3 rel of reference"), |loss - ref| <= 1e-4, gradient norms within 1e-3 relative and
  sampled gradients relative-L2 <= 1e-3.
* bf16 production mode against the bf16-faithful oracle (oracle/cullavo_oracle.py, bf16
  weights: the reference's bf16-cast model under bf16 autocast, reference
  cullavo/load_cullavo.py:123-126): logits relative-L2 <= 1e-2 and |loss - ref| <= 1e-2.

The kernels behind the f32 mode are also checked one by one against float64 torch.
"""
import os

import numpy as np
import pytest
import torch

from oracle import cullavo_oracle as O

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")

CASES = {
    "config1": ("config1", dict(batch=2, text_len=32, image_col=5, seed=0)),
    "config1_pad": ("config1", dict(batch=2, text_len=32, image_col=5, seed=1, pad_tail=[0, 7])),
    "small_gpu": ("small_gpu", dict(batch=2, text_len=40, image_col=4, seed=2)),
}


def ops():
    from cullavo_amd import ops as _ops
    return _ops


def rel_l2(a, b):
    a = torch.as_tensor(np.asarray(a, dtype=np.float64)) if not torch.is_tensor(a) else a.detach().double().cpu()
    b = torch.as_tensor(np.asarray(b, dtype=np.float64)) if not torch.is_tensor(b) else b.detach().double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def _configs(kind):
    from cullavo_amd import config as C
    return (C.config1(), O.config1()) if kind == "config1" else (C.tiny_gpu(), O.config_small_gpu())


def _model(kind, seed, dtype, trainable="full"):
    from cullavo_amd.arch_cullavo import CuLLaVOModel
    cfg, ocfg = _configs(kind)
    m = CuLLaVOModel(cfg, device="cuda", trainable=trainable, init="none", dtype=dtype)
    W = O.make_weights(ocfg, seed)
    m.load_state_dict(W)
    return m, ocfg, W


def _inputs(ocfg, kw):
    return O.make_inputs(ocfg, kw["batch"], kw["text_len"], kw["image_col"], kw["seed"], pad_tail=kw.get("pad_tail"))


# ---- kernels of the f32 mode -------------------------------------------------------------------
@pytest.mark.parametrize("al,bl", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_gemm_f32_operands_epilogue(al, bl):
    """f32 GEMM, every layout, bias + GELU + preact + residual + beta, vs float64"""
    g = torch.Generator(device="cuda").manual_seed(al * 2 + bl)
    M, N, K = 264, 136, 200
    A = torch.randn(M, K, device="cuda", generator=g) if al == 0 else torch.randn(K, M, device="cuda", generator=g)
    B = torch.randn(N, K, device="cuda", generator=g) if bl == 0 else torch.randn(K, N, device="cuda", generator=g)
    bias = torch.randn(N, device="cuda", generator=g)
    res = torch.randn(M, N, device="cuda", generator=g)
    C0 = torch.randn(M, N, device="cuda", generator=g)
    C = C0.clone()
    pre = torch.empty(M, N, device="cuda")
    ops().gemm(al, bl, M, N, K, A, A.stride(0), B, B.stride(0), C, N, alpha=0.5, bias=bias, act=ops().ACT_GELU,
               preact=pre, residual=res, ldr=N, beta=0.25)
    torch.cuda.synchronize()
    Ad = (A if al == 0 else A.T).double()
    Bd = (B.T if bl == 0 else B).double()
    z = 0.5 * (Ad @ Bd) + bias.double()
    ref = torch.nn.functional.gelu(z) + res.double() + 0.25 * C0.double()
    assert (pre.double() - z).abs().max().item() <= 2e-5 * z.abs().max().item()
    assert (C.double() - ref).abs().max().item() <= 2e-5 * ref.abs().max().item()


@pytest.mark.parametrize("mode", [1, 2, 3])
def test_gemm_f32_lora_dropout(mode):
    """operand / output dropout masks of the f32 kernel = the counter hash restated in numpy"""
    g = torch.Generator(device="cuda").manual_seed(7)
    T, F_in, F_out, p, seed = 136, 96, 64, 0.25, 123456789
    x = torch.randn(T, F_in, device="cuda", generator=g)
    keep = torch.as_tensor(O.lora_keep_mask(seed, T, F_in if mode != 3 else F_out, p), device="cuda")
    if mode == 1:  # y = dropout(x) A^T, A [F_out, F_in]
        A = torch.randn(F_out, F_in, device="cuda", generator=g)
        y = torch.empty(T, F_out, device="cuda")
        ops().gemm_ex(0, 0, T, F_out, F_in, x, F_in, A, F_in, y, F_out, drop_operand=1, drop_p=p, drop_seed=seed)
        ref = (x.double() * keep / (1 - p)) @ A.double().T
    elif mode == 2:  # dA = du^T dropout(x): A = du [T, r] read as [K=T][M=r], B = x [T, F_in]
        du = torch.randn(T, F_out, device="cuda", generator=g)
        y = torch.empty(F_out, F_in, device="cuda")
        ops().gemm_ex(1, 1, F_out, F_in, T, du, F_out, x, F_in, y, F_in, drop_operand=2, drop_p=p, drop_seed=seed)
        ref = du.double().T @ (x.double() * keep / (1 - p))
    else:  # output dropout on y[token, feature]
        A = torch.randn(F_out, F_in, device="cuda", generator=g)
        y = torch.empty(T, F_out, device="cuda")
        ops().gemm_ex(0, 0, T, F_out, F_in, x, F_in, A, F_in, y, F_out, drop_operand=3, drop_p=p, drop_seed=seed)
        ref = (x.double() @ A.double().T) * keep / (1 - p)
    torch.cuda.synchronize()
    assert (y.double() - ref).abs().max().item() <= 2e-5 * ref.abs().max().item()


# bf16 at D 64/128 runs the MFMA kernels (tests/test_ops_gpu.py)
@pytest.mark.parametrize("D,dtype", [(16, torch.float32), (32, torch.float32), (64, torch.float32),
                                     (128, torch.float32), (16, torch.bfloat16), (32, torch.bfloat16)])
@pytest.mark.parametrize("causal", [True, False])
def test_attention_generic(D, dtype, causal):
    """attn_generic.hip (f32 storage; bf16 at head dims 16/32) fwd + bwd vs float64, left
    padding through kv_start, ragged L (not a multiple of the 64-row blocks)."""
    B, H, L = 2, 3, 131
    g = torch.Generator(device="cuda").manual_seed(D + causal)
    q, k, v, do = (torch.randn(B * L, H * D, device="cuda", generator=g).to(dtype) for _ in range(4))
    ks = torch.tensor([0, 9], dtype=torch.int32, device="cuda")
    scale = D ** -0.5
    o, lse = ops().attn_fwd(q, k, v, B=B, H=H, Lq=L, Lk=L, D=D, scale=scale, causal=causal, kv_start=ks)
    dq, dk, dv = ops().attn_bwd(q, k, v, o, do, lse, B=B, H=H, Lq=L, Lk=L, D=D, scale=scale, causal=causal,
                                kv_start=ks)
    torch.cuda.synchronize()

    def heads(t):
        return t.double().cpu().view(B, L, H, D).transpose(1, 2).requires_grad_(True)
    qd, kd, vd = heads(q), heads(k), heads(v)
    j = torch.arange(L)
    allowed = (j[None, None, None, :] >= ks.cpu().long()[:, None, None, None])
    if causal:
        allowed = allowed & (j[None, None, None, :] <= j[None, None, :, None])
    s = (qd @ kd.transpose(-1, -2)) * scale
    s = s.masked_fill(~allowed, float("-inf"))
    pr = torch.nan_to_num(torch.softmax(s, -1), nan=0.0)
    od = pr @ vd
    od.backward(heads(do).detach())
    tol = 2e-5 if dtype == torch.float32 else 2e-2
    flat = lambda t: t.transpose(1, 2).reshape(B * L, H * D)  # noqa: E731
    rows_ok = torch.ones(B * L, dtype=torch.bool)
    rows_ok[L:L + 9] = False  # fully masked rows (batch 1, queries < kv_start) in causal mode
    for ours, ref in ((o, flat(od)), (dq, flat(qd.grad)), (dk, flat(kd.grad)), (dv, flat(vd.grad))):
        a, b = ours.double().cpu(), ref.detach()
        if causal:
            a, b = a[rows_ok], b[rows_ok]
        assert rel_l2(a, b) <= tol, (rel_l2(a, b), tol)
    if causal:  # rows that see no key: zero output, lse = +inf, no gradient
        assert o.float().cpu()[~rows_ok].abs().max().item() == 0.0
        assert torch.isinf(lse[1, :, :9]).all()


# ---- end to end --------------------------------------------------------------------------------
@pytest.mark.parametrize("name", list(CASES))
def test_f32_mode_matches_reference_golden(name):
    """CuLLaVOModel in the f32 parity mode vs the reference's own fp32 forward/backward"""
    kind, kw = CASES[name]
    g = np.load(os.path.join(GOLD, name + ".npz"))
    m, ocfg, W = _model(kind, kw["seed"], torch.float32)
    ids, mask, pix, labels = _inputs(ocfg, kw)
    out = m(input_ids=ids.cuda(), pixel_values=pix.cuda(), attention_mask=mask.cuda(), labels=labels.cuda())
    assert tuple(out.logits.shape) == tuple(g["logits_shape"])
    ref_loss = float(g["loss"][0])
    assert abs(out.loss.item() - ref_loss) <= 1e-4, (out.loss.item(), ref_loss)
    rows = torch.as_tensor(g["logits_rows"])
    _, _, aux = O.forward(W, ocfg, ids, pix, mask, labels)  # merged mask (attended rows)
    valid = aux["attention_mask"][:, rows].bool()
    sample = out.logits.detach()[:, rows.cuda()].cpu()
    err = rel_l2(sample[valid], torch.as_tensor(g["logits_sample"])[valid])
    assert err <= 1e-3, err
    out.loss.backward()
    params = {}
    for ar in m.arenas.values():
        params.update(ar.params)
    checked = 0
    for key in g.files:
        if key.startswith("gradnorm/"):
            k = key[len("gradnorm/"):]
            if not params[k].requires_grad:
                continue
            ref = float(g[key][0])
            ours = params[k].grad.double().norm().item()
            assert abs(ours - ref) <= 1e-3 * ref + 1e-7, (k, ours, ref)
            checked += 1
        elif key.startswith("grad/"):
            k = key[len("grad/"):]
            if not params[k].requires_grad:
                continue
            stride = int(g["gradstride/" + k][0])
            ours = params[k].grad.reshape(-1)[::stride].cpu()
            assert rel_l2(ours, g[key]) <= 1e-3, k
    assert checked > 10


@pytest.mark.parametrize("name", ["config1", "small_gpu"])
def test_bf16_mode_matches_bf16_faithful_oracle(name):
    """bf16 production path vs the oracle run with the reference's bf16 rounding points"""
    kind, kw = CASES[name]
    m, ocfg, W = _model(kind, kw["seed"], torch.bfloat16)
    ids, mask, pix, labels = _inputs(ocfg, kw)
    loss_ref, logits_ref, aux = O.forward(O.to_bf16(W), ocfg, ids, pix, mask, labels)
    out = m(input_ids=ids.cuda(), pixel_values=pix.cuda(), attention_mask=mask.cuda(), labels=labels.cuda())
    valid = aux["attention_mask"].bool()
    err = rel_l2(out.logits.detach().float().cpu()[valid], logits_ref.float()[valid])
    assert err <= 1e-2, err
    assert abs(out.loss.item() - loss_ref.item()) <= 1e-2, (out.loss.item(), loss_ref.item())


def test_config1_bf16_pipeline_step():
    """BASELINE config 1 shapes (ViT head dim 16, LM head dim 32) through the product
    pipeline entry point (CuLLaVOPipeline.forward_step, a full train step) on the GPU."""
    from cullavo_amd.trainer import CuLLaVO_Trainer
    opt = {"MODEL": {"NAME": "cullavo_model", "CONFIG": "config1"},
           "DATA": {"BATCH_SIZE_PER_GPU": 2, "TEXT_LEN": 32, "IMAGE_COL": 5, "STEPS": 2}}
    tr = CuLLaVO_Trainer(opt)
    losses = tr.train()
    assert len(losses) == 2 and all(torch.isfinite(torch.as_tensor(float(x))) for x in losses)
