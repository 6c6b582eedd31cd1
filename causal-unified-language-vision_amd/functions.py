"""Autograd Functions of the hot path. Each one runs a whole block of the reference's module
chain on the C-ABI kernels and has a hand-written backward that writes parameter gradients
straight into the arena (arena.grad_slot) and returns only activation gradients.

  LinearFn          nn.Linear (any Linear called on its own)
  LlamaLayerFn      LlamaDecoderLayer   tf:models/llama/modeling_llama.py:284-345
  ClipLayerFn       CLIPEncoderLayer    tf:models/clip/modeling_clip.py:353-384
  ProjectorFn       LlavaMultiModalProjector tf:models/llava/modeling_llava.py:87-107
  EmbeddingFn       embed_tokens        reference cullavo/arch_cullavo.py:582
  MergeFn           _merge_input_ids_with_image_features rows   arch_cullavo.py:600-602
  HeadLossFn        final RMSNorm + lm_head + shifted masked CE   arch_cullavo.py:651-665

Parameters are passed to .apply only so autograd sees a dependency; their returned gradient
is None (the value is already in the arena).
"""
from __future__ import annotations

import os

import torch

from . import ops
from .arena import commit, grad_slot, trainable
from .lora import NO_LORA
from .ops import ACT_GELU, ACT_QUICK_GELU


def _needs_grad(ctx) -> bool:
    # grad mode is off inside Function.forward; needs_input_grad says whether backward will run
    return any(ctx.needs_input_grad)


def _lin_act(x, w, b, act, keep_preact):
    if keep_preact:
        return ops.linear(x, w, b, act=act, want_preact=True)
    return ops.linear(x, w, b, act=act), None


# Weight-gradient GEMMs (dW = dY^T X) feed only the DP exchange and the optimizer, so "side"
# issues them on a side HIP stream beside the dX chain: their CUs fill the tails of the dX
# GEMMs and run under the memory-bound norm / SwiGLU / attention backward kernels. The main
# stream joins the side stream when the backward pass ends (autograd final callback), the DP
# reducer's stream before each bucket. "off" (default) keeps every launch on the compute stream.
# Both give bitwise-equal gradients (same kernels, same inputs). Measured on the MI355X (config
# 3, full FT): side 399.6 ms/step vs off 389.3 -- two GEMMs sharing the CUs (one 8-wave block
# per CU each) slow each other more than the filled tails gain; with the compute stream at high
# priority 386.2 vs 388.4 (noise level), so the single stream stays the default.
DW_STREAM = os.environ.get("CULLAVO_DW_STREAM", "off")
# the down-projection weight gradient on the side stream, launched before the SwiGLU-fused dX GEMM so
# the two share the CUs (CULLAVO_SWG_OVERLAP=1, A/B): the dX GEMM's epilogue bursts (gate|up read,
# d(gate|up) write) then meet the dW GEMM's long K-loops instead of each other
SWG_OVERLAP = os.environ.get("CULLAVO_SWG_OVERLAP", "0") == "1"
# SwiGLU backward in the down-projection dX GEMM's epilogue (CULLAVO_FUSED_SWIGLU_BWD=0: the
# separate swiglu_bwd kernel, for A/B)
FUSED_SWIGLU_BWD = os.environ.get("CULLAVO_FUSED_SWIGLU_BWD", "1") != "0"
if DW_STREAM not in ("side", "off"):
    raise ValueError(f"CULLAVO_DW_STREAM={DW_STREAM!r}: expected side | off")
_DW: dict = {}  # device -> {"stream": side stream, "main": stream to join, "queued": bool}

# bench.py's layer roofline (the north star's "attention + MLP step"): HIP events on the compute
# stream around every decoder layer's forward and backward; None = off
_LAYER_EV: dict | None = None


def trace_layers(on: bool) -> None:
    """start (on) or stop recording LlamaLayerFn forward / backward spans"""
    global _LAYER_EV
    _LAYER_EV = {"fwd": [], "bwd": []} if on else None


def layer_spans() -> dict:
    """{"fwd": [ms, ...], "bwd": [ms, ...]} of the recorded layer spans (synchronises; stops tracing)"""
    global _LAYER_EV
    ev, _LAYER_EV = _LAYER_EV, None
    out = {"fwd": [], "bwd": []}
    if not ev:
        return out
    for k in out:
        if ev[k]:
            ev[k][-1][1].synchronize()
        out[k] = [a.elapsed_time(b) for a, b in ev[k]]
    return out


def _span_begin():
    if _LAYER_EV is None:
        return None
    e = torch.cuda.Event(enable_timing=True)
    e.record(torch.cuda.current_stream())
    return e


def _span_end(e0, kind: str) -> None:
    if e0 is None or _LAYER_EV is None:
        return
    e1 = torch.cuda.Event(enable_timing=True)
    e1.record(torch.cuda.current_stream())
    _LAYER_EV[kind].append((e0, e1))


def _dw_state(dev):
    st = _DW.get(dev)
    if st is None:
        st = _DW[dev] = {"stream": torch.cuda.Stream(device=dev), "main": None, "queued": False}
    return st


def dw_join(dev=None):
    """Make the current stream wait for every weight-gradient launch issued so far."""
    for d, st in _DW.items():
        if dev is None or torch.device(dev) == d:
            torch.cuda.current_stream(d).wait_stream(st["stream"])


def dw_wait(stream):
    """Make `stream` (e.g. the DP reducer's) wait for the weight-gradient launches issued so far."""
    for d, st in _DW.items():
        if d == stream.device:
            stream.wait_stream(st["stream"])


def _join_at_end(st):
    if st["queued"]:  # one join per backward pass, however many callbacks it queued
        st["main"].wait_stream(st["stream"])
        st["queued"] = False


def _dw(dy, x, g, beta, *params, side=False):
    """dW GEMM into the arena slot g, then commit(params) (which may launch DP buckets); side: on the
    side stream whatever DW_STREAM says."""
    if (DW_STREAM == "off" and not side) or not dy.is_cuda:
        ops.linear_dw(dy, x, g, beta=beta)
        commit(*params)
        return
    st = _dw_state(dy.device)
    side, cur = st["stream"], torch.cuda.current_stream(dy.device)
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        ops.linear_dw(dy, x, g, beta=beta)
        commit(*params)
    # the caching allocator must not hand these to the compute stream before the side GEMM read them
    dy.record_stream(side)
    x.record_stream(side)
    st["main"], st["queued"] = cur, True
    torch.autograd.Variable._execution_engine.queue_callback(lambda: _join_at_end(st))


def _write_dw(dy, x, w, side=False):
    if trainable(w):
        g, beta = grad_slot(w)
        _dw(dy, x, g, beta, w, side=side)


def _write_bias(dy, b):
    if trainable(b):
        g, beta = grad_slot(b)
        ops.colsum(dy, g, beta=beta)
        commit(b)


# ---------------------------------------------------------------------------------------------
class LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        shp = x.shape
        x2 = x.reshape(-1, shp[-1])
        y = ops.linear(x2, w, b)
        ctx.save_for_backward(x2, w, b)
        ctx.shp = shp
        return y.view(*shp[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w, b = ctx.saved_tensors
        dy2 = dy.reshape(-1, w.shape[0]).contiguous()
        _write_dw(dy2, x2, w)
        _write_bias(dy2, b)
        dx = ops.linear_dx(dy2, w).view(ctx.shp) if ctx.needs_input_grad[0] else None
        return dx, None, None


# ---------------------------------------------------------------------------------------------
class StepContext:
    """Per-forward shape/index state shared by the decoder layers (built once per step).
    lora_seed: this forward's LoRA-dropout seed (drawn from torch's CPU generator, so
    torch.manual_seed makes runs repeatable; backward reuses it to regenerate the masks)."""

    def __init__(self, B: int, L: int, position_ids, kv_start=None, lora_seed: int | None = None):
        self.B, self.L = B, L
        self.position_ids = position_ids.reshape(-1).contiguous()
        self.kv_start = kv_start
        self.lora_seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if lora_seed is None else lora_seed


class LlamaLayerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, layer, sctx: StepContext, *params):
        cfg = layer.cfg
        T, d = h.shape
        H, D = cfg.num_attention_heads, cfg.head_dim
        Fd = cfg.intermediate_size
        grad = _needs_grad(ctx)
        lg, tr, seed = layer.lora_groups, layer.training, sctx.lora_seed
        span = _span_begin()
        x1, rstd1 = ops.rmsnorm_fwd(h, layer.input_layernorm.weight, cfg.rms_norm_eps)
        t, u_qkv = lg["qkv"].forward(x1, tr, seed)
        qkv = ops.linear(x1, layer.w_qkv(), addend=t)  # [T, 3d]: q | k | v
        q, k, v = qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:]
        ops.rope(q, k, sctx.position_ids, hq=H, hk=H, head_dim=D, theta=cfg.rope_theta)
        o, lse = ops.attn_fwd(q, k, v, B=sctx.B, H=H, Lq=sctx.L, Lk=sctx.L, D=D, scale=D ** -0.5, causal=True,
                              kv_start=sctx.kv_start)
        t, u_o = lg["o"].forward(o, tr, seed)
        h2 = ops.linear(o, layer.self_attn.o_proj.weight, residual=h, addend=t)
        x2, rstd2 = ops.rmsnorm_fwd(h2, layer.post_attention_layernorm.weight, cfg.rms_norm_eps)
        t, u_gu = lg["gu"].forward(x2, tr, seed)
        gu = ops.linear(x2, layer.w_gu(), addend=t)  # [T, 2F]: gate | up
        a = ops.swiglu_fwd(gu)
        t, u_d = lg["down"].forward(a, tr, seed)
        h3 = ops.linear(a, layer.mlp.down_proj.weight, residual=h2, addend=t)
        del t
        _span_end(span, "fwd")
        if grad:
            ctx.layer, ctx.sctx, ctx.train = layer, sctx, tr
            ctx.saved = (h, x1, rstd1, qkv, o, lse, h2, x2, rstd2, gu, a, u_qkv, u_o, u_gu, u_d)
        return h3

    @staticmethod
    def backward(ctx, dh3):
        layer, sctx = ctx.layer, ctx.sctx
        cfg = layer.cfg
        h, x1, rstd1, qkv, o, lse, h2, x2, rstd2, gu, a, u_qkv, u_o, u_gu, u_d = ctx.saved
        ctx.saved = None
        lg, tr, seed = layer.lora_groups, ctx.train, sctx.lora_seed
        T, d = h.shape
        H, D = cfg.num_attention_heads, cfg.head_dim
        span = _span_begin()
        dh3 = dh3.contiguous()
        # MLP. Without a LoRA adapter on down_proj the SwiGLU backward runs in the epilogue of
        # the down-projection dX GEMM (dh never stored); with one, dh collects the adapter's
        # share first (bitwise the same arithmetic either way, tests/test_ops_gpu.py).
        fused_swg = lg["down"] is NO_LORA and FUSED_SWIGLU_BWD and gu.dtype == torch.bfloat16
        overlap = fused_swg and SWG_OVERLAP and dh3.is_cuda
        if overlap:
            _write_dw(dh3, a, layer.mlp.down_proj.weight, side=True)
        if fused_swg:
            dgu = layer.linear_dx(dh3, "down", swiglu_gu=gu)
        else:
            da = layer.linear_dx(dh3, "down")
            lg["down"].backward(dh3, a, u_d, da, tr, seed)
            dgu = ops.swiglu_bwd(da, gu)
            del da
        if not overlap:
            _write_dw(dh3, a, layer.mlp.down_proj.weight)
        dx2 = layer.linear_dx(dgu, "gu")
        lg["gu"].backward(dgu, x2, u_gu, dx2, tr, seed)
        if trainable(layer.mlp.gate_proj.weight):
            g, beta = layer.gu_grad_slot()
            _dw(dgu, x2, g, beta, layer.mlp.gate_proj.weight, layer.mlp.up_proj.weight)
        del dgu
        wpost = layer.post_attention_layernorm.weight
        dw_post, beta_post = grad_slot(wpost) if trainable(wpost) else (None, 0.0)
        dh2 = ops.rmsnorm_bwd(dx2, h2, wpost, rstd2, dres=dh3, dw=dw_post, beta=beta_post)
        commit(wpost)
        del dx2
        # attention
        do = layer.linear_dx(dh2, "o")
        lg["o"].backward(dh2, o, u_o, do, tr, seed)
        _write_dw(dh2, o, layer.self_attn.o_proj.weight)
        dqkv = torch.empty_like(qkv)
        q, k, v = qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:]
        ops.attn_bwd(q, k, v, o, do, lse, B=sctx.B, H=H, Lq=sctx.L, Lk=sctx.L, D=D, scale=D ** -0.5, causal=True,
                     kv_start=sctx.kv_start, dq=dqkv[:, :d], dk=dqkv[:, d:2 * d], dv=dqkv[:, 2 * d:])
        del do
        ops.rope(dqkv[:, :d], dqkv[:, d:2 * d], sctx.position_ids, hq=H, hk=H, head_dim=D, theta=cfg.rope_theta,
                 inverse=True)
        dx1 = layer.linear_dx(dqkv, "qkv")
        lg["qkv"].backward(dqkv, x1, u_qkv, dx1, tr, seed)
        if trainable(layer.self_attn.q_proj.weight):
            g, beta = layer.qkv_grad_slot()
            sa = layer.self_attn
            _dw(dqkv, x1, g, beta, sa.q_proj.weight, sa.k_proj.weight, sa.v_proj.weight)
        del dqkv
        win = layer.input_layernorm.weight
        dw_in, beta_in = grad_slot(win) if trainable(win) else (None, 0.0)
        dh = ops.rmsnorm_bwd(dx1, h, win, rstd1, dres=dh2, dw=dw_in, beta=beta_in)
        commit(win)
        _span_end(span, "bwd")
        return (dh, None, None) + (None,) * len(layer.fn_params())


# ---------------------------------------------------------------------------------------------
class ClipLayerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, layer, B: int, T: int, lora_seed: int, *params):
        cfg = layer.cfg
        d = cfg.hidden_size
        H, D = cfg.num_attention_heads, cfg.head_dim
        grad = _needs_grad(ctx)
        lg, tr = layer.lora_groups, layer.training
        sa, mlp = layer.self_attn, layer.mlp
        x1, m1, r1 = ops.layernorm_fwd(h, layer.layer_norm1.weight, layer.layer_norm1.bias, cfg.layer_norm_eps)
        t, u_qkv = lg["qkv"].forward(x1, tr, lora_seed)
        qkv = ops.linear(x1, layer.w_qkv(), layer.b_qkv(), addend=t)
        q, k, v = qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:]
        o, lse = ops.attn_fwd(q, k, v, B=B, H=H, Lq=T, Lk=T, D=D, scale=D ** -0.5, causal=False)
        h2 = ops.linear(o, sa.out_proj.weight, sa.out_proj.bias, residual=h)
        x2, m2, r2 = ops.layernorm_fwd(h2, layer.layer_norm2.weight, layer.layer_norm2.bias, cfg.layer_norm_eps)
        t, u_1 = lg["fc1"].forward(x2, tr, lora_seed)
        if grad:
            a, pre = ops.linear(x2, mlp.fc1.weight, mlp.fc1.bias, act=ACT_QUICK_GELU, want_preact=True, addend=t)
        else:
            a, pre = ops.linear(x2, mlp.fc1.weight, mlp.fc1.bias, act=ACT_QUICK_GELU, addend=t), None
        t, u_2 = lg["fc2"].forward(a, tr, lora_seed)
        h3 = ops.linear(a, mlp.fc2.weight, mlp.fc2.bias, residual=h2, addend=t)
        del t
        if grad:
            ctx.layer, ctx.B, ctx.T, ctx.train, ctx.seed = layer, B, T, tr, lora_seed
            ctx.saved = (h, x1, m1, r1, qkv, o, lse, h2, x2, m2, r2, a, pre, u_qkv, u_1, u_2)
        return h3

    @staticmethod
    def backward(ctx, dh3):
        layer, B, T = ctx.layer, ctx.B, ctx.T
        cfg = layer.cfg
        d = cfg.hidden_size
        H, D = cfg.num_attention_heads, cfg.head_dim
        h, x1, m1, r1, qkv, o, lse, h2, x2, m2, r2, a, pre, u_qkv, u_1, u_2 = ctx.saved
        ctx.saved = None
        lg, tr, seed = layer.lora_groups, ctx.train, ctx.seed
        sa, mlp = layer.self_attn, layer.mlp
        dh3 = dh3.contiguous()
        da = ops.linear_dx(dh3, mlp.fc2.weight)
        lg["fc2"].backward(dh3, a, u_2, da, tr, seed)
        _write_dw(dh3, a, mlp.fc2.weight)
        _write_bias(dh3, mlp.fc2.bias)
        dpre = ops.act_bwd(ACT_QUICK_GELU, da, pre)
        dx2 = ops.linear_dx(dpre, mlp.fc1.weight)
        lg["fc1"].backward(dpre, x2, u_1, dx2, tr, seed)
        _write_dw(dpre, x2, mlp.fc1.weight)
        _write_bias(dpre, mlp.fc1.bias)
        ln2 = layer.layer_norm2
        dw2, db2, beta2 = _ln_slots(ln2)
        dh2 = ops.layernorm_bwd(dx2, h2, ln2.weight, m2, r2, dres=dh3, dw=dw2, db=db2, beta=beta2)
        commit(ln2.weight, ln2.bias)
        do = ops.linear_dx(dh2, sa.out_proj.weight)
        _write_dw(dh2, o, sa.out_proj.weight)
        _write_bias(dh2, sa.out_proj.bias)
        dqkv = torch.empty_like(qkv)
        ops.attn_bwd(qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:], o, do, lse, B=B, H=H, Lq=T, Lk=T, D=D,
                     scale=D ** -0.5, causal=False, dq=dqkv[:, :d], dk=dqkv[:, d:2 * d], dv=dqkv[:, 2 * d:])
        dx1 = ops.linear_dx(dqkv, layer.w_qkv()) if ctx.needs_input_grad[0] else None
        lg["qkv"].backward(dqkv, x1, u_qkv, dx1, tr, seed)
        if trainable(sa.q_proj.weight):
            g, beta = layer.qkv_grad_slot()
            _dw(dqkv, x1, g, beta, sa.q_proj.weight, sa.k_proj.weight, sa.v_proj.weight)
            gb, betab = layer.qkv_bias_grad_slot()
            ops.colsum(dqkv, gb, beta=betab)
            commit(sa.q_proj.bias, sa.k_proj.bias, sa.v_proj.bias)
        ln1 = layer.layer_norm1
        dh = None
        if ctx.needs_input_grad[0] or trainable(ln1.weight):
            dw1, db1, beta1 = _ln_slots(ln1)
            if dx1 is None:
                dx1 = ops.linear_dx(dqkv, layer.w_qkv())
            dh = ops.layernorm_bwd(dx1, h, ln1.weight, m1, r1, dres=dh2, dw=dw1, db=db1, beta=beta1)
            commit(ln1.weight, ln1.bias)
        return (dh, None, None, None, None) + (None,) * len(layer.fn_params())


def _ln_slots(ln):
    if not trainable(ln.weight):
        return None, None, 0.0
    gw, beta = grad_slot(ln.weight)
    gb, _ = grad_slot(ln.bias)
    return gw, gb, beta


# ---------------------------------------------------------------------------------------------
class ProjectorFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, proj, *params):
        l1, l2 = proj.linear_1, proj.linear_2
        grad = _needs_grad(ctx)
        a, pre = _lin_act(x, l1.weight, l1.bias, ACT_GELU, grad)
        y = ops.linear(a, l2.weight, l2.bias)
        if grad:
            ctx.proj = proj
            ctx.saved = (x, a, pre)
            ctx.x_grad = x.requires_grad
        return y

    @staticmethod
    def backward(ctx, dy):
        proj = ctx.proj
        x, a, pre = ctx.saved
        ctx.saved = None
        l1, l2 = proj.linear_1, proj.linear_2
        dy = dy.contiguous()
        da = ops.linear_dx(dy, l2.weight)
        _write_dw(dy, a, l2.weight)
        _write_bias(dy, l2.bias)
        dpre = ops.act_bwd(ACT_GELU, da, pre)
        _write_dw(dpre, x, l1.weight)
        _write_bias(dpre, l1.bias)
        dx = ops.linear_dx(dpre, l1.weight) if ctx.x_grad else None
        return (dx, None) + (None,) * len(proj.fn_params())


# ---------------------------------------------------------------------------------------------
class EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, weight):
        out = ops.embedding_fwd(ids, weight)
        ctx.ids, ctx.weight = ids, weight
        return out.view(*ids.shape, weight.shape[1])

    @staticmethod
    def backward(ctx, dout):
        w = ctx.weight
        if trainable(w):
            g, beta = grad_slot(w)
            if beta == 0.0:
                g.zero_()
            ops.embedding_bwd(ctx.ids, dout.reshape(-1, w.shape[1]).contiguous(), g, beta=1.0)
            commit(w)
        return None, None


class MergeFn(torch.autograd.Function):
    """out rows = text rows (text_dst) | image rows | zeros, from the merge plan."""

    @staticmethod
    def forward(ctx, text, image, src, text_dst, img_dst):
        out = ops.row_gather2(src.reshape(-1), text, image)
        ctx.idx = (text_dst, img_dst)
        ctx.shapes = (text.shape, image.shape)
        return out

    @staticmethod
    def backward(ctx, dout):
        text_dst, img_dst = ctx.idx
        ts, ims = ctx.shapes
        dout = dout.contiguous()
        dtext = ops.row_gather2(text_dst.reshape(-1), dout, None).view(ts) if ctx.needs_input_grad[0] else None
        dimg = ops.row_gather2(img_dst, dout, None).view(ims) if ctx.needs_input_grad[1] else None
        return dtext, dimg, None, None, None


# ---------------------------------------------------------------------------------------------
class HeadLossFn(torch.autograd.Function):
    """final RMSNorm -> lm_head -> per-row CE over shifted, masked targets -> mean."""

    @staticmethod
    def forward(ctx, h, lm, targets, ignore_index: int, *params):
        norm_w, W = lm.model.norm.weight, lm.lm_head.weight
        eps = lm.cfg.rms_norm_eps
        x, rstd = ops.rmsnorm_fwd(h, norm_w, eps)
        logits = ops.linear(x, W)
        row_loss, lse = ops.ce_fwd(logits, targets, ignore_index)
        out = ops.ce_reduce(row_loss, targets, ignore_index)
        ctx.lm = lm
        ctx.ignore = ignore_index
        # logits are an output for callers that use them; when nothing downstream does (the
        # training step), autograd passes None instead of a materialised zero [T, V] gradient
        ctx.set_materialize_grads(False)
        ctx.saved = (h, x, rstd, logits, targets, lse, out)
        ctx.stats = out  # [loss, count, 1/count] on device (no host sync)
        return out[0].clone(), logits

    @staticmethod
    def backward(ctx, dloss, dlogits):
        lm = ctx.lm
        h, x, rstd, logits, targets, lse, out = ctx.saved
        ctx.saved = None
        norm_w, W = lm.model.norm.weight, lm.lm_head.weight
        gl = dloss.reshape(1).float().contiguous() if dloss is not None else torch.zeros(1, device=h.device)
        dl = ops.ce_bwd(logits, targets, lse, out, gl, ctx.ignore)
        if dlogits is not None:
            dl += dlogits
        dx = ops.linear_dx(dl, W)
        _write_dw(dl, x, W)
        del dl
        dw, beta = grad_slot(norm_w) if trainable(norm_w) else (None, 0.0)
        dh = ops.rmsnorm_bwd(dx, h, norm_w, rstd, dw=dw, beta=beta) if ctx.needs_input_grad[0] else None
        commit(norm_w)
        return (dh, None, None, None) + (None,) * len(lm.head_params())
