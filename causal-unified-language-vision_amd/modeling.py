"""Module tree of the CuLLaVO hot path with the llava-hf (transformers ~4.37) submodule names,
so state-dict keys and LoRA-style targeting by leaf name keep working
(q_proj/k_proj/v_proj/o_proj/gate_proj/up_proj/down_proj in the LM,
q_proj/k_proj/v_proj/out_proj/fc1/fc2 in the ViT).

Parameters live in flat arenas (arena.py); the modules only hold views. Blocks run through the
fused autograd Functions of functions.py.
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn.functional as F
from torch import nn

from . import ops
from .arena import ParamArena
from .config import CLIPVisionConfig, CuLLaVOConfig, LlamaConfig
from .functions import (ClipLayerFn, EmbeddingFn, LinearFn, LlamaLayerFn, ProjectorFn, StepContext)
from .lora import NO_LORA, LoraGroup, LoraSettings, lm_groups, lora_specs, vision_groups

# dX GEMMs of the decoder layers can read K-major weight copies: "side" refreshes them on a side
# HIP stream during the forward, "sync" on the compute stream at first use, "off" (default) reads
# W [N, K] along N (gemm mode (0,1)). All three give bitwise-equal gradients. Measured on the
# MI355X (config 3): isolated dX GEMMs gain 5-18 %, but in the step the gain (~5 ms) is eaten by
# the per-step re-transposes (~4.5 ms at 5-6 TB/s) in full fine-tune, and the LoRA recipe
# (frozen copies, made once) moved by +0.1 % -- so the 13 GB of copies are not kept by default.
KMAJOR_MODE = os.environ.get("CULLAVO_KMAJOR", "off")
if KMAJOR_MODE not in ("side", "sync", "off"):
    raise ValueError(f"CULLAVO_KMAJOR={KMAJOR_MODE!r}: expected side | sync | off")
_SIDE: dict = {}


def _wait_updates(arena, prefix, lora_groups):
    """The current stream waits for the optimizer's pending side-stream update of this layer's
    parameters (and of the LoRA arena) -- no-op unless FusedAdamW(overlap=True) left one."""
    arena.wait_update(*arena.span(prefix))
    for g in lora_groups.values():
        la = getattr(g, "arena", None)
        if la is not None:
            la.wait_update()
            break


def _side_stream(device):
    key = torch.device(device)
    if key not in _SIDE:
        _SIDE[key] = torch.cuda.Stream(device=key)
    return _SIDE[key]


class _Box(nn.Module):
    """Plain container used for structural levels (self_attn, mlp, embeddings, ...)."""


class Linear(nn.Module):
    def __init__(self, weight: nn.Parameter, bias: nn.Parameter | None = None):
        super().__init__()
        self.weight = weight
        self.bias = bias

    @property
    def in_features(self):
        return self.weight.shape[1]

    @property
    def out_features(self):
        return self.weight.shape[0]

    def attach_lora(self, arena, module_prefix: str, s: LoraSettings):
        """peft-style adapter attributes: lora_A.<adapter>.weight, lora_B.<adapter>.weight,
        scaling[adapter] (views into the LoRA arena; the fused layer Functions run them)."""
        self.lora_A, self.lora_B = _Box(), _Box()
        for box, kind in ((self.lora_A, "lora_A"), (self.lora_B, "lora_B")):
            sub = _Box()
            sub.weight = arena.params[f"{module_prefix}{kind}.{s.adapter}.weight"]
            setattr(box, s.adapter, sub)
        self.scaling = {s.adapter: s.scaling}
        self.r = {s.adapter: s.r}
        self.lora_dropout_p = {s.adapter: s.lora_dropout}

    def forward(self, x):
        if hasattr(self, "lora_A"):
            raise NotImplementedError("LoRA-adapted Linears run inside their layer's fused Function")
        return LinearFn.apply(x, self.weight, self.bias)


def _attach_groups(layer, groups_def, lora, prefix: str, uid0: int):
    """Build the layer's LoraGroups (or NO_LORA stand-ins) and the peft attributes of its Linears."""
    layer.lora_groups = {}
    for gi, (name, mods) in enumerate(groups_def):
        if lora is None:
            layer.lora_groups[name] = NO_LORA
            continue
        arena, s = lora
        layer.lora_groups[name] = LoraGroup(arena, prefix, mods, s, uid0 + gi)
        for suf, _, _ in mods:
            mod = layer
            for part in suf.split("."):
                mod = getattr(mod, part)
            mod.attach_lora(arena, prefix + suf + ".", s)


class _NormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, eps, kind):
        shp = x.shape
        x2 = x.reshape(-1, shp[-1]).contiguous()
        if kind == "rms":
            y, rstd = ops.rmsnorm_fwd(x2, w, eps)
            ctx.saved = (x2, w, b, None, rstd)
        else:
            y, mean, rstd = ops.layernorm_fwd(x2, w, b, eps)
            ctx.saved = (x2, w, b, mean, rstd)
        ctx.kind, ctx.shp = kind, shp
        return y.view(shp)

    @staticmethod
    def backward(ctx, dy):
        from .arena import commit, grad_slot, trainable
        x2, w, b, mean, rstd = ctx.saved
        dy2 = dy.reshape(x2.shape).contiguous()
        if ctx.kind == "rms":
            dw, beta = grad_slot(w) if trainable(w) else (None, 0.0)
            dx = ops.rmsnorm_bwd(dy2, x2, w, rstd, dw=dw, beta=beta)
        else:
            if trainable(w):
                dw, beta = grad_slot(w)
                db, _ = grad_slot(b)
            else:
                dw = db = None
                beta = 0.0
            dx = ops.layernorm_bwd(dy2, x2, w, mean, rstd, dw=dw, db=db, beta=beta)
        commit(w, b)
        return dx.view(ctx.shp), None, None, None, None


class RMSNorm(nn.Module):
    def __init__(self, weight, eps):
        super().__init__()
        self.weight = weight
        self.variance_epsilon = eps

    def forward(self, x):
        return _NormFn.apply(x, self.weight, None, self.variance_epsilon, "rms")


class LayerNorm(nn.Module):
    def __init__(self, weight, bias, eps):
        super().__init__()
        self.weight = weight
        self.bias = bias
        self.eps = eps

    def forward(self, x):
        return _NormFn.apply(x, self.weight, self.bias, self.eps, "ln")


# ---------------------------------------------------------------------------------------------
# arena layouts (the order makes q|k|v and gate|up adjacent)
# ---------------------------------------------------------------------------------------------
def clip_specs(cfg: CLIPVisionConfig, prefix: str):
    dv, f = cfg.hidden_size, cfg.intermediate_size
    s = [(prefix + "embeddings.class_embedding", (dv,)),
         (prefix + "embeddings.patch_embedding.weight", (dv, cfg.num_channels, cfg.patch_size, cfg.patch_size)),
         (prefix + "embeddings.position_embedding.weight", (cfg.num_patches + 1, dv)),
         (prefix + "pre_layrnorm.weight", (dv,)), (prefix + "pre_layrnorm.bias", (dv,))]
    for i in range(cfg.num_hidden_layers):
        lp = f"{prefix}encoder.layers.{i}."
        s += [(lp + f"self_attn.{n}_proj.weight", (dv, dv)) for n in "qkv"]
        s += [(lp + f"self_attn.{n}_proj.bias", (dv,)) for n in "qkv"]
        s += [(lp + "self_attn.out_proj.weight", (dv, dv)), (lp + "self_attn.out_proj.bias", (dv,)),
              (lp + "layer_norm1.weight", (dv,)), (lp + "layer_norm1.bias", (dv,)),
              (lp + "mlp.fc1.weight", (f, dv)), (lp + "mlp.fc1.bias", (f,)),
              (lp + "mlp.fc2.weight", (dv, f)), (lp + "mlp.fc2.bias", (dv,)),
              (lp + "layer_norm2.weight", (dv,)), (lp + "layer_norm2.bias", (dv,))]
    s += [(prefix + "post_layernorm.weight", (dv,)), (prefix + "post_layernorm.bias", (dv,))]
    return s


def llama_layer_specs(cfg: LlamaConfig, prefix: str):
    s = []
    d, f = cfg.hidden_size, cfg.intermediate_size
    for i in range(cfg.num_hidden_layers):
        lp = f"{prefix}layers.{i}."
        s += [(lp + f"self_attn.{n}_proj.weight", (d, d)) for n in "qkv"]
        s += [(lp + "self_attn.o_proj.weight", (d, d)),
              (lp + "mlp.gate_proj.weight", (f, d)), (lp + "mlp.up_proj.weight", (f, d)),
              (lp + "mlp.down_proj.weight", (d, f)),
              (lp + "input_layernorm.weight", (d,)), (lp + "post_attention_layernorm.weight", (d,))]
    s += [(prefix + "norm.weight", (d,))]
    return s


# ---------------------------------------------------------------------------------------------
# CLIP vision tower (tf:models/clip/modeling_clip.py:202-651)
# ---------------------------------------------------------------------------------------------
class CLIPEncoderLayer(nn.Module):
    def __init__(self, cfg: CLIPVisionConfig, P: dict, lp: str, arena: ParamArena, lora=None, uid0: int = 0):
        super().__init__()
        self.cfg = cfg
        self._arena, self._lp = arena, lp
        sa = _Box()
        for n in ("q_proj", "k_proj", "v_proj", "out_proj"):
            setattr(sa, n, Linear(P[lp + f"self_attn.{n}.weight"], P[lp + f"self_attn.{n}.bias"]))
        self.self_attn = sa
        self.layer_norm1 = LayerNorm(P[lp + "layer_norm1.weight"], P[lp + "layer_norm1.bias"], cfg.layer_norm_eps)
        mlp = _Box()
        mlp.fc1 = Linear(P[lp + "mlp.fc1.weight"], P[lp + "mlp.fc1.bias"])
        mlp.fc2 = Linear(P[lp + "mlp.fc2.weight"], P[lp + "mlp.fc2.bias"])
        self.mlp = mlp
        self.layer_norm2 = LayerNorm(P[lp + "layer_norm2.weight"], P[lp + "layer_norm2.bias"], cfg.layer_norm_eps)
        arena.check_adjacent([lp + f"self_attn.{n}_proj.weight" for n in "qkv"])
        arena.check_adjacent([lp + f"self_attn.{n}_proj.bias" for n in "qkv"])
        _attach_groups(self, vision_groups(cfg), lora, lp, uid0)

    def w_qkv(self):
        d = self.cfg.hidden_size
        return self._arena.view(self._lp + "self_attn.q_proj.weight", (3 * d, d))

    def b_qkv(self):
        d = self.cfg.hidden_size
        return self._arena.view(self._lp + "self_attn.q_proj.bias", (3 * d,))

    def qkv_grad_slot(self):
        d = self.cfg.hidden_size
        g, beta = self._arena.grad_slot(self._lp + "self_attn.q_proj.weight", (3 * d, d))
        self._arena.mark_written([self._lp + f"self_attn.{n}_proj.weight" for n in "kv"])
        return g, beta

    def qkv_bias_grad_slot(self):
        d = self.cfg.hidden_size
        g, beta = self._arena.grad_slot(self._lp + "self_attn.q_proj.bias", (3 * d,))
        self._arena.mark_written([self._lp + f"self_attn.{n}_proj.bias" for n in "kv"])
        return g, beta

    def fn_params(self):
        return [p for p in self.parameters() if p.requires_grad]

    def run(self, h2d, B, T, lora_seed: int = 0):
        _wait_updates(self._arena, self._lp, self.lora_groups)
        return ClipLayerFn.apply(h2d, self, B, T, lora_seed, *self.fn_params())

    def forward(self, hidden_states, attention_mask=None, causal_attention_mask=None, **kw):
        if attention_mask is not None or causal_attention_mask is not None:
            raise NotImplementedError("CLIP vision layers run unmasked on the CuLLaVO path")
        B, T, d = hidden_states.shape
        return (self.run(hidden_states.reshape(B * T, d).contiguous(), B, T).view(B, T, d),)


class CLIPVisionOutput:
    def __init__(self, last_hidden_state, pooler_output, hidden_states):
        self.last_hidden_state = last_hidden_state
        self.pooler_output = pooler_output
        self.hidden_states = hidden_states

    def __getitem__(self, i):
        return (self.last_hidden_state, self.pooler_output, self.hidden_states)[i]


class CLIPVisionTransformer(nn.Module):
    def __init__(self, cfg: CLIPVisionConfig, P: dict, prefix: str, arena: ParamArena, lora=None):
        super().__init__()
        self.cfg = cfg
        emb = _Box()
        emb.class_embedding = P[prefix + "embeddings.class_embedding"]
        emb.patch_embedding = _Box()
        emb.patch_embedding.weight = P[prefix + "embeddings.patch_embedding.weight"]
        emb.position_embedding = _Box()
        emb.position_embedding.weight = P[prefix + "embeddings.position_embedding.weight"]
        self.embeddings = emb
        self.pre_layrnorm = LayerNorm(P[prefix + "pre_layrnorm.weight"], P[prefix + "pre_layrnorm.bias"],
                                      cfg.layer_norm_eps)
        enc = _Box()
        def _lora(i):
            return lora if lora is not None and i in lora[1].vision_layers and lora[1].vision else None
        enc.layers = nn.ModuleList([CLIPEncoderLayer(cfg, P, f"{prefix}encoder.layers.{i}.", arena, _lora(i),
                                                     uid0=(1 << 20) + 8 * i)
                                    for i in range(cfg.num_hidden_layers)])
        self.encoder = enc
        self.post_layernorm = LayerNorm(P[prefix + "post_layernorm.weight"], P[prefix + "post_layernorm.bias"],
                                        cfg.layer_norm_eps)
        self.kpad = int(math.ceil(cfg.num_channels * cfg.patch_size ** 2 / 64) * 64)
        self._arena = arena
        self._prefix = prefix
        self._wpad = None  # (arena state it was packed from, [d, kpad] patch weight)

    def _wait(self, *parts):
        """pending optimizer updates (FusedAdamW overlap) of these parameter groups: a trainable
        tower's embeddings / pre- / post-layernorm are read here, not in a layer's run()"""
        for part in parts:
            self._arena.wait_update(*self._arena.span(self._prefix + part))

    def packed_patch_weight(self):
        """Conv2d weight [d, C, p, p] as a K-padded GEMM operand [d, kpad], packed once and
        re-packed only when the vision arena was written since (a trainable tower, a load)."""
        st = self._arena._state()
        if self._wpad is None or self._wpad[0] != st:
            w = self.embeddings.patch_embedding.weight
            wk = w.detach().reshape(w.shape[0], -1)
            self._wpad = (st, F.pad(wk, (0, self.kpad - wk.shape[1])).contiguous())
        return self._wpad[1]

    def embed(self, pixel_values):
        """patch conv (im2col + MFMA GEMM) + CLS + positions + pre_layrnorm -> [B*T, d]."""
        cfg = self.cfg
        B = pixel_values.shape[0]
        if pixel_values.shape[-1] != cfg.image_size or pixel_values.shape[-2] != cfg.image_size:
            raise ValueError(f"Input image size ({pixel_values.shape[-2]}*{pixel_values.shape[-1]}) doesn't "
                             f"match model ({cfg.image_size}*{cfg.image_size}).")
        if pixel_values.dtype not in (torch.float32, torch.bfloat16):
            pixel_values = pixel_values.float()
        self._wait("embeddings.", "pre_layrnorm.")
        patches = ops.im2col_patches(pixel_values, cfg.patch_size, self.kpad, dtype=self._arena.dtype)
        x = ops.linear(patches, self.packed_patch_weight())
        T = cfg.num_patches + 1
        return ops.vision_embed_ln(x, self.embeddings.class_embedding, self.embeddings.position_embedding.weight,
                                   self.pre_layrnorm.weight, self.pre_layrnorm.bias, B=B, T=T,
                                   eps=cfg.layer_norm_eps), B, T

    def hidden_state(self, pixel_values, n_layers: int):
        """hidden_states[n_layers] (0 = pre_layrnorm output) running only the layers needed."""
        h, B, T = self.embed(pixel_values)
        for layer in self.encoder.layers[:n_layers]:
            h = layer.run(h, B, T)
        return h.view(B, T, -1)

    def forward(self, pixel_values, output_hidden_states=None, **kw):
        h, B, T = self.embed(pixel_values)
        hs = [h.view(B, T, -1)]
        for layer in self.encoder.layers:
            h = layer.run(h, B, T)
            hs.append(h.view(B, T, -1))
        last = hs[-1]
        self._wait("post_layernorm.")
        pooled = self.post_layernorm(last[:, 0, :])
        return CLIPVisionOutput(last, pooled, tuple(hs) if output_hidden_states else None)


class CLIPVisionModel(nn.Module):
    def __init__(self, cfg: CLIPVisionConfig, arena: ParamArena, lora=None):
        super().__init__()
        self.config = cfg
        self.vision_model = CLIPVisionTransformer(cfg, arena.params, "vision_tower.vision_model.", arena, lora)

    def forward(self, pixel_values, output_hidden_states=None, **kw):
        return self.vision_model(pixel_values, output_hidden_states=output_hidden_states)


# ---------------------------------------------------------------------------------------------
# projector (tf:models/llava/modeling_llava.py:87-107)
# ---------------------------------------------------------------------------------------------
class LlavaMultiModalProjector(nn.Module):
    def __init__(self, P: dict):
        super().__init__()
        self.linear_1 = Linear(P["multi_modal_projector.linear_1.weight"], P["multi_modal_projector.linear_1.bias"])
        self.linear_2 = Linear(P["multi_modal_projector.linear_2.weight"], P["multi_modal_projector.linear_2.bias"])

    def fn_params(self):
        return [p for p in self.parameters() if p.requires_grad]

    def forward(self, image_features):
        shp = image_features.shape
        x = image_features.reshape(-1, shp[-1])
        if not x.is_contiguous():
            x = x.contiguous()
        for p in self.parameters():
            p._cv_arena.wait_update()  # a pending optimizer update (FusedAdamW overlap)
            break
        y = ProjectorFn.apply(x, self, *self.fn_params())
        return y.view(*shp[:-1], y.shape[-1])


# ---------------------------------------------------------------------------------------------
# Llama causal LM (tf:models/llama/modeling_llama.py:53-480)
# ---------------------------------------------------------------------------------------------
class LlamaDecoderLayer(nn.Module):
    def __init__(self, cfg: LlamaConfig, P: dict, lp: str, arena: ParamArena, lora=None, uid0: int = 0):
        super().__init__()
        self.cfg = cfg
        self._arena, self._lp = arena, lp
        sa = _Box()
        for n in ("q_proj", "k_proj", "v_proj", "o_proj"):
            setattr(sa, n, Linear(P[lp + f"self_attn.{n}.weight"]))
        self.self_attn = sa
        mlp = _Box()
        for n in ("gate_proj", "up_proj", "down_proj"):
            setattr(mlp, n, Linear(P[lp + f"mlp.{n}.weight"]))
        self.mlp = mlp
        self.input_layernorm = RMSNorm(P[lp + "input_layernorm.weight"], cfg.rms_norm_eps)
        self.post_attention_layernorm = RMSNorm(P[lp + "post_attention_layernorm.weight"], cfg.rms_norm_eps)
        arena.check_adjacent([lp + f"self_attn.{n}_proj.weight" for n in "qkv"])
        arena.check_adjacent([lp + "mlp.gate_proj.weight", lp + "mlp.up_proj.weight"])
        _attach_groups(self, lm_groups(cfg), lora if lora is not None and lora[1].lm else None, lp, uid0)

    def w_qkv(self):
        d = self.cfg.hidden_size
        return self._arena.view(self._lp + "self_attn.q_proj.weight", (3 * d, d))

    def w_gu(self):
        return self._arena.view(self._lp + "mlp.gate_proj.weight", (2 * self.cfg.intermediate_size, self.cfg.hidden_size))

    def qkv_grad_slot(self):
        d = self.cfg.hidden_size
        g, beta = self._arena.grad_slot(self._lp + "self_attn.q_proj.weight", (3 * d, d))
        self._arena.mark_written([self._lp + f"self_attn.{n}_proj.weight" for n in "kv"])
        return g, beta

    def _kmajor_specs(self):
        d, F = self.cfg.hidden_size, self.cfg.intermediate_size
        lp = self._lp
        return {"qkv": (lp + "self_attn.q_proj.weight", (3 * d, d)), "o": (lp + "self_attn.o_proj.weight", (d, d)),
                "gu": (lp + "mlp.gate_proj.weight", (2 * F, d)), "down": (lp + "mlp.down_proj.weight", (d, F))}

    def prefetch_kmajor(self):
        """Refresh this layer's K-major weight copies on the side stream while its forward runs
        (KMAJOR_MODE "side"), so the backward's dX GEMMs read reduction-contiguous weights."""
        if KMAJOR_MODE == "off":
            return
        st = _side_stream(self._arena.device) if KMAJOR_MODE == "side" else None
        for key, shape in self._kmajor_specs().values():
            self._arena.prefetch_transposed(key, shape, st)

    def linear_dx(self, dy, which: str, swiglu_gu=None):
        """dx = dy @ W for which in qkv | o | gu | down (fused weights), via the K-major copy;
        swiglu_gu: return swiglu_bwd(dx, gu) from the GEMM epilogue instead (ops.linear_dx)."""
        key, shape = self._kmajor_specs()[which]
        if KMAJOR_MODE == "off":
            return ops.linear_dx(dy, self._arena.view(key, shape), swiglu_gu=swiglu_gu)
        return ops.linear_dx_t(dy, self._arena.transposed(key, shape), swiglu_gu=swiglu_gu)

    def gu_grad_slot(self):
        g, beta = self._arena.grad_slot(self._lp + "mlp.gate_proj.weight",
                                        (2 * self.cfg.intermediate_size, self.cfg.hidden_size))
        self._arena.mark_written([self._lp + "mlp.up_proj.weight"])
        return g, beta

    def fn_params(self):
        return [p for p in self.parameters() if p.requires_grad]

    def run(self, h2d, sctx: StepContext):
        _wait_updates(self._arena, self._lp, self.lora_groups)
        if torch.is_grad_enabled() and h2d.requires_grad:
            self.prefetch_kmajor()
        return LlamaLayerFn.apply(h2d, self, sctx, *self.fn_params())


class LlamaModel(nn.Module):
    def __init__(self, cfg: LlamaConfig, embed_arena: ParamArena, layer_arena: ParamArena, lora=None):
        super().__init__()
        self.config = cfg
        self.embed_tokens = _Embedding(embed_arena.params["language_model.model.embed_tokens.weight"])
        P = layer_arena.params
        self.layers = nn.ModuleList([LlamaDecoderLayer(cfg, P, f"language_model.model.layers.{i}.", layer_arena,
                                                       lora, uid0=8 * i)
                                     for i in range(cfg.num_hidden_layers)])
        self.norm = RMSNorm(P["language_model.model.norm.weight"], cfg.rms_norm_eps)


class _Embedding(nn.Module):
    def __init__(self, weight):
        super().__init__()
        self.weight = weight

    @property
    def num_embeddings(self):
        return self.weight.shape[0]

    @property
    def embedding_dim(self):
        return self.weight.shape[1]

    def forward(self, ids):
        self.weight._cv_arena.wait_update()  # a pending optimizer update (FusedAdamW overlap)
        return EmbeddingFn.apply(ids.contiguous(), self.weight)


class CausalLMOutput:
    def __init__(self, logits, hidden_states=None, past_key_values=None, attentions=None):
        self.logits = logits
        self.hidden_states = hidden_states
        self.past_key_values = past_key_values
        self.attentions = attentions

    def __getitem__(self, i):
        return (self.logits, self.past_key_values, self.hidden_states, self.attentions)[i]

    def to_tuple(self):
        return tuple(x for x in (self.logits, self.past_key_values, self.hidden_states, self.attentions)
                     if x is not None)


class LlamaForCausalLM(nn.Module):
    def __init__(self, cfg: LlamaConfig, embed_arena, layer_arena, head_arena, lora=None):
        super().__init__()
        self.cfg = self.config = cfg
        self.model = LlamaModel(cfg, embed_arena, layer_arena, lora)
        self.lm_head = Linear(head_arena.params["language_model.lm_head.weight"])

    def head_params(self):
        return [p for p in (self.model.norm.weight, self.lm_head.weight) if p.requires_grad]

    def decode(self, h2d, sctx: StepContext, collect: bool = False):
        hs = [h2d] if collect else None
        for layer in self.model.layers:
            h2d = layer.run(h2d, sctx)
            if collect:
                hs.append(h2d)
        return h2d, hs

    def forward(self, input_ids=None, attention_mask=None, position_ids=None, past_key_values=None,
                inputs_embeds=None, use_cache=None, output_attentions=None, output_hidden_states=None,
                return_dict=None, **kw):
        if inputs_embeds is None:
            inputs_embeds = self.model.embed_tokens(input_ids)
        if past_key_values is not None or use_cache:
            from .generation import lm_infer
            with torch.no_grad():
                logits, cache = lm_infer(self, inputs_embeds, attention_mask, position_ids, past_key_values,
                                         inputs_embeds.shape[1] + 256)
            return CausalLMOutput(logits, past_key_values=cache)
        B, L, d = inputs_embeds.shape
        if position_ids is None:
            position_ids = torch.arange(L, device=inputs_embeds.device).expand(B, L)
        kv_start = None
        if attention_mask is not None:
            kv_start = (attention_mask.cumsum(-1) == 0).sum(-1).to(torch.int32)
        sctx = StepContext(B, L, position_ids, kv_start)
        h, hs = self.decode(inputs_embeds.reshape(B * L, d).contiguous(), sctx, bool(output_hidden_states))
        x = self.model.norm(h)
        logits = self.lm_head(x).view(B, L, -1)
        hs_t = tuple(t.view(B, L, d) for t in hs) if hs else None
        return CausalLMOutput(logits, hidden_states=hs_t)


# ---------------------------------------------------------------------------------------------
# construction helpers
# ---------------------------------------------------------------------------------------------
TRAINABLE_POLICIES = {
    # LLaVA-1.5 fine-tune recipe: vision frozen, projector + whole LM trained (full-FT headline)
    "full": {"vision": False, "projector": True, "embed": True, "layers": True, "head": True},
    # the reference's non-LoRA trainable set (cullavo/load_cullavo.py:128-138): projector,
    # lm_head and embed_tokens; base weights frozen (LoRA adapters: SURVEY.md §8(f) row 1)
    "reference": {"vision": False, "projector": True, "embed": True, "layers": False, "head": True},
    # what the reference actually trains: the "reference" set plus LoRA adapters on the LM and on
    # ViT layers 12-22 (cullavo/load_cullavo.py:94-138)
    "lora": {"vision": False, "projector": True, "embed": True, "layers": False, "head": True, "lora": True},
    "none": {"vision": False, "projector": False, "embed": False, "layers": False, "head": False},
}


def build_arenas(cfg: CuLLaVOConfig, device, trainable: str = "full", dtype=torch.bfloat16,
                 lora: LoraSettings | None = None):
    pol = TRAINABLE_POLICIES[trainable]
    v, t = cfg.vision_config, cfg.text_config
    d = t.hidden_size
    ar = {
        "vision": ParamArena("vision", clip_specs(v, "vision_tower.vision_model."), device=device, dtype=dtype,
                             trainable=pol["vision"]),
        "projector": ParamArena("projector", [("multi_modal_projector.linear_1.weight", (d, v.hidden_size)),
                                              ("multi_modal_projector.linear_1.bias", (d,)),
                                              ("multi_modal_projector.linear_2.weight", (d, d)),
                                              ("multi_modal_projector.linear_2.bias", (d,))],
                                device=device, dtype=dtype, trainable=pol["projector"]),
        "embed": ParamArena("embed", [("language_model.model.embed_tokens.weight", (t.vocab_size, d))],
                            device=device, dtype=dtype, trainable=pol["embed"]),
        "layers": ParamArena("layers", llama_layer_specs(t, "language_model.model."), device=device, dtype=dtype,
                             trainable=pol["layers"]),
        "head": ParamArena("head", [("language_model.lm_head.weight", (t.vocab_size, d))], device=device,
                           dtype=dtype, trainable=pol["head"]),
    }
    if pol.get("lora"):
        ar["lora"] = ParamArena("lora", lora_specs(cfg, lora or LoraSettings()), device=device, dtype=dtype,
                                trainable=True)
    return ar


def init_random_(arenas: dict, seed: int = 0):
    """Random init directly in HBM (no checkpoints offline): N(0, 1/fan_in) linears, 1 norms,
    0.02 biases/embeddings. Used for the synthetic-data benchmark."""
    g = torch.Generator(device=next(iter(arenas.values())).device)
    g.manual_seed(seed)
    for name, ar in arenas.items():
        if name == "lora":
            from .lora import init_lora_
            init_lora_(ar, seed + 1)
            continue
        for key, (o, n, shape) in ar.offsets.items():
            v = ar.flat[o:o + n]
            if key.endswith("norm.weight") or "layer_norm" in key and key.endswith("weight") or \
                    key.endswith("layrnorm.weight") or key.endswith("layernorm.weight"):
                v.fill_(1.0)
            elif key.endswith("bias") or "embedding" in key:
                v.normal_(0.0, 0.02, generator=g)
            elif key.endswith("embed_tokens.weight"):
                v.normal_(0.0, 0.5, generator=g)
            else:
                fan_in = int(math.prod(shape[1:]))
                v.normal_(0.0, fan_in ** -0.5, generator=g)
