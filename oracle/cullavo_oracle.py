"""CPU oracle for the CuLLaVO forward/backward hot path — TEST INFRASTRUCTURE ONLY.

This module is the checker the parity tests, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg compare against; the product path (``cullavo_amd``) never imports it.

It is a plain PyTorch restatement (torch autograd supplies the backward) of what the
reference executes for one training step. With fp32 weights it is the reference's fp32 path
(pinned below); with bf16 weights (``to_bf16``) it is the bf16-faithful mode: every module
output, residual add and norm output rounds to bf16 where the reference's bf16-cast model
under bf16 autocast rounds (reference cullavo/load_cullavo.py:123-126,
configs/accel/ddp_accel.yaml:8), RMSNorm keeps f32 statistics and casts before the weight
(tf:llama :63-67), RoPE casts its f32 cos/sin to bf16 (:121-125), attention keeps FA2's f32
scores/softmax with bf16 P, and the loss upcasts the bf16 logits to f32 (4.37). Every bf16
product (Linear, patch conv, attention PV) accumulates in f32 and rounds its output once, the
arithmetic of the reference's bf16 GEMMs on a GPU (hipBLASLt/cuBLAS bf16 with f32 accumulate and
the bias in the epilogue); torch's CPU bf16 matmul blocks the reduction differently, which alone
moves the small_gpu logits by rel-L2 8.3e-3 (tools/bf16_noise_floor.py):

* ``forward``          — reference cullavo/arch_cullavo.py:546-677 (CuLLaVOModel.forward):
                          embed :582, vision tower :586, feature select :588-597,
                          projector :599, merge :600-602, default labels :603-604,
                          language model :638-647, shifted masked CE :651-665.
* ``vision_hidden_states`` — HF CLIPVisionTransformer (tf:models/clip/modeling_clip.py:202-218
                          embeddings, :280-336 attention, :338-351 MLP, :353-384 layer,
                          :600-651 tower; hidden_states[0] = pre_layrnorm output).
* ``projector``        — tf:models/llava/modeling_llava.py:87-107.
* ``merge``            — transformers ~4.37 LlavaForConditionalGeneration.
                          _merge_input_ids_with_image_features (absent from the installed
                          5.15; restated from its published algorithm, the index form that
                          marks non-text slots as image slots).
* ``llama_hidden``     — tf:models/llama/modeling_llama.py:53-70 RMSNorm, :73-160 RoPE,
                          :163-176 MLP, :191-214 eager attention (fp32 softmax), :284-345
                          decoder layer, :347-419 model, :480 lm_head.

Pinning: tests/golden/make_golden.py runs the REFERENCE's own CuLLaVOModel.forward (imported
from /root/reference through a small compat shim over transformers 5.15) on seeded weights
and inputs and commits the outputs under tests/golden/; tests/test_oracle_golden.py checks
this restatement against them.
"""
from __future__ import annotations

import math
import zlib
from dataclasses import dataclass, field

import numpy as np
import torch
import torch.nn.functional as F

IGNORE_INDEX = -100


# ---------------------------------------------------------------------------------------------
# configuration
# ---------------------------------------------------------------------------------------------
@dataclass
class VisionCfg:
    image_size: int = 336
    patch_size: int = 14
    hidden_size: int = 1024
    num_hidden_layers: int = 24
    num_attention_heads: int = 16
    intermediate_size: int = 4096
    layer_norm_eps: float = 1e-5
    num_channels: int = 3

    @property
    def num_patches(self) -> int:
        return (self.image_size // self.patch_size) ** 2

    @property
    def head_dim(self) -> int:
        return self.hidden_size // self.num_attention_heads


@dataclass
class TextCfg:
    hidden_size: int = 4096
    num_hidden_layers: int = 32
    num_attention_heads: int = 32
    intermediate_size: int = 11008
    vocab_size: int = 32064
    rms_norm_eps: float = 1e-5
    rope_theta: float = 10000.0

    @property
    def head_dim(self) -> int:
        return self.hidden_size // self.num_attention_heads


@dataclass
class CuLLaVOCfg:
    vision: VisionCfg = field(default_factory=VisionCfg)
    text: TextCfg = field(default_factory=TextCfg)
    image_token_index: int = 32000
    pad_token_id: int = 32001
    ignore_index: int = IGNORE_INDEX
    vision_feature_layer: int = -2
    vision_feature_select_strategy: str = "default"


def config1() -> CuLLaVOCfg:
    """BASELINE config 1: 224 px / 14, ViT d=64 x 3 layers x 4 heads,
    LM 2 layers d=128 x 4 heads, ffn 344, vocab 1024, image id 1000, pad 1001."""
    return CuLLaVOCfg(
        vision=VisionCfg(image_size=224, patch_size=14, hidden_size=64, num_hidden_layers=3,
                         num_attention_heads=4, intermediate_size=256),
        text=TextCfg(hidden_size=128, num_hidden_layers=2, num_attention_heads=4, intermediate_size=344,
                     vocab_size=1024),
        image_token_index=1000, pad_token_id=1001)


def config_small_gpu() -> CuLLaVOCfg:
    """A small config whose head dims match the production kernels (ViT 64, LM 128)."""
    return CuLLaVOCfg(
        vision=VisionCfg(image_size=224, patch_size=14, hidden_size=128, num_hidden_layers=3,
                         num_attention_heads=2, intermediate_size=512),
        text=TextCfg(hidden_size=256, num_hidden_layers=2, num_attention_heads=2, intermediate_size=688,
                     vocab_size=1024),
        image_token_index=1000, pad_token_id=1001)


def config_7b() -> CuLLaVOCfg:
    """llava-1.5-7b-hf: CLIP ViT-L/14-336 + Vicuna-7B v1.5 (public model-card dims)."""
    return CuLLaVOCfg()


# ---------------------------------------------------------------------------------------------
# seeded weights under the llava-hf (transformers ~4.37) state-dict key names
# ---------------------------------------------------------------------------------------------
def weight_shapes(cfg: CuLLaVOCfg) -> dict[str, tuple[tuple[int, ...], str]]:
    """{key: (shape, kind)}; kind picks the init distribution."""
    v, t = cfg.vision, cfg.text
    d, dv = t.hidden_size, v.hidden_size
    s: dict[str, tuple[tuple[int, ...], str]] = {}
    vp = "vision_tower.vision_model."
    s[vp + "embeddings.class_embedding"] = ((dv,), "emb")
    s[vp + "embeddings.patch_embedding.weight"] = ((dv, v.num_channels, v.patch_size, v.patch_size), "lin")
    s[vp + "embeddings.position_embedding.weight"] = ((v.num_patches + 1, dv), "emb")
    s[vp + "pre_layrnorm.weight"] = ((dv,), "norm")
    s[vp + "pre_layrnorm.bias"] = ((dv,), "bias")
    for i in range(v.num_hidden_layers):
        lp = f"{vp}encoder.layers.{i}."
        for n in ("q_proj", "k_proj", "v_proj", "out_proj"):
            s[lp + f"self_attn.{n}.weight"] = ((dv, dv), "lin")
            s[lp + f"self_attn.{n}.bias"] = ((dv,), "bias")
        s[lp + "layer_norm1.weight"] = ((dv,), "norm")
        s[lp + "layer_norm1.bias"] = ((dv,), "bias")
        s[lp + "mlp.fc1.weight"] = ((v.intermediate_size, dv), "lin")
        s[lp + "mlp.fc1.bias"] = ((v.intermediate_size,), "bias")
        s[lp + "mlp.fc2.weight"] = ((dv, v.intermediate_size), "lin")
        s[lp + "mlp.fc2.bias"] = ((dv,), "bias")
        s[lp + "layer_norm2.weight"] = ((dv,), "norm")
        s[lp + "layer_norm2.bias"] = ((dv,), "bias")
    s[vp + "post_layernorm.weight"] = ((dv,), "norm")
    s[vp + "post_layernorm.bias"] = ((dv,), "bias")
    s["multi_modal_projector.linear_1.weight"] = ((d, dv), "lin")
    s["multi_modal_projector.linear_1.bias"] = ((d,), "bias")
    s["multi_modal_projector.linear_2.weight"] = ((d, d), "lin")
    s["multi_modal_projector.linear_2.bias"] = ((d,), "bias")
    s["language_model.model.embed_tokens.weight"] = ((t.vocab_size, d), "tok")
    for i in range(t.num_hidden_layers):
        lp = f"language_model.model.layers.{i}."
        for n in ("q_proj", "k_proj", "v_proj", "o_proj"):
            s[lp + f"self_attn.{n}.weight"] = ((d, d), "lin")
        s[lp + "mlp.gate_proj.weight"] = ((t.intermediate_size, d), "lin")
        s[lp + "mlp.up_proj.weight"] = ((t.intermediate_size, d), "lin")
        s[lp + "mlp.down_proj.weight"] = ((d, t.intermediate_size), "lin")
        s[lp + "input_layernorm.weight"] = ((d,), "norm")
        s[lp + "post_attention_layernorm.weight"] = ((d,), "norm")
    s["language_model.model.norm.weight"] = ((d,), "norm")
    s["language_model.lm_head.weight"] = ((t.vocab_size, d), "lin")
    return s


def init_tensor(key: str, shape: tuple[int, ...], kind: str, seed: int) -> torch.Tensor:
    g = torch.Generator().manual_seed((zlib.crc32(key.encode()) ^ (seed * 0x9E3779B1)) & 0x7FFFFFFF)
    x = torch.randn(shape, generator=g, dtype=torch.float32)
    if kind == "lin":
        fan_in = int(math.prod(shape[1:]))
        return x * fan_in ** -0.5
    if kind == "norm":
        return 1.0 + 0.1 * x
    if kind == "bias":
        return 0.02 * x
    if kind == "emb":
        return 0.1 * x
    if kind == "tok":
        return 0.5 * x
    raise ValueError(kind)


def make_weights(cfg: CuLLaVOCfg, seed: int = 0) -> dict[str, torch.Tensor]:
    return {k: init_tensor(k, shp, kind, seed) for k, (shp, kind) in weight_shapes(cfg).items()}


def to_bf16(W: dict[str, torch.Tensor]) -> dict[str, torch.Tensor]:
    """The bf16 cast of every parameter (reference cullavo/load_cullavo.py:123-126)."""
    return {k: v.detach().to(torch.bfloat16) for k, v in W.items()}


# ---------------------------------------------------------------------------------------------
# synthetic inputs (SURVEY.md §8(d) config 1 / config 3 recipes)
# ---------------------------------------------------------------------------------------------
def make_inputs(cfg: CuLLaVOCfg, batch: int, text_len: int, image_col: int, seed: int,
                n_label: int | None = None, pad_tail: list[int] | None = None):
    """input_ids [B,S] (BOS=1 at 0, one <image> at image_col, rest U[2, image_token)),
    attention_mask (ones; optional right padding of pad_tail[b] tokens), pixel N(0,1),
    labels [B, S+P-1] = -100 except the last n_label text positions (their next-token ids)."""
    g = torch.Generator().manual_seed(seed)
    v = cfg.vision
    ids = torch.randint(2, cfg.image_token_index, (batch, text_len), generator=g)
    ids[:, 0] = 1
    ids[:, image_col] = cfg.image_token_index
    mask = torch.ones(batch, text_len, dtype=torch.long)
    if pad_tail:
        for b, n in enumerate(pad_tail):
            if n:
                ids[b, text_len - n:] = cfg.pad_token_id
                mask[b, text_len - n:] = 0
    pix = torch.randn(batch, v.num_channels, v.image_size, v.image_size, generator=g)
    L = text_len + v.num_patches - 1
    labels = torch.full((batch, L), IGNORE_INDEX, dtype=torch.long)
    if n_label is None:
        n_label = text_len // 2
    labels[:, L - n_label:] = torch.randint(2, cfg.image_token_index, (batch, n_label), generator=g)
    return ids, mask, pix, labels


# ---------------------------------------------------------------------------------------------
# ops
# ---------------------------------------------------------------------------------------------
def linear(x, w, b=None):
    """F.linear; bf16 operands accumulate in f32 and round once (a GPU bf16 GEMM + bias epilogue)"""
    if x.dtype == torch.bfloat16:
        return F.linear(x.float(), w.float(), None if b is None else b.float()).to(torch.bfloat16)
    return F.linear(x, w, b)


def rmsnorm(x, w, eps):
    """tf:models/llama/modeling_llama.py:53-70: f32 statistics, then weight * x.to(input dtype)
    (a no-op cast in f32; the bf16 rounding point in the bf16-faithful mode)"""
    xf = x.float()
    var = xf.pow(2).mean(-1, keepdim=True)
    return w * (xf * torch.rsqrt(var + eps)).to(x.dtype)


def layernorm(x, w, b, eps):
    return F.layer_norm(x, (x.shape[-1],), w, b, eps)


def rope_cos_sin(position_ids, head_dim, theta):
    """tf:models/llama/modeling_llama.py:73-128 (default rope, attention_scaling 1)"""
    inv_freq = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.int64).float() / head_dim))
    freqs = position_ids.float()[..., None] * inv_freq
    emb = torch.cat((freqs, freqs), dim=-1)
    return emb.cos(), emb.sin()


def rotate_half(x):
    """tf:models/llama/modeling_llama.py:130-135"""
    x1, x2 = x[..., : x.shape[-1] // 2], x[..., x.shape[-1] // 2:]
    return torch.cat((-x2, x1), dim=-1)


def apply_rope(x, cos, sin):
    """x [B,H,L,D], cos/sin [B,L,D] (tf:models/llama/modeling_llama.py:138-160); cos/sin are
    computed in f32 and cast to the activation dtype (:121-125)"""
    cos, sin = cos.to(x.dtype), sin.to(x.dtype)
    return x * cos[:, None] + rotate_half(x) * sin[:, None]


def attention(q, k, v, scale, allowed=None):
    """eager attention, fp32 softmax (tf:models/llama/modeling_llama.py:191-214,
    tf:models/clip/modeling_clip.py eager path); q/k/v [B,H,L,D]; allowed [B,1|H,Lq,Lk] bool.
    Rows with no allowed key return zeros."""
    # scores and softmax in f32 (the flash kernels' and FA2's arithmetic), P cast to the value
    # dtype for the PV product: with f32 inputs this is the plain fp32 eager path
    s = torch.matmul(q.float(), k.float().transpose(-1, -2)) * scale
    if allowed is not None:
        s = s.masked_fill(~allowed, float("-inf"))
        p = torch.softmax(s.float(), dim=-1)
        p = torch.nan_to_num(p, nan=0.0)
    else:
        p = torch.softmax(s.float(), dim=-1)
    if v.dtype == torch.bfloat16:  # bf16 P, f32 accumulation (FA2 / the flash kernels)
        return torch.matmul(p.to(v.dtype).float(), v.float()).to(v.dtype)
    return torch.matmul(p.to(v.dtype), v)


def quick_gelu(x):
    return x * torch.sigmoid(1.702 * x)


# ---- LoRA (peft LoraLayer on nn.Linear; reference cullavo/load_cullavo.py:94-112) -----------------
# peft is not vendored in the reference and is absent here: restated from its published
# algorithm, result = base_layer(x) + lora_B(lora_A(dropout(x))) * scaling, scaling = alpha / r.
# Parity for this row is "unpinned by the reference" (no peft run possible); the base path it
# extends is pinned by the golden vectors.
_M32 = 0xFFFFFFFF


def _fmix32(h):
    h = h ^ (h >> 16)
    h = (h * 0x85EBCA6B) & _M32
    h = h ^ (h >> 13)
    h = (h * 0xC2B2AE35) & _M32
    return h ^ (h >> 16)


def lora_keep_mask(seed: int, rows: int, cols: int, p: float):
    """numpy restatement of csrc/common.h drop_row / drop_pair / drop_keep: bool [rows, cols];
    one 32-bit hash per (token, feature pair), element (token, feature) kept iff its 16-bit half
    (low: even feature, high: odd) >= round(p * 2^16) (float32 arithmetic as in C)."""
    tok = np.arange(rows, dtype=np.uint64)[:, None]
    feat = np.arange(cols, dtype=np.uint64)[None, :]
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    t = _fmix32((tok * np.uint64(0x9E3779B1) + np.uint64(seed >> 32)) & np.uint64(_M32))
    row = _fmix32(np.uint64(seed & _M32) ^ t)
    h = _fmix32(row ^ (((feat >> np.uint64(1)) * np.uint64(0x27D4EB2F) + np.uint64(0x165667B1)) & np.uint64(_M32)))
    u16 = (h >> (np.uint64(16) * (feat & np.uint64(1)))) & np.uint64(0xFFFF)
    thr = int(np.float32(p) * np.float32(65536.0) + np.float32(0.5))
    return u16 >= np.uint64(thr)


class LoraOracle:
    """Adapter weights (keys `<linear>.lora_A.<adapter>.weight` in W), scaling, dropout p and
    an optional per-module keep mask {linear path: bool [tokens, in]} (None = no dropout)."""

    def __init__(self, adapter: str, scaling: float, p: float = 0.0, masks: dict | None = None):
        self.adapter, self.scaling, self.p, self.masks = adapter, scaling, p, masks or {}


def lora_linear(x, W, path: str, lora: LoraOracle | None, bias: bool = False):
    """peft LoraLayer.forward around F.linear (bias='none': the adapters carry no bias)."""
    y = linear(x, W[path + ".weight"], W[path + ".bias"] if bias else None)
    if lora is None or f"{path}.lora_A.{lora.adapter}.weight" not in W:
        return y
    A, B = W[f"{path}.lora_A.{lora.adapter}.weight"], W[f"{path}.lora_B.{lora.adapter}.weight"]
    xd = x
    mask = lora.masks.get(path)
    if mask is not None:
        m = torch.as_tensor(mask, dtype=x.dtype).reshape(*x.shape[:-1], x.shape[-1])
        xd = x * m / (1.0 - lora.p)
    return y + linear(linear(xd, A), B) * lora.scaling


def clip_layer(h, W, prefix, cfg: VisionCfg, lora: LoraOracle | None = None):
    """CLIPEncoderLayer (tf:models/clip/modeling_clip.py:353-384), optional peft LoRA"""
    B, T, d = h.shape
    H, D = cfg.num_attention_heads, cfg.head_dim
    x = layernorm(h, W[prefix + "layer_norm1.weight"], W[prefix + "layer_norm1.bias"], cfg.layer_norm_eps)

    def proj(n, t):
        return lora_linear(t, W, prefix + f"self_attn.{n}", lora, bias=True)

    q = proj("q_proj", x).view(B, T, H, D).transpose(1, 2)
    k = proj("k_proj", x).view(B, T, H, D).transpose(1, 2)
    v = proj("v_proj", x).view(B, T, H, D).transpose(1, 2)
    o = attention(q, k, v, D ** -0.5).transpose(1, 2).reshape(B, T, d)
    h = h + proj("out_proj", o)
    x = layernorm(h, W[prefix + "layer_norm2.weight"], W[prefix + "layer_norm2.bias"], cfg.layer_norm_eps)
    x = lora_linear(x, W, prefix + "mlp.fc1", lora, bias=True)
    x = lora_linear(quick_gelu(x), W, prefix + "mlp.fc2", lora, bias=True)
    return h + x


def vision_hidden_states(pixel_values, W, cfg: VisionCfg, n_layers: int | None = None,
                         lora: LoraOracle | None = None):
    """CLIPVisionTransformer with output_hidden_states=True; returns the tuple
    (pre_layrnorm output, layer 1 output, ..., layer n output)."""
    vp = "vision_tower.vision_model."
    B = pixel_values.shape[0]
    wpe = W[vp + "embeddings.patch_embedding.weight"]
    if wpe.dtype == torch.bfloat16:  # the conv as a GEMM: f32 accumulation, one rounding
        pe = F.conv2d(pixel_values.float(), wpe.float(), stride=cfg.patch_size).to(torch.bfloat16)
    else:
        pe = F.conv2d(pixel_values, wpe, stride=cfg.patch_size)
    pe = pe.flatten(2).transpose(1, 2)
    cls = W[vp + "embeddings.class_embedding"].expand(B, 1, -1)
    emb = torch.cat([cls, pe], dim=1) + W[vp + "embeddings.position_embedding.weight"][None]
    h = layernorm(emb, W[vp + "pre_layrnorm.weight"], W[vp + "pre_layrnorm.bias"], cfg.layer_norm_eps)
    hs = [h]
    n = cfg.num_hidden_layers if n_layers is None else n_layers
    for i in range(n):
        h = clip_layer(h, W, f"{vp}encoder.layers.{i}.", cfg, lora)
        hs.append(h)
    return hs


def projector(x, W):
    """LlavaMultiModalProjector: linear_1 -> GELU(erf) -> linear_2"""
    x = linear(x, W["multi_modal_projector.linear_1.weight"], W["multi_modal_projector.linear_1.bias"])
    x = F.gelu(x)
    return linear(x, W["multi_modal_projector.linear_2.weight"], W["multi_modal_projector.linear_2.bias"])


def merge(image_features, inputs_embeds, input_ids, attention_mask, cfg: CuLLaVOCfg, labels=None):
    """transformers ~4.37 _merge_input_ids_with_image_features (called at reference
    cullavo/arch_cullavo.py:600-602). Returns (embeds, attention_mask, labels, position_ids)."""
    num_images, num_image_patches, embed_dim = image_features.shape
    batch_size, sequence_length = input_ids.shape
    left_padding = not torch.sum(input_ids[:, -1] == torch.tensor(cfg.pad_token_id))
    special_image_token_mask = input_ids == cfg.image_token_index
    num_special_image_tokens = torch.sum(special_image_token_mask, dim=-1)
    max_embed_dim = int(num_special_image_tokens.max()) * (num_image_patches - 1) + sequence_length
    batch_indices, non_image_indices = torch.where(input_ids != cfg.image_token_index)
    new_token_positions = torch.cumsum((special_image_token_mask * (num_image_patches - 1) + 1), -1) - 1
    nb_image_pad = max_embed_dim - 1 - new_token_positions[:, -1]
    if left_padding:
        new_token_positions = new_token_positions + nb_image_pad[:, None]
    text_to_overwrite = new_token_positions[batch_indices, non_image_indices]
    final_embedding = torch.zeros(batch_size, max_embed_dim, embed_dim, dtype=inputs_embeds.dtype)
    final_attention_mask = torch.zeros(batch_size, max_embed_dim, dtype=attention_mask.dtype)
    final_labels = None
    if labels is not None:
        final_labels = torch.full((batch_size, max_embed_dim), cfg.ignore_index, dtype=input_ids.dtype)
    final_embedding = final_embedding.index_put((batch_indices, text_to_overwrite),
                                                inputs_embeds[batch_indices, non_image_indices])
    final_attention_mask[batch_indices, text_to_overwrite] = attention_mask[batch_indices, non_image_indices]
    if labels is not None:
        final_labels[batch_indices, text_to_overwrite] = labels[batch_indices, non_image_indices]
    image_to_overwrite = torch.full((batch_size, max_embed_dim), True, dtype=torch.bool)
    image_to_overwrite[batch_indices, text_to_overwrite] = False
    image_to_overwrite &= image_to_overwrite.cumsum(-1) - 1 >= nb_image_pad[:, None]
    if image_to_overwrite.sum() != image_features.shape[:-1].numel():
        raise ValueError(
            f"The input provided to the model are wrong. The number of image tokens is "
            f"{torch.sum(special_image_token_mask)} while the number of image given to the model is {num_images}.")
    final_embedding = final_embedding.masked_scatter(image_to_overwrite[..., None],
                                                     image_features.reshape(-1, embed_dim))
    final_attention_mask = final_attention_mask | image_to_overwrite
    position_ids = (final_attention_mask.cumsum(-1) - 1).masked_fill_((final_attention_mask == 0), 1)
    return final_embedding, final_attention_mask, final_labels, position_ids


def llama_layer(h, W, prefix, cfg: TextCfg, cos, sin, allowed, lora: LoraOracle | None = None):
    """LlamaDecoderLayer (tf:models/llama/modeling_llama.py:284-345), optional peft LoRA"""
    B, L, d = h.shape
    H, D = cfg.num_attention_heads, cfg.head_dim

    def lin(t, n):
        return lora_linear(t, W, prefix + n, lora)

    x = rmsnorm(h, W[prefix + "input_layernorm.weight"], cfg.rms_norm_eps)
    q = lin(x, "self_attn.q_proj").view(B, L, H, D).transpose(1, 2)
    k = lin(x, "self_attn.k_proj").view(B, L, H, D).transpose(1, 2)
    v = lin(x, "self_attn.v_proj").view(B, L, H, D).transpose(1, 2)
    q, k = apply_rope(q, cos, sin), apply_rope(k, cos, sin)
    o = attention(q, k, v, D ** -0.5, allowed).transpose(1, 2).reshape(B, L, d)
    h = h + lin(o, "self_attn.o_proj")
    x = rmsnorm(h, W[prefix + "post_attention_layernorm.weight"], cfg.rms_norm_eps)
    g = lin(x, "mlp.gate_proj")
    u = lin(x, "mlp.up_proj")
    return h + lin(F.silu(g) * u, "mlp.down_proj")


def causal_allowed(attention_mask):
    """[B,1,L,L]: key j visible from query i iff j <= i and mask[b,j] != 0 (HF causal+padding)"""
    B, L = attention_mask.shape
    causal = torch.ones(L, L, dtype=torch.bool).tril()
    return (causal[None] & (attention_mask[:, None, :] != 0))[:, None]


def llama_hidden(embeds, attention_mask, position_ids, W, cfg: TextCfg, lora: LoraOracle | None = None):
    """LlamaModel: layers + final norm; returns (final normed hidden, per-layer hidden list)"""
    cos, sin = rope_cos_sin(position_ids, cfg.head_dim, cfg.rope_theta)
    allowed = causal_allowed(attention_mask)
    h = embeds
    hs = [h]
    for i in range(cfg.num_hidden_layers):
        h = llama_layer(h, W, f"language_model.model.layers.{i}.", cfg, cos, sin, allowed, lora)
        hs.append(h)
    return rmsnorm(h, W["language_model.model.norm.weight"], cfg.rms_norm_eps), hs


def shifted_ce(logits, labels, attention_mask):
    """reference cullavo/arch_cullavo.py:651-665"""
    if attention_mask is not None:
        shift_attention_mask = attention_mask[..., 1:]
        shift_logits = logits[..., :-1, :][shift_attention_mask != 0].contiguous()
        shift_labels = labels[..., 1:][shift_attention_mask != 0].contiguous()
    else:
        shift_logits = logits[..., :-1, :].contiguous()
        shift_labels = labels[..., 1:].contiguous()
    return torch.nn.CrossEntropyLoss()(shift_logits.view(-1, shift_logits.size(-1)).float(), shift_labels.view(-1))


def needed_vision_layers(cfg: CuLLaVOCfg, layer: int) -> int:
    n = cfg.vision.num_hidden_layers
    return n + 1 + layer if layer < 0 else layer


def forward(W, cfg: CuLLaVOCfg, input_ids, pixel_values, attention_mask=None, labels=None,
            vision_feature_layer=None, vision_feature_select_strategy=None, lora: LoraOracle | None = None,
            vision_lora: LoraOracle | None = None):
    """CuLLaVOModel.forward (reference cullavo/arch_cullavo.py:546-677), training branch.
    Returns (loss or None, logits f32 [B,L,V], aux dict)."""
    layer = cfg.vision_feature_layer if vision_feature_layer is None else vision_feature_layer
    strategy = cfg.vision_feature_select_strategy if vision_feature_select_strategy is None \
        else vision_feature_select_strategy
    inputs_embeds = W["language_model.model.embed_tokens.weight"][input_ids]
    # bf16-faithful mode (bf16 weights): the processor's f32 pixels meet the bf16 conv weight
    pixel_values = pixel_values.to(W["vision_tower.vision_model.embeddings.patch_embedding.weight"].dtype)
    # image_outputs.hidden_states[vision_feature_layer]: only layers up to that index are needed
    n_needed = needed_vision_layers(cfg, layer)
    hs = vision_hidden_states(pixel_values, W, cfg.vision, n_needed, vision_lora)
    selected = hs[n_needed]
    if strategy == "default":
        selected = selected[:, 1:]
    elif strategy == "full":
        pass
    else:
        raise ValueError(f"Unexpected select feature strategy: {strategy}")
    image_features = projector(selected, W)
    if attention_mask is None:
        attention_mask = torch.ones_like(input_ids)
    embeds, mask, _, pos = merge(image_features, inputs_embeds, input_ids, attention_mask, cfg, labels)
    if labels is None:
        labels = torch.full_like(mask, cfg.ignore_index).to(torch.long)
    hidden, lm_hs = llama_hidden(embeds, mask, pos, W, cfg.text, lora)
    logits = linear(hidden, W["language_model.lm_head.weight"]).float()
    loss = shifted_ce(logits, labels, mask)
    return loss, logits, {"attention_mask": mask, "position_ids": pos, "image_features": image_features,
                          "inputs_embeds": embeds, "hidden": hidden}
