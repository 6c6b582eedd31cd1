"""KV-cache decode and generate().

Reference: CuLLaVOModel.generate(**inputs, do_sample=True, temperature=0.9, top_k=50,
top_p=0.95, max_new_tokens=1000, use_cache=True) (cullavo/arch_cullavo.py:362-363, the
step-2 pre-labelling loop) runs HF's GenerationMixin over forward(); the cached branch of that
forward is :605-636 (transformers ~4.37 llava: the new token's position is the number of
attended tokens so far, position_ids = attention_mask.sum(-1) - 1).

MI355X design: the cache is preallocated once per generate() call in HBM as K, V
[layers, B, Lmax, H*D] bf16; the prompt (text + 576 image rows, merged exactly as training
does) is prefilled through the same fused kernels (GEMMs, RoPE, causal flash attention) with
its rotated keys/values appended by kv_append; every decode step runs the layers on one row
per sequence and attends with the split-KV attn_decode kernel. Left-padded batches are
supported through kv_start (keys before the first attended token are masked); a prompt with
holes in its attention mask is not (decode attention reads one contiguous key range).
Sampling (temperature, top-k, top-p, multinomial; or greedy) follows HF's warper order on the
GPU with torch ops: it is O(B x vocab) per token and not a kernel of the hot path.
"""
from __future__ import annotations

import torch

from . import ops
from .functions import StepContext
from .lora import NO_LORA

import os

# decode-step fusions (all bitwise the unfused values), CULLAVO_DECODE_FUSE = comma list:
#   "gu"    (default on) the SwiGLU in the gate|up product's epilogue (cullavo_decode_linear
#           transform 3: one launch instead of the product + cullavo_swiglu_fwd);
#   "rope"  (default on) RoPE + KV append inside decode attention (cullavo_attn_decode_rope);
#   "norm"  the two RMSNorms into the q|k|v and gate|up products' X loads, "swiglu" the SwiGLU into
#           down_proj's X loads (round 4: ~2x slower per product, profiles/r04/decode/decode_fusions_ab.txt;
#           round 5, the whole workgroup normalising: 3.73 vs 3.53 ms per token at batch 1, 4.67 vs
#           4.02 at batch 4 -- every workgroup redoing the row norm still costs more than the one
#           norm launch: off by default). A norm in the TAIL of o_proj / down_proj instead (the last
#           workgroup by an agent-scope counter normalises the rows) measured 3.78 vs 3.53 ms
#           (profiles/r05/decode/pnorm_ab_*): not kept
_FUSE = {f.strip() for f in os.environ.get("CULLAVO_DECODE_FUSE", "gu,rope").split(",") if f.strip()}
FUSE_DECODE_NORMS = "norm" in _FUSE
FUSE_DECODE_SWIGLU = "swiglu" in _FUSE
FUSE_DECODE_GU = "gu" in _FUSE
FUSE_DECODE_ROPE = "rope" in _FUSE


class KVCache:
    """Per-layer K, V [B, Lmax, H*D] in HBM plus the per-row state the decode kernels read."""

    def __init__(self, n_layers: int, B: int, max_len: int, H: int, D: int, device, dtype=torch.bfloat16):
        self.k = torch.empty((n_layers, B, max_len, H * D), dtype=dtype, device=device)
        self.v = torch.empty_like(self.k)
        self.B, self.max_len, self.H, self.D = B, max_len, H, D
        self.length = 0                      # rows written (same for every sequence)
        self.kv_start = None                 # int32 [B]: first attended key (left padding)
        self.next_pos = None                 # int64 [B]: RoPE position of the next token

    def __len__(self):
        return self.k.shape[0]

    def __getitem__(self, layer: int):
        """HF legacy view: (key, value) as [B, H, L, D] over the filled rows."""
        B, L, H, D = self.B, self.length, self.H, self.D
        return (self.k[layer, :, :L].view(B, L, H, D).transpose(1, 2),
                self.v[layer, :, :L].view(B, L, H, D).transpose(1, 2))

    def get_seq_length(self) -> int:
        return self.length

    def to_legacy_cache(self):
        """transformers' legacy tuple: ((key, value) [B, H, L, D] per layer), views of this cache"""
        return tuple(self[i] for i in range(len(self)))

    def grow(self, max_len: int):
        """re-allocate with room for max_len rows per sequence, keeping the filled rows"""
        if max_len <= self.max_len:
            return
        k = torch.empty((self.k.shape[0], self.B, max_len, self.k.shape[3]), dtype=self.k.dtype, device=self.k.device)
        v = torch.empty_like(k)
        k[:, :, :self.length].copy_(self.k[:, :, :self.length])
        v[:, :, :self.length].copy_(self.v[:, :, :self.length])
        self.k, self.v, self.max_len = k, v, max_len

    @classmethod
    def from_legacy(cls, legacy, attention_mask=None, extra: int = 256):
        """A transformers-layout cache -- the legacy tuple of per-layer (key, value) [B, H, L, D]
        (what the reference's decode branch indexes, arch_cullavo.py:608-614) or any object with
        to_legacy_cache() (DynamicCache) -- copied into a KVCache with `extra` free rows.
        Attended keys: the reference's rule (:611-632) -- a cached position whose first-layer
        keys are zero is not attended, nor are the
        left-padding positions of the caller's attention_mask -- which must leave one contiguous
        span per sequence (what the decode kernels read)."""
        if hasattr(legacy, "to_legacy_cache"):
            legacy = legacy.to_legacy_cache()
        if not isinstance(legacy, (tuple, list)) or not legacy or len(legacy[0]) != 2:
            raise TypeError(f"past_key_values: expected a KVCache or a transformers legacy cache (tuple of per-layer "
                            f"(key, value) [B, H, L, D]), got {type(legacy).__name__}")
        k0 = legacy[0][0]
        B, H, L, D = k0.shape
        cache = cls(len(legacy), B, L + extra, H, D, k0.device, dtype=k0.dtype)
        for i, (k, v) in enumerate(legacy):
            if k.shape != (B, H, L, D) or v.shape != (B, H, L, D):
                raise ValueError(f"layer {i}: key {tuple(k.shape)} / value {tuple(v.shape)} vs {(B, H, L, D)}")
            cache.k[i, :, :L].copy_(k.transpose(1, 2).reshape(B, L, H * D))
            cache.v[i, :, :L].copy_(v.transpose(1, 2).reshape(B, L, H * D))
        # a slot is unattended when its first-layer keys are all zero: the reference tests only the
        # head-dim component 0 summed over the heads, which a real key also hits by chance (two
        # bf16 values of opposite sign over 2 heads: seen in the tiny config), so every component
        # is required to vanish here
        att = k0.float().abs().sum((1, 3)) != 0
        if attention_mask is not None:
            if attention_mask.shape[1] >= L:  # a mask over the merged rows
                att &= attention_mask[:, :L].to(k0.device) != 0
            else:  # the caller's text-level mask (:618-632): its leading zeros are the left padding
                lead = (attention_mask.to(torch.int64).cumsum(-1) == 0).sum(-1).to(k0.device)
                att &= torch.arange(L, device=k0.device)[None] >= lead[:, None]
        am = att.to(torch.int64)
        first = (am.cumsum(-1) == 0).sum(-1)
        if bool((am.sum(-1) + first != L).any()):
            raise NotImplementedError("KV-cache decode needs one contiguous attended span per sequence "
                                      "(left padding only)")
        cache.length = L
        cache.kv_start = first.to(torch.int32)
        cache.next_pos = am.sum(-1)
        return cache


def layer_infer(layer, h, sctx: StepContext, cache: KVCache, li: int, Lnew: int, start, kv_len,
                attn_len: int | None = None):
    """One LlamaDecoderLayer over Lnew new rows per sequence (prefill: Lnew = prompt length on an
    empty cache; decode: Lnew = 1), appending their keys/values to the cache. No autograd.
    attn_len: the key range decode attention is sized for (default: the filled rows + 1)."""
    cfg = layer.cfg
    d, H, D = cfg.hidden_size, cfg.num_attention_heads, cfg.head_dim
    lg = layer.lora_groups
    B = sctx.B
    # FUSE_DECODE_NORMS: the RMSNorms inside the q|k|v and gate|up weight-streaming products
    # (cullavo_decode_linear transform 1 / 4: every workgroup normalises the rows once into LDS; the
    # round-4 per-fragment form was ~2x slower, profiles/r04/decode/decode_fusions_ab.txt) for the
    # rows that fit LDS (M (d + 8) * 2 <= 64 KiB); FUSE_DECODE_SWIGLU: the SwiGLU in down_proj's
    # X loads (transform 2), only without FUSE_DECODE_GU. All bitwise the unfused values.
    fused = (FUSE_DECODE_NORMS and Lnew == 1 and h.shape[0] <= 16 and h.shape[0] * (d + 8) * 2 <= 65536
             and h.dtype == torch.bfloat16
             and all(g is NO_LORA for g in lg.values()))
    if fused:
        qkv = ops.decode_linear(h, layer.w_qkv(), transform=1, norm_w=layer.input_layernorm.weight,
                                eps=cfg.rms_norm_eps)
    else:
        x1, _ = ops.rmsnorm_fwd(h, layer.input_layernorm.weight, cfg.rms_norm_eps)
        t, _ = lg["qkv"].forward(x1, False, 0)
        qkv = ops.linear(x1, layer.w_qkv(), addend=t)
    q, k, v = qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:]
    if Lnew == 1 and qkv.dtype == torch.bfloat16 and FUSE_DECODE_ROPE:
        # decode: RoPE, the cache append and attention in one pass (the cache row is start[b])
        o = ops.attn_decode_rope(q, k, v, sctx.position_ids, cache.k[li], cache.v[li], start, B=B, H=H, D=D,
                                 max_len=attn_len if attn_len is not None else cache.length + 1,
                                 scale=D ** -0.5, theta=cfg.rope_theta, kv_start=sctx.kv_start)
    elif Lnew == 1 and qkv.dtype == torch.bfloat16:
        # decode: rotated k goes straight to the cache (one launch for RoPE + append)
        ops.rope_kv_append(q, k, v, sctx.position_ids, cache.k[li], cache.v[li], start, hq=H, head_dim=D,
                           theta=cfg.rope_theta, B=B, Lnew=1)
    else:
        ops.rope(q, k, sctx.position_ids, hq=H, hk=H, head_dim=D, theta=cfg.rope_theta)
        ops.kv_append(k, v, cache.k[li], cache.v[li], start, B=B, Lnew=Lnew)
    if Lnew > 1:
        o, _ = ops.attn_fwd(q, k, v, B=B, H=H, Lq=Lnew, Lk=Lnew, D=D, scale=D ** -0.5, causal=True,
                            kv_start=sctx.kv_start)
    elif not (qkv.dtype == torch.bfloat16 and FUSE_DECODE_ROPE):
        o = ops.attn_decode(q, cache.k[li], cache.v[li], kv_len, B=B, H=H, D=D,
                            max_len=attn_len if attn_len is not None else cache.length + 1,
                            scale=D ** -0.5, kv_start=sctx.kv_start)
    t, _ = lg["o"].forward(o, False, 0)
    h2 = ops.linear(o, layer.self_attn.o_proj.weight, residual=h, addend=t)
    if fused:
        if FUSE_DECODE_GU:  # RMSNorm, gate|up product and SwiGLU in one launch (transform 4)
            a = ops.decode_linear(h2, layer.w_gu(), transform=4, norm_w=layer.post_attention_layernorm.weight,
                                  eps=cfg.rms_norm_eps)
            return ops.linear(a, layer.mlp.down_proj.weight, residual=h2)
        gu = ops.decode_linear(h2, layer.w_gu(), transform=1, norm_w=layer.post_attention_layernorm.weight,
                               eps=cfg.rms_norm_eps)
        if FUSE_DECODE_SWIGLU:
            return ops.decode_linear(gu, layer.mlp.down_proj.weight, transform=2, residual=h2)
        return ops.linear(ops.swiglu_fwd(gu), layer.mlp.down_proj.weight, residual=h2)
    x2, _ = ops.rmsnorm_fwd(h2, layer.post_attention_layernorm.weight, cfg.rms_norm_eps)
    t, _ = lg["gu"].forward(x2, False, 0)
    if FUSE_DECODE_GU and t is None and Lnew == 1 and x2.shape[0] <= 16 and x2.dtype == torch.bfloat16:
        a = ops.decode_linear(x2, layer.w_gu(), transform=3)  # gate|up product + SwiGLU, one launch
    else:
        gu = ops.linear(x2, layer.w_gu(), addend=t)
        a = ops.swiglu_fwd(gu)
    t, _ = lg["down"].forward(a, False, 0)
    return ops.linear(a, layer.mlp.down_proj.weight, residual=h2, addend=t)


class DecodeGraph:
    """One cached decode step of the LM -- the new token's embedding row, every decoder layer at one
    row per sequence, the final norm and lm_head -- captured once as a HIP graph and replayed per
    token (about 330 kernel launches per 7B step; replayed, the host no longer issues them one by
    one). Everything the step reads that changes from token to token lives in device buffers the
    graph owns and advances itself: the token ids (written by the caller before each replay), the
    RoPE positions and the cache write row (+1 at the end of every replay); decode attention runs
    over the cache's full capacity (chunks past a row's length exit at once), so the grid does not
    depend on the current length. The cache must not grow while the graph is alive (generate()
    sizes it for prompt + max_new_tokens)."""

    def __init__(self, model, cache: KVCache):
        lm = model.language_model
        self.cache, self.lm = cache, lm
        B = cache.B
        dev = cache.k.device
        self.ids = torch.zeros(B, dtype=torch.long, device=dev)
        self.pos = cache.next_pos.to(torch.int64).clone()
        self.start = torch.full((B,), cache.length, dtype=torch.int32, device=dev)
        self.embed = model.get_input_embeddings()
        self.graph = torch.cuda.CUDAGraph()
        self.steps_left = cache.max_len - cache.length
        stream = torch.cuda.Stream(device=dev)
        stream.wait_stream(torch.cuda.current_stream(dev))
        traced = ops._TRACE["key"]
        ops._TRACE["key"] = None  # no per-launch timing events inside the captured graph
        try:
            with torch.cuda.stream(stream):
                with torch.cuda.graph(self.graph, stream=stream, capture_error_mode="thread_local"):
                    self.logits = self._step()
        finally:
            ops._TRACE["key"] = traced
        torch.cuda.current_stream(dev).wait_stream(stream)
        cache.next_pos = self.pos  # advanced in place by every replay

    def _step(self):
        lm, cache = self.lm, self.cache
        cfg = lm.cfg
        B = cache.B
        h = self.embed(self.ids[:, None]).reshape(B, cfg.hidden_size)
        sctx = StepContext(B, 1, self.pos[:, None], cache.kv_start, lora_seed=0)
        # the unfused decode attention reads kv_len = start + 1 (the fused one derives it from start)
        kv_len = None if FUSE_DECODE_ROPE and cache.k.dtype == torch.bfloat16 else self.start + 1
        for li, layer in enumerate(lm.model.layers):
            h = layer_infer(layer, h, sctx, cache, li, 1, self.start, kv_len, attn_len=cache.max_len)
        x, _ = ops.rmsnorm_fwd(h, lm.model.norm.weight, cfg.rms_norm_eps)
        logits = ops.linear(x, lm.lm_head.weight)
        self.pos.add_(1)
        self.start.add_(1)
        return logits.view(B, 1, -1)

    def step(self, tokens):
        """Append `tokens` ([B] ids) to the cache and return the next logits [B, 1, V] (a view of
        the graph's output buffer, overwritten by the next replay)."""
        if self.steps_left <= 0:
            raise ValueError("decode graph: the KV cache is full")
        self.ids.copy_(tokens.reshape(-1))
        self.graph.replay()
        self.cache.length += 1
        self.steps_left -= 1
        return self.logits


def lm_infer(lm, embeds, attention_mask, position_ids, cache: KVCache | None, max_len: int):
    """LlamaForCausalLM with a KV cache: prefill (cache None or empty) or one decode step.
    Returns (logits [B, Lnew, V] bf16, cache)."""
    B, Lnew, d = embeds.shape
    cfg = lm.cfg
    if embeds.dtype != torch.bfloat16:
        raise NotImplementedError("KV-cache decode runs on the bf16 model (the f32 mode is a parity mode)")
    if cache is None:
        cache = KVCache(cfg.num_hidden_layers, B, max_len, cfg.num_attention_heads, cfg.head_dim, embeds.device)
    if cache.length == 0:
        if Lnew > cache.max_len:  # kv_append writes rows [0, Lnew) of every sequence's cache
            raise ValueError(f"prompt of {Lnew} rows does not fit the KV cache ({cache.max_len} rows)")
        if attention_mask is None:
            attention_mask = torch.ones(B, Lnew, dtype=torch.long, device=embeds.device)
        am = attention_mask.to(torch.int64)
        first = (am.cumsum(-1) == 0).sum(-1)
        # contiguous valid range only: zeros may appear only before the first attended token
        holes = (am.sum(-1) + first != Lnew)
        if bool(holes.any()):
            raise NotImplementedError("KV-cache generation needs left padding (no masked tokens after the "
                                      "first attended one)")
        cache.kv_start = first.to(torch.int32)
        if position_ids is None:
            position_ids = (am.cumsum(-1) - 1).masked_fill(am == 0, 1)
        cache.next_pos = position_ids[:, -1].to(torch.int64) + 1
    else:
        if Lnew != 1:
            raise NotImplementedError("after the prefill, cached steps take one token per sequence")
        if cache.length + 1 > cache.max_len:  # room for 256 more steps (one copy per 256 steps)
            cache.grow(cache.max_len + 256)
        if position_ids is None:
            position_ids = cache.next_pos[:, None]
        cache.next_pos = cache.next_pos + 1
    sctx = StepContext(B, Lnew, position_ids, cache.kv_start, lora_seed=0)
    h = embeds.reshape(B * Lnew, d).contiguous()
    start = torch.full((B,), cache.length, dtype=torch.int32, device=h.device)
    kv_len = start + Lnew
    for li, layer in enumerate(lm.model.layers):
        h = layer_infer(layer, h, sctx, cache, li, Lnew, start, kv_len)
    cache.length += Lnew
    x, _ = ops.rmsnorm_fwd(h, lm.model.norm.weight, cfg.rms_norm_eps)
    logits = ops.linear(x, lm.lm_head.weight)
    return logits.view(B, Lnew, -1), cache


def sample_next(logits, *, do_sample: bool, temperature: float = 1.0, top_k: int = 0, top_p: float = 1.0,
                generator=None):
    """HF's warper order (temperature -> top-k -> top-p) then multinomial; argmax when greedy."""
    if not do_sample:
        return logits.argmax(-1)
    x = logits.float()
    if temperature != 1.0:
        x = x / temperature
    if top_k and top_k > 0:
        kth = torch.topk(x, min(top_k, x.shape[-1]), dim=-1).values[..., -1:]
        x = x.masked_fill(x < kth, float("-inf"))
    if top_p < 1.0:
        sx, si = torch.sort(x, descending=False, dim=-1)
        cum = sx.softmax(-1).cumsum(-1)
        remove = cum <= (1 - top_p)
        remove[..., -1:] = False
        x = x.masked_fill(remove.scatter(-1, si, remove), float("-inf"))
    return torch.multinomial(x.softmax(-1), 1, generator=generator).squeeze(-1)
