"""Algorithmic work of one CuLLaVO training sample, used by bench.py for
model TFLOP/s, MFU and the roofline of the dominant kernel. Matmul FLOPs only (2 per MAC);
causal attention counts the lower triangle; backward of a GEMM = 2x forward (dX + dW) when
its weight trains, 1x (dX only) when frozen; attention backward = 2.5x forward (5 products vs
2, FA2 convention). Recompute is never credited (there is none: activations stay in HBM).
"""
from __future__ import annotations

from .config import CuLLaVOConfig


def needed_vision_layers(cfg: CuLLaVOConfig) -> int:
    n = cfg.vision_config.num_hidden_layers
    layer = cfg.vision_feature_layer
    return n + 1 + layer if layer < 0 else layer


def _lora_fwd(tokens: int, r: int, mods) -> int:
    """forward MACs x2 of the adapters on the given (out, in) Linears: x A^T then u B^T"""
    return sum(2 * tokens * r * (i + o) for o, i in mods)


def flops_per_sample(cfg: CuLLaVOConfig, text_len: int, trainable: str = "full", lora_r: int = 64,
                     lora_vision_layers=range(12, 23)) -> dict[str, float]:
    """trainable "full": every LM GEMM trains (dX + dW). "reference" / "lora": base weights
    frozen (dX only); "lora" adds the adapters (forward, and 2x forward in backward: du, dB, dA,
    dX share) on every LM Linear and on q,k,v,fc1,fc2 of ViT layers 12-22, and the vision
    backward (dX through the adapted ViT layers)."""
    v, t = cfg.vision_config, cfg.text_config
    T = v.num_patches + 1
    L = text_len + v.num_patches - 1
    dv = v.hidden_size
    vit_layer = 2 * T * (4 * dv * dv + 2 * dv * v.intermediate_size) + 4 * T * T * dv
    vit = needed_vision_layers(cfg) * vit_layer + 2 * v.num_patches * dv * v.num_channels * v.patch_size ** 2
    d, f = t.hidden_size, t.intermediate_size
    proj = 2 * v.num_patches * (dv * d + d * d)
    gemm_layer = 2 * L * (4 * d * d + 3 * d * f)
    attn_layer = 2 * L * L * d  # causal half of QK^T + PV (4 L^2 d)
    head = 2 * L * d * t.vocab_size
    fwd = vit + proj + t.num_hidden_layers * (gemm_layer + attn_layer) + head
    lm_gemm_bwd = 2 * gemm_layer if trainable == "full" else gemm_layer
    bwd = t.num_hidden_layers * (lm_gemm_bwd + 2.5 * attn_layer) + 2 * head + 2 * proj
    lora = 0.0
    if trainable == "lora":
        lm_mods = [(d, d)] * 4 + [(f, d)] * 2 + [(d, f)]
        vit_mods = [(dv, dv)] * 3 + [(v.intermediate_size, dv), (dv, v.intermediate_size)]
        n_vit = len([i for i in lora_vision_layers if i < needed_vision_layers(cfg)])
        lora_fwd = t.num_hidden_layers * _lora_fwd(L, lora_r, lm_mods) + n_vit * _lora_fwd(T, lora_r, vit_mods)
        vit_layer_gemm = 2 * T * (4 * dv * dv + 2 * dv * v.intermediate_size)
        lora = 3 * lora_fwd
        fwd += lora_fwd
        # the vision backward runs from the last needed layer down to the first adapted one
        first = min(lora_vision_layers)
        n_bwd = max(0, needed_vision_layers(cfg) - first)
        bwd += n_bwd * (vit_layer_gemm + 2.5 * 4 * T * T * dv) + 2 * lora_fwd
    return {"fwd": float(fwd), "train": float(fwd + bwd), "lm_gemm_layer": float(gemm_layer),
            "lm_attn_layer": float(attn_layer), "vit": float(vit), "head": float(head), "proj": float(proj),
            "lora": float(lora)}
