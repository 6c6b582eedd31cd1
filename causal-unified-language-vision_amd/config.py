"""Configuration objects with the attribute names the reference reads from the HF configs
(reference cullavo/arch_cullavo.py:562-575 reads config.{output_attentions, output_hidden_states,
use_return_dict, vision_feature_layer, vision_feature_select_strategy, ignore_index,
image_token_index, pad_token_id}; the towers read CLIPVisionConfig / LlamaConfig fields).
``CuLLaVOConfig.from_hf`` accepts a transformers LlavaConfig so an existing llava-hf config
drives this model unchanged.
"""
from __future__ import annotations

from dataclasses import dataclass, field


@dataclass
class CLIPVisionConfig:
    image_size: int = 336
    patch_size: int = 14
    hidden_size: int = 1024
    num_hidden_layers: int = 24
    num_attention_heads: int = 16
    intermediate_size: int = 4096
    layer_norm_eps: float = 1e-5
    num_channels: int = 3
    hidden_act: str = "quick_gelu"

    @property
    def num_patches(self) -> int:
        return (self.image_size // self.patch_size) ** 2

    @property
    def head_dim(self) -> int:
        return self.hidden_size // self.num_attention_heads


@dataclass
class LlamaConfig:
    hidden_size: int = 4096
    num_hidden_layers: int = 32
    num_attention_heads: int = 32
    intermediate_size: int = 11008
    vocab_size: int = 32064
    rms_norm_eps: float = 1e-5
    rope_theta: float = 10000.0
    hidden_act: str = "silu"

    @property
    def head_dim(self) -> int:
        return self.hidden_size // self.num_attention_heads


@dataclass
class CuLLaVOConfig:
    vision_config: CLIPVisionConfig = field(default_factory=CLIPVisionConfig)
    text_config: LlamaConfig = field(default_factory=LlamaConfig)
    image_token_index: int = 32000
    pad_token_id: int = 32001
    ignore_index: int = -100
    vision_feature_layer: int = -2
    vision_feature_select_strategy: str = "default"
    projector_hidden_act: str = "gelu"
    output_attentions: bool = False
    output_hidden_states: bool = False
    use_return_dict: bool = True

    @classmethod
    def from_json(cls, path: str) -> "CuLLaVOConfig":
        """From a llava-hf config.json (a directory or the file) without transformers."""
        import json
        import os
        from types import SimpleNamespace
        if os.path.isdir(path):
            path = os.path.join(path, "config.json")
        with open(path) as f:
            d = json.load(f)

        def ns(x):
            return SimpleNamespace(**{k: ns(v) if isinstance(v, dict) else v for k, v in x.items()})
        hf = ns(d)
        v = hf.vision_config
        for k, dv in (("image_size", 336), ("patch_size", 14), ("hidden_size", 1024), ("num_hidden_layers", 24),
                      ("num_attention_heads", 16), ("intermediate_size", 4096), ("layer_norm_eps", 1e-5),
                      ("hidden_act", "quick_gelu")):
            if not hasattr(v, k):
                setattr(v, k, dv)
        t = hf.text_config
        for k, dv in (("hidden_size", 4096), ("num_hidden_layers", 32), ("num_attention_heads", 32),
                      ("intermediate_size", 11008), ("vocab_size", 32064), ("rms_norm_eps", 1e-5)):
            if not hasattr(t, k):
                setattr(t, k, dv)
        for k, dv in (("vision_feature_layer", -2), ("vision_feature_select_strategy", "default")):
            if not hasattr(hf, k):
                setattr(hf, k, dv)
        return cls.from_hf(hf)

    @classmethod
    def from_hf(cls, hf) -> "CuLLaVOConfig":
        """Build from a transformers LlavaConfig (any version with vision_config/text_config)."""
        v, t = hf.vision_config, hf.text_config
        if getattr(t, "num_key_value_heads", t.num_attention_heads) != t.num_attention_heads:
            raise ValueError("grouped-query attention is not on the CuLLaVO path (Vicuna-7B is MHA)")
        rope = getattr(t, "rope_theta", None)
        if rope is None:
            rope = (getattr(t, "rope_parameters", None) or {}).get("rope_theta", 10000.0)
        return cls(
            vision_config=CLIPVisionConfig(
                image_size=v.image_size, patch_size=v.patch_size, hidden_size=v.hidden_size,
                num_hidden_layers=v.num_hidden_layers, num_attention_heads=v.num_attention_heads,
                intermediate_size=v.intermediate_size, layer_norm_eps=v.layer_norm_eps,
                num_channels=getattr(v, "num_channels", 3), hidden_act=v.hidden_act),
            text_config=LlamaConfig(
                hidden_size=t.hidden_size, num_hidden_layers=t.num_hidden_layers,
                num_attention_heads=t.num_attention_heads, intermediate_size=t.intermediate_size,
                vocab_size=t.vocab_size, rms_norm_eps=t.rms_norm_eps, rope_theta=float(rope)),
            image_token_index=getattr(hf, "image_token_index", getattr(hf, "image_token_id", 32000)),
            pad_token_id=getattr(hf, "pad_token_id", None) or getattr(t, "pad_token_id", None) or 32001,
            ignore_index=getattr(hf, "ignore_index", -100),
            vision_feature_layer=hf.vision_feature_layer,
            vision_feature_select_strategy=hf.vision_feature_select_strategy,
            projector_hidden_act=getattr(hf, "projector_hidden_act", "gelu"),
        )


def llava_1_5_7b() -> CuLLaVOConfig:
    """llava-hf/llava-1.5-7b-hf: CLIP ViT-L/14-336 + Vicuna-7B v1.5 (BASELINE configs 2-4)."""
    return CuLLaVOConfig()


def llava_1_5_13b() -> CuLLaVOConfig:
    """ViT-L/14-336 + Llama-2-13B (BASELINE config 5)."""
    return CuLLaVOConfig(text_config=LlamaConfig(hidden_size=5120, num_hidden_layers=40, num_attention_heads=40,
                                                 intermediate_size=13824, vocab_size=32064))


def tiny_gpu() -> CuLLaVOConfig:
    """Small config with the production head dims (ViT 64, LM 128) for parity tests."""
    return CuLLaVOConfig(
        vision_config=CLIPVisionConfig(image_size=224, patch_size=14, hidden_size=128, num_hidden_layers=3,
                                       num_attention_heads=2, intermediate_size=512),
        text_config=LlamaConfig(hidden_size=256, num_hidden_layers=2, num_attention_heads=2, intermediate_size=688,
                                vocab_size=1024),
        image_token_index=1000, pad_token_id=1001)


def config1() -> CuLLaVOConfig:
    """BASELINE config 1: 224 px / 14, ViT d=64 x 3 layers x 4 heads (head
    dim 16), LM 2 layers d=128 x 4 heads (head dim 32), ffn 344, vocab 1024."""
    return CuLLaVOConfig(
        vision_config=CLIPVisionConfig(image_size=224, patch_size=14, hidden_size=64, num_hidden_layers=3,
                                       num_attention_heads=4, intermediate_size=256),
        text_config=LlamaConfig(hidden_size=128, num_hidden_layers=2, num_attention_heads=4, intermediate_size=344,
                                vocab_size=1024),
        image_token_index=1000, pad_token_id=1001)
