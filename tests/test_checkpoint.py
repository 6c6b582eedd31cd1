"""Checkpoint interop: llava-hf safetensors in the ~4.37 and >= 4.45
key layouts, peft base_layer names, and CuLLaVO's own save format (reference
modeling/BaseModel.py:20-136). Runs on CPU: the arenas are built on the host (no kernels run)."""
import json
import os

import pytest
import torch

from cullavo_amd.checkpoint import load_cullavo, load_llava_safetensors, normalize_llava_key, save_cullavo


def tiny(trainable="full", seed=0, lora=None):
    from cullavo_amd.arch_cullavo import CuLLaVOModel
    from cullavo_amd.config import tiny_gpu
    return CuLLaVOModel(tiny_gpu(), device="cpu", trainable=trainable, init="random", seed=seed, lora=lora)


def to_new_layout(k):
    if k.startswith("vision_tower.") or k.startswith("multi_modal_projector."):
        return "model." + k
    if k.startswith("language_model.model."):
        return "model.language_model." + k[len("language_model.model."):]
    if k.startswith("language_model.lm_head."):
        return k[len("language_model."):]
    return k


def test_normalize_keys():
    assert normalize_llava_key("model.vision_tower.vision_model.encoder.layers.3.mlp.fc1.weight") == \
        "vision_tower.vision_model.encoder.layers.3.mlp.fc1.weight"
    assert normalize_llava_key("model.language_model.layers.0.self_attn.q_proj.weight") == \
        "language_model.model.layers.0.self_attn.q_proj.weight"
    assert normalize_llava_key("lm_head.weight") == "language_model.lm_head.weight"
    assert normalize_llava_key("language_model.model.layers.1.mlp.up_proj.base_layer.weight") == \
        "language_model.model.layers.1.mlp.up_proj.weight"
    k = "language_model.model.norm.weight"
    assert normalize_llava_key(k) == k


@pytest.mark.parametrize("layout", ["4.37", "new"])
def test_llava_safetensors_roundtrip(tmp_path, layout):
    from safetensors.torch import save_file
    src = tiny(seed=1)
    sd = {k: v.clone() for k, v in src.state_dict().items()}
    if layout == "new":
        sd = {to_new_layout(k): v for k, v in sd.items()}
    keys = sorted(sd)
    half = len(keys) // 2
    save_file({k: sd[k] for k in keys[:half]}, str(tmp_path / "model-00001-of-00002.safetensors"))
    save_file({k: sd[k] for k in keys[half:]}, str(tmp_path / "model-00002-of-00002.safetensors"))
    dst = tiny(seed=2)
    missing, unexpected = load_llava_safetensors(dst, str(tmp_path))
    assert not missing and not unexpected
    for k, v in src.state_dict().items():
        assert torch.equal(dst.state_dict()[k], v), k


def test_from_pretrained_directory(tmp_path):
    from safetensors.torch import save_file

    from cullavo_amd.arch_cullavo import CuLLaVOModel
    src = tiny(seed=3)
    cfg = src.config
    v, t = cfg.vision_config, cfg.text_config
    hf = {"model_type": "llava", "image_token_index": cfg.image_token_index, "pad_token_id": cfg.pad_token_id,
          "vision_feature_layer": -2, "vision_feature_select_strategy": "default", "projector_hidden_act": "gelu",
          "vision_config": {"image_size": v.image_size, "patch_size": v.patch_size, "hidden_size": v.hidden_size,
                            "num_hidden_layers": v.num_hidden_layers, "num_attention_heads": v.num_attention_heads,
                            "intermediate_size": v.intermediate_size, "hidden_act": "quick_gelu"},
          "text_config": {"hidden_size": t.hidden_size, "num_hidden_layers": t.num_hidden_layers,
                          "num_attention_heads": t.num_attention_heads, "intermediate_size": t.intermediate_size,
                          "vocab_size": t.vocab_size, "rms_norm_eps": t.rms_norm_eps, "rope_theta": t.rope_theta}}
    with open(tmp_path / "config.json", "w") as f:
        json.dump(hf, f)
    save_file({k: v.clone() for k, v in src.state_dict().items()}, str(tmp_path / "model.safetensors"))
    m = CuLLaVOModel.from_pretrained(str(tmp_path), device="cpu")
    assert m.config.text_config.hidden_size == t.hidden_size and m.config.image_token_index == cfg.image_token_index
    for k, v in src.state_dict().items():
        assert torch.equal(m.state_dict()[k], v), k


def test_cullavo_save_format_roundtrip(tmp_path):
    from cullavo_amd.lora import LoraSettings
    s = LoraSettings(vision_layers=(1, 2))
    src = tiny("lora", seed=4, lora=s)
    with torch.no_grad():
        for k, p in src.arenas["lora"].params.items():
            p.normal_(0, 0.1)
    save_cullavo(src, str(tmp_path), epoch=3)
    root = tmp_path / "epoch3"
    for f in ["CuLLaVO.pt", "cullavo/multi_modal_projector.pt", "cullavo/lm_head.pt", "cullavo/embed_tokens.pt",
              "cullavo/vision_tower/adapter_model.safetensors", "cullavo/language_model/adapter_model.safetensors",
              "cullavo/language_model/adapter_config.json"]:
        assert (root / f).exists(), f
    from safetensors import safe_open
    with safe_open(str(root / "cullavo/language_model/adapter_model.safetensors"), "pt") as h:
        keys = list(h.keys())
    # transformers save_pretrained of a PEFT-adapted tower: base_model.model. + tower-relative key,
    # adapter name dropped (tf:modeling_utils.py:3410-3422, tf:integrations/peft.py:537-564)
    assert "base_model.model.model.layers.0.self_attn.q_proj.lora_A.weight" in keys
    assert torch.load(root / "cullavo/lm_head.pt", weights_only=True).keys() == {"weight"}
    cfg = json.load(open(root / "cullavo/vision_tower/adapter_config.json"))
    assert (cfg["r"], cfg["lora_alpha"], cfg["layers_to_transform"]) == (64, 16.0, [1, 2])
    dst = tiny("lora", seed=5, lora=s)
    base_before = {k: v.clone() for k, v in dst.arenas["layers"].params.items()}
    load_cullavo(dst, str(root / "CuLLaVO.pt"))
    for name in ("lora", "projector", "head", "embed"):
        for k, p in src.arenas[name].params.items():
            assert torch.equal(dst.arenas[name].params[k], p), k
    for k, v in base_before.items():  # frozen base weights are not part of the save format
        assert torch.equal(dst.arenas["layers"].params[k], v)


def test_full_policy_checkpoint_keeps_trained_decoder(tmp_path):
    """'full' trains the decoder layers: save_cullavo writes them (language_model/model.safetensors)
    and load_cullavo restores them -- nothing trained is silently dropped."""
    src = tiny("full", seed=6)
    with torch.no_grad():
        src.arenas["layers"].flat.normal_(0, 0.05)
    save_cullavo(src, str(tmp_path), epoch=1)
    f = tmp_path / "epoch1" / "cullavo" / "language_model" / "model.safetensors"
    assert f.exists()
    from safetensors import safe_open
    with safe_open(str(f), "pt") as h:
        assert "model.layers.0.mlp.down_proj.weight" in set(h.keys())
    dst = tiny("full", seed=7)
    load_cullavo(dst, str(tmp_path / "epoch1" / "CuLLaVO.pt"))
    for name in ("layers", "projector", "head", "embed"):
        for k, p in src.arenas[name].params.items():
            assert torch.equal(dst.arenas[name].params[k], p), k
