"""Checkpoint interop.

1. llava-hf weights: `*.safetensors` shards (optionally with `model.safetensors.index.json`) in
   either key layout
     transformers ~4.37 (what the reference loads, cullavo/load_cullavo.py:86):
       vision_tower.vision_model.*, multi_modal_projector.*, language_model.model.*,
       language_model.lm_head.weight
     transformers >= 4.45 / 5.x (nested LlavaModel):
       model.vision_tower.vision_model.*, model.multi_modal_projector.*,
       model.language_model.*, lm_head.weight
   and peft-wrapped names (`<linear>.base_layer.weight`). Tensors are streamed one at a time
   from safe_open straight into the HBM arenas (no full host copy of a 13.5 GB checkpoint).

2. CuLLaVO's own save format (reference modeling/BaseModel.py:20-69 save, :71-136 load):
     <save_dir>/epoch{e}/CuLLaVO.pt                                   non-LLM state (torch.save)
     <save_dir>/epoch{e}/cullavo/vision_tower/adapter_model.safetensors    LoRA of the ViT
     <save_dir>/epoch{e}/cullavo/vision_tower/adapter_config.json
     <save_dir>/epoch{e}/cullavo/language_model/adapter_model.safetensors  LoRA of the LM
     <save_dir>/epoch{e}/cullavo/language_model/adapter_config.json
     <save_dir>/epoch{e}/cullavo/multi_modal_projector.pt   {linear_1.weight, ...}
     <save_dir>/epoch{e}/cullavo/lm_head.pt                 {weight}
     <save_dir>/epoch{e}/cullavo/embed_tokens.pt            {weight}
   Adapter keys are what the reference's `<tower>.save_pretrained(path)` writes for a model
   carrying transformers-PEFT adapters (reference modeling/BaseModel.py:41-42 on towers set up
   with add_adapter, cullavo/load_cullavo.py:111-112): transformers' save_pretrained
   (tf:modeling_utils.py:3410-3422, save_peft_format=True by default) takes
   get_adapter_state_dict (tf:integrations/peft.py:537-564 -> peft get_peft_model_state_dict,
   which drops the adapter name) and prefixes `base_model.model.`:
     base_model.model.vision_model.encoder.layers.N.self_attn.q_proj.lora_A.weight
     base_model.model.model.layers.N.self_attn.q_proj.lora_A.weight
   The loader accepts that form, the unprefixed form and the adapter-named parameter names.
   (peft itself is not importable here: the key form is pinned to the transformers code above,
   the peft step is restated -- parity of the adapter file layout is otherwise unpinned.)
   Trainable arenas the reference never trains (this build's full fine-tune recipe) are saved
   too, in the tower's own safetensors layout, so no trained weight is dropped:
     <save_dir>/epoch{e}/cullavo/language_model/model.safetensors   model.layers.N.*, model.norm.weight
     <save_dir>/epoch{e}/cullavo/vision_tower/model.safetensors     vision_model.* (trainable tower only)
   .pt files are read with torch.load(weights_only=True) only.
"""
from __future__ import annotations

import glob
import json
import os

import torch

VISION_PREFIX = "vision_tower."
LM_PREFIX = "language_model."
PEFT_PREFIX = "base_model.model."
# arenas saved as whole-tower safetensors when trainable: arena -> (sub-directory, key prefix)
TOWER_ARENAS = {"layers": ("language_model", LM_PREFIX), "vision": ("vision_tower", VISION_PREFIX)}
COVERED_ARENAS = {"lora", "projector", "head", "embed", *TOWER_ARENAS}


# ---------------------------------------------------------------------------------------------
# key normalisation
# ---------------------------------------------------------------------------------------------
def normalize_llava_key(key: str) -> str:
    """Any llava-hf / peft layout -> the ~4.37 names the arenas use."""
    key = key.replace(".base_layer.", ".")
    if key.startswith("model.vision_tower."):
        return key[len("model."):]
    if key.startswith("model.multi_modal_projector."):
        return key[len("model."):]
    if key.startswith("model.language_model."):
        return "language_model.model." + key[len("model.language_model."):]
    if key.startswith("lm_head."):
        return "language_model." + key
    return key


def _own_params(model) -> dict:
    own = {}
    for ar in model.arenas.values():
        own.update(ar.params)
    return own


def load_llava_safetensors(model, path: str, strict: bool = True):
    """Stream a llava-hf checkpoint directory (or one .safetensors file) into the model.
    Returns (missing, unexpected) key lists like nn.Module.load_state_dict."""
    from safetensors import safe_open
    files = [path] if path.endswith(".safetensors") else sorted(glob.glob(os.path.join(path, "*.safetensors")))
    if not files:
        raise FileNotFoundError(f"no .safetensors under {path}")
    own = _own_params(model)
    seen, unexpected = set(), []
    with torch.no_grad():
        for f in files:
            with safe_open(f, framework="pt", device="cpu") as h:
                for k in h.keys():
                    nk = normalize_llava_key(k)
                    if nk not in own:
                        unexpected.append(k)
                        continue
                    t = h.get_tensor(k)
                    p = own[nk]
                    if tuple(t.shape) != tuple(p.shape):
                        raise ValueError(f"{k}: checkpoint shape {tuple(t.shape)} != model {tuple(p.shape)}")
                    p.copy_(t.to(device=p.device, dtype=p.dtype))
                    seen.add(nk)
    missing = [k for k in own if k not in seen and ".lora_" not in k]
    if strict and (missing or unexpected):
        raise RuntimeError(f"load_llava_safetensors: missing {missing[:5]}..., unexpected {unexpected[:5]}...")
    return missing, unexpected


# ---------------------------------------------------------------------------------------------
# CuLLaVO save format
# ---------------------------------------------------------------------------------------------
def _adapter_state(model, prefix: str, adapter: str) -> dict:
    out = {}
    for k, p in model.arenas["lora"].params.items():
        if k.startswith(prefix):
            out[PEFT_PREFIX + k[len(prefix):].replace(f".{adapter}.", ".")] = p.detach().to("cpu").contiguous()
    return out


def _adapter_config(s, targets, layers=None) -> dict:
    cfg = {"peft_type": "LORA", "task_type": "CAUSAL_LM", "r": s.r, "lora_alpha": s.lora_alpha,
           "lora_dropout": s.lora_dropout, "bias": "none", "target_modules": list(targets),
           "inference_mode": False, "fan_in_fan_out": False, "init_lora_weights": True}
    if layers is not None:
        cfg["layers_to_transform"] = list(layers)
    return cfg


def save_cullavo(model, save_dir: str, epoch: int, is_main_process: bool = True):
    """reference modeling/BaseModel.py:20-69 (the LLM branch: LOAD_LLM=True)."""
    if not is_main_process:
        return
    from safetensors.torch import save_file

    from .lora import LM_TARGETS, VISION_TARGETS
    uncovered = [n for n, a in model.arenas.items() if a.trainable and n not in COVERED_ARENAS]
    if uncovered:
        raise RuntimeError(f"save_cullavo: trainable arenas {uncovered} have no place in the save format")
    root = os.path.join(save_dir, f"epoch{epoch}")
    cul = os.path.join(root, "cullavo")
    os.makedirs(cul, exist_ok=True)
    # every parameter of the wrapper lives under cullavo_model.*, which :25 filters out
    torch.save({}, os.path.join(root, "CuLLaVO.pt"))
    s = getattr(model, "lora_settings", None)
    if s is not None and "lora" in model.arenas:
        for sub, prefix, targets, layers in (("vision_tower", VISION_PREFIX, VISION_TARGETS, s.vision_layers),
                                             ("language_model", LM_PREFIX, LM_TARGETS, None)):
            d = os.path.join(cul, sub)
            os.makedirs(d, exist_ok=True)
            save_file(_adapter_state(model, prefix, s.adapter), os.path.join(d, "adapter_model.safetensors"))
            with open(os.path.join(d, "adapter_config.json"), "w") as f:
                json.dump(_adapter_config(s, targets, layers), f, indent=2)

    def sub_state(arena, strip):
        return {k[len(strip):]: p.detach().to("cpu").clone() for k, p in model.arenas[arena].params.items()}

    torch.save(sub_state("projector", "multi_modal_projector."), os.path.join(cul, "multi_modal_projector.pt"))
    torch.save(sub_state("head", "language_model.lm_head."), os.path.join(cul, "lm_head.pt"))
    torch.save(sub_state("embed", "language_model.model.embed_tokens."), os.path.join(cul, "embed_tokens.pt"))
    for arena, (sub, prefix) in TOWER_ARENAS.items():
        if arena in model.arenas and model.arenas[arena].trainable:
            d = os.path.join(cul, sub)
            os.makedirs(d, exist_ok=True)
            save_file({k[len(prefix):]: p.detach().to("cpu").contiguous() for k, p in model.arenas[arena].params.items()},
                      os.path.join(d, "model.safetensors"))


def _copy_into(params: dict, state: dict, prefix: str, what: str):
    with torch.no_grad():
        for k, v in state.items():
            key = prefix + k
            if key not in params:
                raise KeyError(f"{what}: unexpected key {k}")
            params[key].copy_(v.to(device=params[key].device, dtype=params[key].dtype))
    missing = [k for k in params if k.startswith(prefix) and k[len(prefix):] not in state]
    if missing:
        raise KeyError(f"{what}: missing {missing[:3]}")


def load_cullavo(model, load_dir: str):
    """reference modeling/BaseModel.py:71-136: load_dir is .../epoch{e}/CuLLaVO.pt; the cullavo/
    directory next to it carries the adapters and the trainable non-LoRA modules."""
    from safetensors import safe_open
    base = os.path.dirname(load_dir)
    cul = os.path.join(base, "cullavo")
    if os.path.isdir(cul):
        s = getattr(model, "lora_settings", None)
        if s is not None and "lora" in model.arenas:
            lp = model.arenas["lora"].params
            for sub, prefix in (("vision_tower", VISION_PREFIX), ("language_model", LM_PREFIX)):
                f = os.path.join(cul, sub, "adapter_model.safetensors")
                with safe_open(f, framework="pt", device="cpu") as h, torch.no_grad():
                    for k in h.keys():
                        if "lora" not in k:
                            continue
                        rel = k[len(PEFT_PREFIX):] if k.startswith(PEFT_PREFIX) else k
                        key = prefix + rel
                        if key not in lp:  # peft-saved keys drop the adapter name
                            key = prefix + rel.replace(".lora_A.", f".lora_A.{s.adapter}.").replace(
                                ".lora_B.", f".lora_B.{s.adapter}.")
                        if key not in lp:
                            raise KeyError(f"adapter key {k} matches no LoRA parameter")  # reference: "No!"
                        lp[key].copy_(h.get_tensor(k).to(device=lp[key].device, dtype=lp[key].dtype))
        ld = dict(weights_only=True, map_location="cpu")
        _copy_into(model.arenas["projector"].params, torch.load(os.path.join(cul, "multi_modal_projector.pt"), **ld),
                   "multi_modal_projector.", "multi_modal_projector")
        _copy_into(model.arenas["head"].params, torch.load(os.path.join(cul, "lm_head.pt"), **ld),
                   "language_model.lm_head.", "lm_head")
        _copy_into(model.arenas["embed"].params, torch.load(os.path.join(cul, "embed_tokens.pt"), **ld),
                   "language_model.model.embed_tokens.", "embed_tokens")
        for arena, (sub, prefix) in TOWER_ARENAS.items():
            f = os.path.join(cul, sub, "model.safetensors")
            if os.path.exists(f) and arena in model.arenas:
                params = model.arenas[arena].params
                with safe_open(f, framework="pt", device="cpu") as h, torch.no_grad():
                    keys = set(h.keys())
                    for k in keys:
                        if prefix + k not in params:
                            raise KeyError(f"{sub}/model.safetensors: unexpected key {k}")
                        params[prefix + k].copy_(h.get_tensor(k).to(device=params[prefix + k].device,
                                                                    dtype=params[prefix + k].dtype))
                missing = [k for k in params if k[len(prefix):] not in keys]
                if missing:
                    raise KeyError(f"{sub}/model.safetensors: missing {missing[:3]}")
                model.arenas[arena].note_written()
    rest = torch.load(load_dir, weights_only=True, map_location="cpu")
    if rest:
        model.load_state_dict({normalize_llava_key(k.split("cullavo_model.", 1)[-1]): v for k, v in rest.items()},
                              strict=False)
    return model
