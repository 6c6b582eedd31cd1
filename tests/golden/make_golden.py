"""Generate the golden fixtures that pin the CPU oracle to the REFERENCE's own forward.

Runs in the build container only (it reads /root/reference; nothing here travels to the GPU
box). It imports the reference's ``CuLLaVOModel`` (reference cullavo/arch_cullavo.py:24) and
calls its ``forward`` (:546-677) UNMODIFIED, through the compat shim described in SURVEY.md
§8(c):

* ``detectron2`` (imported at arch_cullavo.py:12 for prompt drawing only) is stubbed;
* transformers 5.15 nests the towers under ``.model``: ``vision_tower`` /
  ``multi_modal_projector`` properties forward there, and ``language_model`` becomes a view
  that runs the LlamaModel then ``lm_head`` and upcasts logits to f32 (4.37 behaviour);
* ``_merge_input_ids_with_image_features`` (transformers ~4.37, absent from 5.15) is restated
  here as an independent per-row loop (the oracle's version is vectorised; the fixtures
  cross-check the two);
* ``config.ignore_index = -100``.

Weights come from oracle.make_weights (seeded by key name) and are loaded into the HF modules
by key (4.37 names -> 5.15 names); inputs from oracle.make_inputs. Outputs are stored as
float32 .npz (each file < 1 MB): loss, sampled logits rows, a few full gradients and
summary norms of the rest.

Usage: python tests/golden/make_golden.py
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)

from oracle import cullavo_oracle as O  # noqa: E402


def _stub_detectron2():
    for name in ["detectron2", "detectron2.utils", "detectron2.utils.visualizer", "detectron2.data",
                 "detectron2.structures", "detectron2.utils.comm", "detectron2.data.detection_utils"]:
        m = types.ModuleType(name)
        sys.modules.setdefault(name, m)
    sys.modules["detectron2.utils.visualizer"].Visualizer = type("Visualizer", (), {})


def _import_reference():
    _stub_detectron2()
    sys.path.insert(0, REF)
    # the reference's top-level utils package pulls dataset/prompt helpers; only
    # utils.constants is needed by arch_cullavo (COCO_PANOPTIC_CLASSES)
    utils_pkg = types.ModuleType("utils")
    utils_pkg.__path__ = [os.path.join(REF, "utils")]
    sys.modules["utils"] = utils_pkg
    from cullavo.arch_cullavo import CuLLaVOModel  # noqa: E402
    return CuLLaVOModel


def merge_loop(self, image_features, inputs_embeds, input_ids, attention_mask, labels):
    """transformers ~4.37 _merge_input_ids_with_image_features, restated row by row."""
    cfg = self.config
    n_img, P, D = image_features.shape
    B, S = input_ids.shape
    pad = cfg.pad_token_id
    left_padding = not bool((input_ids[:, -1] == pad).sum())
    n_special = [int((input_ids[b] == cfg.image_token_index).sum()) for b in range(B)]
    L = max(n_special) * (P - 1) + S
    emb = torch.zeros(B, L, D, dtype=inputs_embeds.dtype)
    mask = torch.zeros(B, L, dtype=attention_mask.dtype)
    is_text_slot = torch.zeros(B, L, dtype=torch.bool)
    for b in range(B):
        pos, positions = -1, []
        for s in range(S):
            pos += P if int(input_ids[b, s]) == cfg.image_token_index else 1
            positions.append(pos)
        nb_pad = L - 1 - positions[-1]
        for s in range(S):
            if int(input_ids[b, s]) == cfg.image_token_index:
                continue
            p = positions[s] + (nb_pad if left_padding else 0)
            emb[b, p] = inputs_embeds[b, s]
            mask[b, p] = attention_mask[b, s]
            is_text_slot[b, p] = True
        cnt = 0
        for l in range(L):
            if not is_text_slot[b, l]:
                cnt += 1
                if cnt - 1 < nb_pad:
                    is_text_slot[b, l] = True  # excluded: padding slot
    k = 0
    flat = image_features.reshape(-1, D)
    for b in range(B):
        for l in range(L):
            if not is_text_slot[b, l]:
                emb[b, l] = flat[k]
                mask[b, l] = 1
                k += 1
    if k != flat.shape[0]:
        raise ValueError("image token / image count mismatch")
    pos_ids = (mask.cumsum(-1) - 1).masked_fill_(mask == 0, 1)
    return emb, mask, None, pos_ids


def build_reference_model(cfg: O.CuLLaVOCfg, W: dict[str, torch.Tensor]):
    from transformers import CLIPVisionConfig, LlamaConfig, LlavaConfig
    from transformers.modeling_outputs import CausalLMOutputWithPast

    CuLLaVOModel = _import_reference()
    v, t = cfg.vision, cfg.text
    vc = CLIPVisionConfig(hidden_size=v.hidden_size, intermediate_size=v.intermediate_size,
                          num_hidden_layers=v.num_hidden_layers, num_attention_heads=v.num_attention_heads,
                          image_size=v.image_size, patch_size=v.patch_size, hidden_act="quick_gelu",
                          layer_norm_eps=v.layer_norm_eps, projection_dim=t.hidden_size)
    tc = LlamaConfig(hidden_size=t.hidden_size, intermediate_size=t.intermediate_size,
                     num_hidden_layers=t.num_hidden_layers, num_attention_heads=t.num_attention_heads,
                     num_key_value_heads=t.num_attention_heads, vocab_size=t.vocab_size,
                     rms_norm_eps=t.rms_norm_eps, rope_theta=t.rope_theta, max_position_embeddings=4096,
                     tie_word_embeddings=False, pad_token_id=cfg.pad_token_id)
    lc = LlavaConfig(vision_config=vc, text_config=tc, image_token_index=cfg.image_token_index,
                     projector_hidden_act="gelu", vision_feature_layer=cfg.vision_feature_layer,
                     vision_feature_select_strategy=cfg.vision_feature_select_strategy,
                     tie_word_embeddings=False)
    lc.pad_token_id = cfg.pad_token_id
    lc._attn_implementation = "eager"
    vc._attn_implementation = "eager"
    tc._attn_implementation = "eager"

    class LMView:
        def __init__(self, outer):
            self.outer = outer

        def __call__(self, attention_mask=None, position_ids=None, past_key_values=None, inputs_embeds=None,
                     use_cache=None, output_attentions=None, output_hidden_states=None, return_dict=None):
            out = self.outer.model.language_model(attention_mask=attention_mask, position_ids=position_ids,
                                                  inputs_embeds=inputs_embeds, use_cache=False,
                                                  output_hidden_states=output_hidden_states)
            logits = self.outer.lm_head(out.last_hidden_state).float()
            return CausalLMOutputWithPast(logits=logits, past_key_values=None, hidden_states=out.hidden_states)

    class Shim(CuLLaVOModel):
        vision_tower = property(lambda self: self.model.vision_tower)
        multi_modal_projector = property(lambda self: self.model.multi_modal_projector)
        language_model = property(lambda self: LMView(self))
        _merge_input_ids_with_image_features = merge_loop

    model = Shim(lc)
    model.config.ignore_index = O.IGNORE_INDEX
    model.config.pad_token_id = cfg.pad_token_id
    sd = {}
    for k, val in W.items():
        if k.startswith("vision_tower.vision_model."):  # 5.15 drops the vision_model level
            nk = "model.vision_tower." + k[len("vision_tower.vision_model."):]
        elif k.startswith("multi_modal_projector."):
            nk = "model." + k
        elif k == "language_model.lm_head.weight":
            nk = "lm_head.weight"
        elif k.startswith("language_model.model."):
            nk = "model.language_model." + k[len("language_model.model."):]
        else:
            raise KeyError(k)
        sd[nk] = val
    missing, unexpected = model.load_state_dict(sd, strict=False)
    missing = [m for m in missing if "position_ids" not in m]
    assert not missing and not unexpected, (missing, unexpected)
    model.train()
    return model


GRAD_FULL = [
    "multi_modal_projector.linear_2.weight",
    "multi_modal_projector.linear_1.bias",
    "language_model.model.layers.0.self_attn.q_proj.weight",
    "language_model.model.layers.1.mlp.down_proj.weight",
    "language_model.model.norm.weight",
]


def _ref_grad_key(k: str) -> str:
    if k.startswith("vision_tower.vision_model."):
        return "model.vision_tower." + k[len("vision_tower.vision_model."):]
    if k.startswith("multi_modal_projector."):
        return "model." + k
    if k == "language_model.lm_head.weight":
        return "lm_head.weight"
    return "model.language_model." + k[len("language_model.model."):]


def generate(name: str, cfg: O.CuLLaVOCfg, batch: int, text_len: int, image_col: int, seed: int,
             pad_tail=None, grads: bool = True):
    W = O.make_weights(cfg, seed)
    ids, mask, pix, labels = O.make_inputs(cfg, batch, text_len, image_col, seed, pad_tail=pad_tail)
    model = build_reference_model(cfg, W)
    out = model(input_ids=ids, pixel_values=pix, attention_mask=mask, labels=labels, return_dict=True)
    loss, logits = out.loss, out.logits
    rec = {"loss": np.array([loss.item()], np.float32), "logits_shape": np.array(logits.shape, np.int64)}
    L = logits.shape[1]
    rows = np.arange(0, L, max(1, L // 24))
    rec["logits_rows"] = rows.astype(np.int64)
    rec["logits_sample"] = logits[:, rows].detach().numpy().astype(np.float32)
    rec["logits_rownorm"] = logits.detach().norm(dim=-1).numpy().astype(np.float32)
    rec["logits_mean"] = logits.detach().mean(dim=-1).numpy().astype(np.float32)
    if grads:
        loss.backward()
        named = dict(model.named_parameters())
        for k in W:
            g = named[_ref_grad_key(k)].grad
            if g is None:
                continue
            rec["gradnorm/" + k] = np.array([g.norm().item()], np.float32)
            if k in GRAD_FULL:  # large tensors: a fixed-stride sample of the flattened grad
                flat = g.detach().reshape(-1)
                stride = max(1, flat.numel() // 32768)
                rec["grad/" + k] = flat[::stride].numpy().astype(np.float32)
                rec["gradstride/" + k] = np.array([stride], np.int64)
    meta = {"seed": seed, "batch": batch, "text_len": text_len, "image_col": image_col,
            "pad_tail": pad_tail or []}
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **rec, meta=np.array(repr(meta)))
    print(f"{path}: {os.path.getsize(path) / 1024:.0f} KiB, loss={loss.item():.6f}, logits {tuple(logits.shape)}")


def main():
    torch.manual_seed(0)
    c1 = O.config1()
    # config 1: ids [2,32], image at col 5, seed 0
    generate("config1", c1, batch=2, text_len=32, image_col=5, seed=0)
    # right padding (the reference tokenizer pads right: cullavo/load_cullavo.py:140)
    generate("config1_pad", c1, batch=2, text_len=32, image_col=5, seed=1, pad_tail=[0, 7])
    # kernel-shaped small config (head dims 64 / 128) used by the GPU end-to-end parity test
    generate("small_gpu", O.config_small_gpu(), batch=2, text_len=40, image_col=4, seed=2)


if __name__ == "__main__":
    main()
