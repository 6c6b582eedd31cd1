"""CuLLaVOModel: drop-in for the reference's model class (reference cullavo/arch_cullavo.py:24,
546-677) whose dense math runs on the gfx950 kernels.

Same constructor-visible structure (.vision_tower, .multi_modal_projector, .language_model with
.model/.lm_head, .get_input_embeddings(), .config), same forward signature, same
CullavoCausalLMOutputWithPast result (tuple form when return_dict=False) and the same
ValueError for an unknown vision_feature_select_strategy.
"""
from __future__ import annotations

from dataclasses import dataclass, fields
from typing import Optional, Tuple

import torch
from torch import nn

from . import ops
from .config import CuLLaVOConfig
from .functions import HeadLossFn, MergeFn, StepContext
from .lora import LoraSettings
from .modeling import (CLIPVisionModel, LlamaForCausalLM, LlavaMultiModalProjector, build_arenas, init_random_)


@dataclass
class CullavoCausalLMOutputWithPast:
    """reference cullavo/arch_cullavo.py:14-21"""
    loss: Optional[torch.Tensor] = None
    logits: torch.Tensor = None
    past_key_values: Optional[list] = None
    hidden_states: Optional[Tuple[torch.Tensor]] = None
    attentions: Optional[Tuple[torch.Tensor]] = None
    image_hidden_states: Optional[Tuple[torch.Tensor]] = None

    def __getitem__(self, k):
        if isinstance(k, str):
            return getattr(self, k)
        return self.to_tuple()[k]

    def to_tuple(self):
        return tuple(getattr(self, f.name) for f in fields(self) if getattr(self, f.name) is not None)


class CuLLaVOModel(nn.Module):
    def __init__(self, config: CuLLaVOConfig, *, device="cuda", trainable: str = "full", init: str = "random",
                 seed: int = 0, lora: LoraSettings | None = None, dtype=torch.bfloat16):
        """trainable: "full" | "reference" | "lora" | "none" (modeling.TRAINABLE_POLICIES); "lora"
        adds the reference's peft adapters (lora.LoraSettings, default r=64, alpha=16, p=0.05).
        dtype: torch.bfloat16 (production: the reference's bf16-cast model under bf16 autocast,
        reference cullavo/load_cullavo.py:123-126) or torch.float32 (the parity mode: every
        parameter, activation and kernel operand f32, nothing rounded to bf16)."""
        if dtype not in (torch.bfloat16, torch.float32):
            raise ValueError(f"dtype {dtype}: bf16 (production) or float32 (parity mode)")
        super().__init__()
        self.dtype = dtype
        if config.vision_config.hidden_act != "quick_gelu" or config.projector_hidden_act != "gelu":
            raise ValueError("CuLLaVO path: CLIP quick_gelu + projector gelu")
        self.config = config
        if trainable == "lora" and lora is None:
            lora = LoraSettings()
        self.lora_settings = lora if trainable == "lora" else None
        self.arenas = build_arenas(config, device, trainable, dtype=dtype, lora=self.lora_settings)
        if init == "random":
            init_random_(self.arenas, seed)
        la = (self.arenas["lora"], self.lora_settings) if "lora" in self.arenas else None
        self.vision_tower = CLIPVisionModel(config.vision_config, self.arenas["vision"], la)
        self.multi_modal_projector = LlavaMultiModalProjector(self.arenas["projector"].params)
        self.language_model = LlamaForCausalLM(config.text_config, self.arenas["embed"], self.arenas["layers"],
                                               self.arenas["head"], la)
        self.trainable_policy = trainable

    @classmethod
    def from_pretrained(cls, path: str, *, device="cuda", trainable: str = "full", lora: LoraSettings | None = None,
                        **kw) -> "CuLLaVOModel":
        """llava-hf checkpoint directory (config.json + *.safetensors, ~4.37 or >= 4.45 key
        layout) -> model, streamed into HBM (reference cullavo/load_cullavo.py:86)."""
        from .checkpoint import load_llava_safetensors
        m = cls(CuLLaVOConfig.from_json(path), device=device, trainable=trainable, init="none", lora=lora)
        if "lora" in m.arenas:
            from .lora import init_lora_
            init_lora_(m.arenas["lora"], kw.get("seed", 0))
        load_llava_safetensors(m, path)
        return m

    # -- reference API -------------------------------------------------------------------------
    # ---- data step (reference cullavo/arch_cullavo.py:28-339, 397-543) ----
    @staticmethod
    def make_system_prompt(processor, device, ignore_index):
        from .prompting import make_system_prompt
        return make_system_prompt(processor, device, ignore_index)

    @staticmethod
    def make_and_add_prompt_and_label(cullavo_prompt, cullavo_label, prompt, answer, processor, device, ignore_index):
        from .prompting import make_and_add_prompt_and_label
        return make_and_add_prompt_and_label(cullavo_prompt, cullavo_label, prompt, answer, processor, device,
                                             ignore_index)

    def step1_process(self, inputs, processor, device, fix_num=5):
        """reference cullavo/arch_cullavo.py:96-339 (prompting.step1_process; boxes drawn on the GPU)"""
        from .prompting import step1_process
        return step1_process(inputs, processor, device, self.config.ignore_index, fix_num)

    def step2_process(self, batched_inputs, processor, device):
        from .prompting import step2_process
        return step2_process(batched_inputs, processor, device, self.config.ignore_index,
                             self.config.vision_config.image_size)

    def step2_preprocess(self, batched_inputs, processor, device, **kw):
        """reference cullavo/arch_cullavo.py:341-395 (prompting.step2_preprocess, on generate())"""
        from .prompting import step2_preprocess
        return step2_preprocess(self, batched_inputs, processor, device, **kw)

    def eval_process(self, images, aux_prompt=None, prompt=None, processor=None, device=None):
        from .prompting import eval_process
        return eval_process(images, aux_prompt, prompt, processor, device, self.config.ignore_index)

    def get_input_embeddings(self):
        return self.language_model.model.embed_tokens

    def get_output_embeddings(self):
        return self.language_model.lm_head

    def to(self, *a, **k):  # parameters are views into HBM arenas: moving would break them
        raise RuntimeError("CuLLaVOModel lives where it was built (pass device= to the constructor)")

    def zero_grad(self, set_to_none: bool = False):
        for ar in self.arenas.values():
            ar.zero_grad()

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        """Load llava-hf (transformers ~4.37) keys; copies into the arenas in place. peft-wrapped
        keys (`<linear>.base_layer.weight`) map to the base weight."""
        own = {}
        for ar in self.arenas.values():
            own.update(ar.params)
        state_dict = {k.replace(".base_layer.", "."): v for k, v in state_dict.items()}
        missing = [k for k in own if k not in state_dict]
        unexpected = [k for k in state_dict if k not in own]
        if strict and (missing or unexpected):
            raise RuntimeError(f"load_state_dict: missing {missing[:5]}..., unexpected {unexpected[:5]}...")
        with torch.no_grad():
            for k, v in state_dict.items():
                if k in own:
                    own[k].copy_(v.to(own[k].dtype))
        return missing, unexpected

    def state_dict(self, *a, **k):
        out = {}
        for ar in self.arenas.values():
            out.update({key: p.detach() for key, p in ar.params.items()})
        return out

    # -- forward (reference cullavo/arch_cullavo.py:546-677) ------------------------------------
    def forward(self, input_ids=None, pixel_values=None, attention_mask=None, position_ids=None, past_key_values=None,
                inputs_embeds=None, vision_feature_layer=None, vision_feature_select_strategy=None, labels=None,
                use_cache=None, output_attentions=None, output_hidden_states=None, return_dict=None):
        cfg = self.config
        output_hidden_states = output_hidden_states if output_hidden_states is not None else cfg.output_hidden_states
        return_dict = return_dict if return_dict is not None else cfg.use_return_dict
        vision_feature_layer = vision_feature_layer if vision_feature_layer is not None else cfg.vision_feature_layer
        strategy = (vision_feature_select_strategy if vision_feature_select_strategy is not None
                    else cfg.vision_feature_select_strategy)
        if past_key_values is not None or use_cache:
            return self._forward_cached(input_ids, pixel_values, attention_mask, position_ids, past_key_values,
                                        inputs_embeds, vision_feature_layer, strategy, labels, return_dict)
        if output_attentions:
            raise NotImplementedError("flash attention never materialises attention probabilities")

        self.vision_tower.eval()  # :578 (no dropout in this tower; kept for parity of intent)

        if inputs_embeds is None:
            B, S = input_ids.shape
            inputs_embeds = self.get_input_embeddings()(input_ids)  # :582
            if pixel_values is not None and S != 1:
                stats = self._merge_stats_async(input_ids)  # read back while the tower runs
                image_features = self._image_features(pixel_values, vision_feature_layer, strategy)  # :586-599
                inputs_embeds, attention_mask, position_ids = self._merge(image_features, inputs_embeds, input_ids,
                                                                          attention_mask, stats)  # :600-602
                if labels is None:  # :603-604
                    labels = torch.full_like(attention_mask, cfg.ignore_index).to(torch.long)
        B, L, d = inputs_embeds.shape
        if position_ids is None:
            position_ids = torch.arange(L, device=inputs_embeds.device).expand(B, L)
        kv_start = None
        if attention_mask is not None:
            kv_start = (attention_mask.cumsum(-1) == 0).sum(-1).to(torch.int32)
        sctx = StepContext(B, L, position_ids, kv_start)
        lm = self.language_model
        h, hs = lm.decode(inputs_embeds.reshape(B * L, d).contiguous(), sctx, bool(output_hidden_states))  # :638
        loss = None
        if labels is not None:  # :651-665
            if labels.shape != (B, L):  # the reference's masked / shifted indexing raises here
                if attention_mask is not None:
                    raise IndexError(f"The shape of the mask [{B}, {L - 1}] at index 1 does not match the shape of "
                                     f"the indexed tensor [{labels.shape[0]}, {labels.shape[-1] - 1}] at index 1")
                raise ValueError(f"Expected input batch_size ({B * (L - 1)}) to match target batch_size "
                                 f"({labels.shape[0] * (labels.shape[-1] - 1)}).")
            targets = ops.shift_targets(labels, attention_mask, cfg.ignore_index)
            for ar in self.arenas.values():  # final norm / lm_head: pending optimizer updates
                ar.wait_update()
            loss, logits = HeadLossFn.apply(h, lm, targets, cfg.ignore_index, *lm.head_params())
        else:
            for ar in self.arenas.values():
                ar.wait_update()
            logits = lm.lm_head(lm.model.norm(h))
        logits = logits.view(B, L, -1)
        hs_t = tuple(t.view(B, L, d) for t in hs) if hs else None
        if not return_dict:  # :667-669
            out = (logits,) + ((hs_t,) if hs_t is not None else ())
            return (loss,) + out if loss is not None else out
        return CullavoCausalLMOutputWithPast(loss=loss, logits=logits, past_key_values=None, hidden_states=hs_t,
                                             attentions=None)

    # -- KV-cache inference (reference :605-636 and HF generate; generation.py) ------------------
    def _forward_cached(self, input_ids, pixel_values, attention_mask, position_ids, cache, inputs_embeds,
                        vision_feature_layer, strategy, labels, return_dict, max_len: int | None = None):
        from .generation import KVCache, lm_infer
        if cache is not None and not isinstance(cache, KVCache):
            # transformers-layout cache (legacy tuple / DynamicCache, as the reference's decode branch
            # receives it, arch_cullavo.py:605-636): copied once; the KVCache returned in
            # past_key_values indexes like the legacy tuple (cache[layer] -> (key, value) [B,H,L,D])
            cache = KVCache.from_legacy(cache, attention_mask)
        if torch.is_grad_enabled() and any(p.requires_grad for ar in self.arenas.values() for p in ar.params.values()):
            torch.set_grad_enabled(False)  # inference only, as under the reference's torch.inference_mode()
            try:
                return self._forward_cached(input_ids, pixel_values, attention_mask, position_ids, cache,
                                            inputs_embeds, vision_feature_layer, strategy, labels, return_dict,
                                            max_len)
            finally:
                torch.set_grad_enabled(True)
        self.vision_tower.eval()
        first = cache is None or cache.get_seq_length() == 0
        if inputs_embeds is None:
            inputs_embeds = self.get_input_embeddings()(input_ids)
            if first and pixel_values is not None and input_ids.shape[1] != 1:
                image_features = self._image_features(pixel_values, vision_feature_layer, strategy)
                inputs_embeds, attention_mask, position_ids = self._merge(image_features, inputs_embeds, input_ids,
                                                                          attention_mask)
        B, L = inputs_embeds.shape[:2]
        if max_len is None:
            max_len = L + 256
        logits, cache = lm_infer(self.language_model, inputs_embeds, attention_mask, position_ids, cache, max_len)
        out = CullavoCausalLMOutputWithPast(loss=None, logits=logits, past_key_values=cache, hidden_states=None,
                                            attentions=None)
        return out if return_dict else out.to_tuple()

    @torch.no_grad()
    def generate(self, input_ids=None, pixel_values=None, attention_mask=None, max_new_tokens: int = 20,
                 do_sample: bool = False, temperature: float = 1.0, top_k: int = 50, top_p: float = 1.0,
                 eos_token_id: int | None = None, pad_token_id: int | None = None, use_cache: bool = True,
                 generator=None, **kw):
        """Decoder-only generate: returns [B, S + new] (prompt ids then sampled ids), stopping when
        every sequence has produced eos_token_id (finished rows are padded with pad_token_id)."""
        from .generation import sample_next
        if not use_cache:
            raise NotImplementedError("generate() runs on the KV cache (use_cache=True)")
        for ar in self.arenas.values():  # pending optimizer updates (FusedAdamW overlap)
            ar.wait_update()
        cfg = self.config
        pad = pad_token_id if pad_token_id is not None else cfg.pad_token_id
        B, S = input_ids.shape
        if attention_mask is None:
            attention_mask = torch.ones_like(input_ids)
        n_img = int((input_ids == cfg.image_token_index).sum(-1).max()) if pixel_values is not None else 0
        strategy = kw.get("vision_feature_select_strategy", cfg.vision_feature_select_strategy)
        # image feature rows per <image> token: the patches, plus CLS under "full" (:588-597)
        n_feat = cfg.vision_config.num_patches + (1 if strategy == "full" else 0)
        L0 = S + n_img * (n_feat - 1)
        out = self._forward_cached(input_ids, pixel_values, attention_mask, None, None, None,
                                   cfg.vision_feature_layer, strategy, None, True,
                                   max_len=L0 + max_new_tokens)
        cache = out.past_key_values
        logits = out.logits[:, -1]
        finished = torch.zeros(B, dtype=torch.bool, device=input_ids.device)
        new = []
        # the decode steps replay one captured HIP graph (generation.DecodeGraph) unless asked not to
        graph = None
        if kw.get("decode_graph", True) and max_new_tokens > 1 and input_ids.is_cuda:
            from .generation import DecodeGraph
            graph = DecodeGraph(self, cache)
        check_every = 16  # all-finished test every 16 tokens: one host sync per 16 steps, not per step
        for step in range(max_new_tokens):
            tok = sample_next(logits, do_sample=do_sample, temperature=temperature, top_k=top_k, top_p=top_p,
                              generator=generator)
            tok = torch.where(finished, torch.full_like(tok, pad), tok)
            new.append(tok)
            if eos_token_id is not None:
                finished |= tok == eos_token_id
                if (step + 1) % check_every == 0 and bool(finished.all()):
                    break
            if step + 1 == max_new_tokens:
                break
            if graph is not None:
                logits = graph.step(tok)[:, -1]
            else:
                out = self._forward_cached(tok[:, None], None, None, None, cache, None, cfg.vision_feature_layer,
                                           cfg.vision_feature_select_strategy, None, True)
                logits = out.logits[:, -1]
        gen = torch.stack(new, 1)
        if eos_token_id is not None:
            # HF stops at the first step where every row has finished; the steps run past it (at
            # most check_every - 1) hold only padding and are dropped
            done = torch.cumsum((gen == eos_token_id).to(torch.int64), 1) > 0
            all_done = done.all(0)
            if bool(all_done.any()):
                gen = gen[:, :int(all_done.to(torch.int64).argmax()) + 1]
        return torch.cat([input_ids, gen.to(input_ids.dtype)], 1)

    # -- pieces ---------------------------------------------------------------------------------
    def _image_features(self, pixel_values, layer: int, strategy: str):
        vt = self.vision_tower.vision_model
        n = vt.cfg.num_hidden_layers
        idx = n + 1 + layer if layer < 0 else layer
        if not 0 <= idx <= n:
            raise IndexError(f"vision_feature_layer {layer} out of range")
        feats = vt.hidden_state(pixel_values, idx)  # hidden_states[layer], only the layers needed
        if strategy == "default":
            feats = feats[:, 1:]
        elif strategy == "full":
            pass
        else:
            raise ValueError(f"Unexpected select feature strategy: {self.config.vision_feature_select_strategy}")
        return self.multi_modal_projector(feats)

    def _merge_stats_async(self, input_ids):
        """The three integers that size the merge (max image tokens per row, total image
        tokens, rows ending in <pad>), reduced on the GPU and copied to pinned host memory
        without waiting: the copy completes long before the vision tower enqueued behind it,
        so the host read in _merge does not drain the GPU queue."""
        cfg = self.config
        is_img = input_ids == cfg.image_token_index
        st = torch.stack([is_img.sum(-1).max(), is_img.sum(), (input_ids[:, -1] == cfg.pad_token_id).sum()])
        host = torch.empty(3, dtype=st.dtype, pin_memory=True)
        host.copy_(st, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        return host, ev

    def _merge(self, image_features, inputs_embeds, input_ids, attention_mask, stats=None):
        """transformers ~4.37 _merge_input_ids_with_image_features on the merge_plan kernel.
        One small device->host read (image-token counts, left-padding flag) sizes the output,
        as the reference's .max() / torch.where do."""
        cfg = self.config
        n_img, P, d = image_features.shape
        B, S = input_ids.shape
        host, ev = stats if stats is not None else self._merge_stats_async(input_ids)
        ev.synchronize()
        n_max, n_total, n_pad_last = (int(x) for x in host.tolist())
        if n_total != n_img:
            raise ValueError(f"The input provided to the model are wrong. The number of image tokens is {n_total} "
                             f"while the number of image given to the model is {n_img}. This prevents correct "
                             f"indexing and breaks batch generation.")
        left_padding = n_pad_last == 0
        L = n_max * (P - 1) + S
        if attention_mask is None:
            attention_mask = torch.ones_like(input_ids)
        text_dst, src, mmask, pos = ops.merge_plan(input_ids, attention_mask, L=L, image_token=cfg.image_token_index,
                                                   n_patches=P, left_padding=left_padding)
        n_text = B * S
        flat = src.reshape(-1)
        rows = torch.arange(B * L, device=flat.device)
        is_img_row = flat >= n_text
        img_dst = torch.empty(n_img * P + 1, dtype=torch.int64, device=flat.device)
        img_dst.scatter_(0, torch.where(is_img_row, flat - n_text, n_img * P), rows)
        merged = MergeFn.apply(inputs_embeds.reshape(n_text, d), image_features.reshape(n_img * P, d), flat,
                               text_dst, img_dst[:-1])
        return merged.view(B, L, d), mmask, pos


def build_cullavo(config: CuLLaVOConfig | None = None, **kw) -> CuLLaVOModel:
    from .config import llava_1_5_7b
    return CuLLaVOModel(config or llava_1_5_7b(), **kw)
