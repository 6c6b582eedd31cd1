"""CuLLaVOPipeline and the CuLLaVO model wrapper — drop-ins for reference
pipeline/CuLLaVOPipeline.py:26-133 and modeling/architectures/cullavo_model.py:12-214.

The reference's forward_step1/2 first turn raw records into prompts (cullavo/arch_cullavo.py:96-339,
397-543); its eval mode runs the step-2-pre generation (cullavo_model.py:53-58, :73-76 ->
arch_cullavo.py:341-395) through CuLLaVOModel.generate on the KV cache, and evaluate_model gathers
the new entries across ranks (CuLLaVOPipeline.py:95-133). forward_step1 / forward_step2 do the
same here when given raw records and a processor (prompting.step1_process / step2_process:
prompt/label builders, GPU box drawing and GPU image preprocessing); without a processor they take
the already-tokenised tensors the prompt builders would have produced. Both return
{'loss_llm': loss} like the reference.
"""
from __future__ import annotations

import torch
from torch import nn

from .arch_cullavo import CuLLaVOModel
from .config import CuLLaVOConfig, config1, llava_1_5_13b, llava_1_5_7b, tiny_gpu
from .data import SyntheticLoader

MODEL_CONFIGS = {"llava-1.5-7b": llava_1_5_7b, "llava-1.5-13b": llava_1_5_13b, "tiny": tiny_gpu, "config1": config1}
_REGISTRY = {}


def register_model(fn):
    """reference modeling/architectures/build.py: name -> constructor"""
    _REGISTRY[fn.__name__.replace("get_", "")] = fn
    return fn


def build_model(opt):
    return _REGISTRY[opt["MODEL"]["NAME"]](opt)


class CuLLaVO(nn.Module):
    """reference modeling/architectures/cullavo_model.py:12-83"""

    def __init__(self, cfg: dict, cullavo_model: CuLLaVOModel, cullavo_processor=None):
        super().__init__()
        self.cfg = cfg
        self.cullavo_model = cullavo_model
        self.cullavo_processor = cullavo_processor

    @classmethod
    def from_config(cls, cfg: dict, device=None):
        name = cfg["MODEL"].get("CONFIG", "llava-1.5-7b")
        mcfg = name if isinstance(name, CuLLaVOConfig) else MODEL_CONFIGS[name]()
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        m = CuLLaVOModel(mcfg, device=device, trainable=cfg["LLM"].get("TRAINABLE", "full"),
                         seed=int(cfg.get("SEED", 0)))
        return cls(cfg, m)

    def forward(self, batched_inputs, accel=None, mode=None):
        """reference cullavo_model.py:45-58"""
        if self.training:
            if self.cfg["NAME"] == "cullavo_step1.yaml":
                return self.forward_step1(batched_inputs, accel)
            if self.cfg["NAME"] == "cullavo_step2.yaml":
                return self.forward_step2(batched_inputs, accel)
            raise ValueError(f"unknown step config {self.cfg['NAME']}")
        if self.cfg["NAME"] == "cullavo_step2_pre.yaml":
            return self.forward_step2_pre(batched_inputs, accel)
        return self.evaluate_with_llm(batched_inputs, accel)

    def _device(self, accel):
        return accel.device if accel is not None else torch.device("cuda", torch.cuda.current_device())

    def forward_step2_pre(self, batched_inputs, accel=None, **kw):
        """reference cullavo_model.py:73-76: lbk records -> new lbk.json entries (generation)"""
        if self.cullavo_processor is None:
            raise ValueError("step-2-pre generation needs a CuLLaVOProcessor (tokenizer)")
        return self.cullavo_model.step2_preprocess(batched_inputs, self.cullavo_processor, self._device(accel), **kw)

    def evaluate_with_llm(self, batched_inputs, accel=None, **generate_kwargs):
        """reference cullavo_model.py:85-149: resize the records' images to 336x336, ask for the
        objects and their boxes, generate with the reference's sampling settings and return the
        decoded answers (the reference's version is a debugging scratchpad that overwrites its
        inputs seven times and draws with detectron2; its effective generation is this one,
        per record, with the parsed boxes attached)."""
        import torch.nn.functional as F

        from .prompting import STEP2_PRE_GENERATE, box_and_class_parser
        if self.cullavo_processor is None:
            raise ValueError("evaluation needs a CuLLaVOProcessor (tokenizer)")
        size = self.cullavo_model.config.vision_config.image_size
        dev = self._device(accel)
        gk = dict(STEP2_PRE_GENERATE, **generate_kwargs)
        out = []
        for x in batched_inputs:
            img = F.interpolate(torch.as_tensor(x["image"])[None].float(), size=(size, size))[0]
            inputs = self.cullavo_model.eval_process(
                images=img.round().clamp(0, 255).to(torch.uint8),
                prompt="provide multiple object names with their numbering index and the objects' bounding box "
                       "coordinates in this image.", processor=self.cullavo_processor, device=dev)
            with torch.inference_mode():
                ids = self.cullavo_model.generate(**inputs, **gk)
            text = self.cullavo_processor.batch_decode(ids, skip_special_tokens=True)[0]
            try:
                boxes, classes, flag = box_and_class_parser(text)
            except Exception:
                boxes, classes, flag = None, None, True
            out.append({"text": text, "boxes": None if flag else boxes.tolist(), "classes": None if flag else classes})
        return out

    def forward_step(self, batched_inputs):
        """forward_step1 / forward_step2 (reference :60-83) on pre-tokenised inputs"""
        out = self.cullavo_model(**batched_inputs)
        return {"loss_llm": out.loss}

    def forward_step1(self, batched_inputs, accel=None):
        """reference cullavo_model.py:60-71: detectron2-style records -> step1_process (boxes drawn
        into the images) -> model -> loss; a batch without thing instances gives loss 0"""
        if isinstance(batched_inputs, (list, tuple)):
            if self.cullavo_processor is None:
                raise ValueError("forward_step1 on raw records needs a CuLLaVOProcessor (tokenizer)")
            device = self._device(accel)
            batched_inputs = self.cullavo_model.step1_process(batched_inputs, self.cullavo_processor, device)
            if batched_inputs["input_ids"] is None:
                return {"loss_llm": torch.tensor([0]).to(device)}
        return self.forward_step(batched_inputs)

    def forward_step2(self, batched_inputs, accel=None):
        """reference cullavo_model.py:78-83: records -> step2_process -> model -> loss"""
        if isinstance(batched_inputs, (list, tuple)):
            if self.cullavo_processor is None:
                raise ValueError("forward_step2 on raw records needs a CuLLaVOProcessor (tokenizer)")
            device = accel.device if accel is not None else torch.device("cuda", torch.cuda.current_device())
            batched_inputs = self.cullavo_model.step2_process(batched_inputs, self.cullavo_processor, device)
        return self.forward_step(batched_inputs)


@register_model
def get_cullavo_model(cfg, **kwargs):
    """registered as MODEL.NAME = cullavo_model (reference cullavo_model.py:212-214)"""
    return CuLLaVO.from_config(cfg)


class BaseModel(nn.Module):
    """reference modeling/BaseModel.py:11-18 (checkpoint I/O: SURVEY.md §8(f) row 3)"""

    def __init__(self, opt, module):
        super().__init__()
        self.opt = opt
        self.model = module

    @property
    def cullavo_model(self):
        return self.model.cullavo_model

    def forward(self, *a, **k):
        return self.model(*a, **k)

    def save_pretrained(self, save_dir, epoch, accel):
        """reference modeling/BaseModel.py:20-69 (checkpoint.save_cullavo)"""
        from .checkpoint import save_cullavo
        for ar in self.cullavo_model.arenas.values():  # pending optimizer updates (FusedAdamW overlap)
            ar.wait_update()
        save_cullavo(self.cullavo_model, save_dir, epoch, is_main_process=accel.is_main_process)
        import torch.distributed as dist
        if dist.is_initialized() and dist.get_world_size() > 1:
            dist.barrier()

    def from_pretrained(self, load_dir, accel=None):
        """reference modeling/BaseModel.py:71-136 (checkpoint.load_cullavo)"""
        from .checkpoint import load_cullavo
        load_cullavo(self.cullavo_model, load_dir)
        return self


class CuLLaVOPipeline:
    def __init__(self, opt):
        self._opt = opt

    def initialize_model(self):
        model = build_model(self._opt)
        model.train()
        return BaseModel(self._opt, model)

    def get_dataloaders(self, trainer, dataset_label: str, is_evaluation: bool):
        if is_evaluation:
            return self._eval_loader(trainer, dataset_label)
        if not hasattr(self, "train_loader"):
            d = self._opt["DATA"]
            cm = trainer.model.cullavo_model
            self.train_loader = SyntheticLoader(cm.config, int(d["BATCH_SIZE_PER_GPU"]), int(d["STEPS"]),
                                                text_len=int(d["TEXT_LEN"]), image_col=int(d["IMAGE_COL"]),
                                                rank=int(self._opt.get("rank", 0)), device=trainer.accel.device)
        return self.train_loader

    @staticmethod
    def forward_func(trainer, batch):
        return trainer.model(batch, trainer.accel)

    def forward_step(self, trainer, batch):
        """reference pipeline/CuLLaVOPipeline.py:76-93, without the per-step barrier;
        losses stay on device unless opt['SYNC_LOSS'] asks for host floats."""
        loss = trainer.compute_loss(self.forward_func, batch)
        if self._opt.get("SYNC_LOSS", False):
            loss_info = {k: v.detach().item() for k, v in loss.items()}
        else:
            loss_info = {k: v.detach() for k, v in loss.items()}
        # raw record lists (the reference's collate=list batches, CuLLaVOPipeline.py:85 len(batch))
        # or pre-tokenised tensor dicts
        n = len(batch) if isinstance(batch, (list, tuple)) else int(batch["input_ids"].shape[0])
        sample_size_info = {"num_samples": n}
        total = sum(loss.values())
        if total.requires_grad:
            trainer.backward_loss(total)
            if trainer.accel.sync_gradients:
                cm = trainer.model.cullavo_model
                for ar in cm.arenas.values():
                    ar.finalize_grads()
                trainer.accel.clip_grad_norm_(None, self._opt["OPTIMIZER"]["GRAD_MAX"])
                trainer.update_model()
        return loss_info, sample_size_info, {}

    def _eval_loader(self, trainer, dataset_label: str):
        """lbk records of one evaluation dataset (reference datasets/build.py test loaders over
        register_lbkllava_datasets.py), sharded across ranks like accel.prepare: rank r takes
        records r, r + N, ... in batches of BATCH_SIZE_PER_GPU (lists of record dicts, as the
        reference's collate=list does). opt['DATA']['EVAL_RECORDS'][label] holds the records
        (or a path to an lbk.json, read with prompting.load_lbk_records)."""
        from .prompting import load_lbk_records
        d = self._opt["DATA"]
        src = d.get("EVAL_RECORDS", {}).get(dataset_label)
        if src is None:
            raise KeyError(f"no evaluation records for {dataset_label} (opt['DATA']['EVAL_RECORDS'])")
        recs = load_lbk_records(src, d.get("IMAGE_ROOT")) if isinstance(src, str) else list(src)
        world, rank = trainer.accel.num_processes, trainer.accel.process_index
        mine = recs[rank::world]
        bs = int(d.get("BATCH_SIZE_PER_GPU", 1))
        return [mine[i:i + bs] for i in range(0, len(mine), bs)]

    @staticmethod
    def all_gather(data, world_size):
        """reference pipeline/CuLLaVOPipeline.py:66-69"""
        import torch.distributed as dist
        output = [None for _ in range(world_size)]
        dist.all_gather_object(output, data, group=None)
        return output

    def evaluate_model(self, trainer):
        """reference pipeline/CuLLaVOPipeline.py:95-133: run the eval-mode model (step-2-pre
        generation) over every TEST dataset, all_gather_object the new entries across ranks and
        write them as one JSON list on rank 0 (opt['EVAL_OUTPUT'], default
        <SAVE_DIR>/lbk_new_version.json). Returns the gathered list."""
        import json
        import os
        model = trainer.model.eval()
        out = []
        with torch.no_grad():
            for label in self._opt.get("DATASETS", {}).get("TEST", []):
                for batch in self.get_dataloaders(trainer, label, is_evaluation=True):
                    out.extend(model(batch, accel=trainer.accel))
        trainer.accel.wait_for_everyone()
        world = trainer.accel.num_processes
        if world > 1:
            out = [e for part in self.all_gather(out, world) for e in part]
        if trainer.accel.is_main_process:
            path = self._opt.get("EVAL_OUTPUT") or os.path.join(self._opt.get("SAVE_DIR", "."), "lbk_new_version.json")
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
            with open(path, "w") as f:
                json.dump(out, f)
        trainer.accel.wait_for_everyone()
        return out
