"""CuLLaVOPipeline and the CuLLaVO model wrapper — drop-ins for reference
pipeline/CuLLaVOPipeline.py:26-133 and modeling/architectures/cullavo_model.py:12-214.

The reference's forward_step1/2 first turn raw records into prompts (cullavo/arch_cullavo.py:96-339,
397-543). forward_step2 does the same here when it is given lbk.json records and a processor
(prompting.step2_process: prompt/label builder + GPU image preprocessing); step 1's
detectron2 box drawing is out of scope, so it (like step 2 without a processor) takes the
already-tokenised tensors the prompt builder would have produced. Both return
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
        if self.training:
            if self.cfg["NAME"] == "cullavo_step1.yaml":
                return self.forward_step1(batched_inputs)
            if self.cfg["NAME"] == "cullavo_step2.yaml":
                return self.forward_step2(batched_inputs, accel)
            raise ValueError(f"unknown step config {self.cfg['NAME']}")
        raise NotImplementedError("evaluation / step-2-pre generation needs KV-cache decode (SURVEY.md §8(f) row 2)")

    def forward_step(self, batched_inputs):
        """forward_step1 / forward_step2 (reference :60-83) on pre-tokenised inputs"""
        out = self.cullavo_model(**batched_inputs)
        return {"loss_llm": out.loss}

    forward_step1 = forward_step

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
            raise NotImplementedError("evaluation loaders: SURVEY.md §8(f) rows 2 and 4")
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
        sample_size_info = {"num_samples": int(batch["input_ids"].shape[0])}
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

    def evaluate_model(self, trainer):
        raise NotImplementedError("step-2-pre generation / eval needs KV-cache decode (SURVEY.md §8(f) row 2)")
