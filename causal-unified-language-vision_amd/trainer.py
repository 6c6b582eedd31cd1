"""Trainer shell: drop-in for CuLLaVO_Trainer / DefaultTrainer / DistributedTrainer
(reference trainer/cullavo_trainer.py:11-14, trainer/default_trainer.py:24-197,
trainer/distributed_trainer.py:13-64) on one process per GPU.

Differences by design (SURVEY.md §8(e), §5 "Distributed comm backend"):
 * gradients are averaged across ranks (bucketed RCCL all-reduce overlapped with backward,
   dist.GradReducer) — the reference's DDP-then-unwrap most likely never reduced them;
 * no per-step barrier or empty_cache (reference pipeline/CuLLaVOPipeline.py:87,
   trainer/default_trainer.py:177), no per-step .item() unless logging asks for it;
 * AdamW + clip run fused on device (optim.FusedAdamW).
"""
from __future__ import annotations

import contextlib
import datetime
import math
import os

import torch
import torch.distributed as dist

from .dist import GradReducer
from .optim import FusedAdamW

DEFAULT_OPT = {
    "NAME": "cullavo_step1.yaml",
    "PIPELINE": "CuLLaVOPipeline",
    "OPTIMIZER": {"LR": 2e-5, "LAST_LR": 1e-6, "WEIGHT_DECAY": 0.0, "EPOCH": 1, "GRAD_MAX": 10.0, "GRAD_CUM": 1,
                  "PERIOD": 4},
    "LLM": {"LOAD_LLM": True, "TRAINABLE": "full"},
    "MODEL": {"NAME": "cullavo_model", "CONFIG": "llava-1.5-7b"},
    "DATA": {"BATCH_SIZE_PER_GPU": 8, "TEXT_LEN": 513, "IMAGE_COL": 35, "STEPS": 10},
}


def _merge(a: dict, b: dict) -> dict:
    out = dict(a)
    for k, v in (b or {}).items():
        out[k] = _merge(out[k], v) if isinstance(v, dict) and isinstance(out.get(k), dict) else v
    return out


class Accel:
    """The subset of accelerate.Accelerator the reference calls (device, backward,
    wait_for_everyone, clip_grad_norm_, accumulate, sync_gradients, process flags)."""

    def __init__(self, grad_accum: int = 1):
        self.distributed = dist.is_available() and dist.is_initialized()
        self.num_processes = dist.get_world_size() if self.distributed else 1
        self.process_index = dist.get_rank() if self.distributed else 0
        self.local_process_index = int(os.environ.get("LOCAL_RANK", 0))
        self.device = torch.device("cuda", local_device_index()) if torch.cuda.is_available() else \
            torch.device("cpu")
        self.is_main_process = self.process_index == 0
        self.is_local_main_process = self.local_process_index == 0
        self.gradient_accumulation_steps = grad_accum
        self._micro = 0
        self.sync_gradients = True
        self.optimizer: FusedAdamW | None = None
        self.reducer: GradReducer | None = None

    def backward(self, loss):
        loss.backward()
        if self.sync_gradients and self.reducer is not None:
            self.reducer.finish()

    def wait_for_everyone(self):
        if self.distributed:
            dist.barrier()

    def clip_grad_norm_(self, parameters, max_norm):
        return self.optimizer.clip_grad_norm_(max_norm)

    @contextlib.contextmanager
    def accumulate(self, model=None):
        self._micro += 1
        self.sync_gradients = self._micro % self.gradient_accumulation_steps == 0
        if self.reducer is not None:
            self.reducer.enabled = self.sync_gradients and self.reducer.world > 1
        yield


def local_device_index() -> int:
    """LOCAL_RANK's GPU; more ranks than GPUs (a gloo rehearsal of the DP path on one GPU) share
    the GPUs round-robin."""
    return int(os.environ.get("LOCAL_RANK", 0)) % max(torch.cuda.device_count(), 1)


def init_distributed(backend: str | None = None):
    """One process per GPU from torchrun's env (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_*)."""
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) > 1 and not dist.is_initialized():
        if torch.cuda.is_available():
            torch.cuda.set_device(local_device_index())
        backend = backend or os.environ.get("CULLAVO_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        dist.init_process_group(backend, timeout=datetime.timedelta(seconds=18000))  # :16 of the ref


class DefaultTrainer:
    def __init__(self, opt: dict | None = None):
        self.opt = _merge(DEFAULT_OPT, opt or {})
        init_distributed(self.opt.get("DIST_BACKEND"))
        self.accel = Accel(int(self.opt["OPTIMIZER"]["GRAD_CUM"]))
        self.opt["world_size"] = self.accel.num_processes
        self.opt["rank"] = self.accel.process_index
        from .pipeline import CuLLaVOPipeline
        self.pipeline = CuLLaVOPipeline(self.opt)
        self.train_params = {"optim_steps": 0}

    # reference trainer/default_trainer.py:74-90
    def compute_loss(self, forward_func, batch):
        return forward_func(self, batch)

    def backward_loss(self, loss):
        self.accel.backward(loss)

    def update_model(self):
        self.optimizer.step()
        self.optimizer.zero_grad()
        self.train_params["optim_steps"] += 1
        self.lr_scheduler.step()

    def train_step(self, batch):
        self.model.train()
        return self.pipeline.forward_step(self, batch)

    def init_train(self):
        self.model = self.pipeline.initialize_model()
        self.train_dataloaders = self.pipeline.get_dataloaders(self, "train", is_evaluation=False)
        self.create_optimizer_and_scheduler()
        self._initialize_accelerator()

    def _initialize_accelerator(self):
        cm = self.model.cullavo_model if hasattr(self.model, "cullavo_model") else self.model
        arenas = [a for a in cm.arenas.values() if a.trainable]
        order = ["head", "layers", "lora", "embed", "projector", "vision"]
        arenas.sort(key=lambda a: order.index(a.name))
        self.accel.optimizer = self.optimizer
        if self.accel.num_processes > 1:
            self.broadcast_parameters(cm)
            self.accel.reducer = GradReducer(arenas, bucket_bytes=int(self.opt.get("BUCKET_MB", 256)) << 20)

    @staticmethod
    def broadcast_parameters(cm):
        """identical replicas at start (one RCCL broadcast per arena from rank 0)"""
        for ar in cm.arenas.values():
            dist.broadcast(ar.flat, src=0)
            ar.note_written()

    def eval(self):
        """reference trainer/default_trainer.py:51-71: build the model, optionally load a CuLLaVO
        checkpoint (opt['WEIGHT'] + opt['RESUME_FROM'] = .../epochN/CuLLaVO.pt) and run the
        pipeline's evaluate_model (step-2-pre generation, gathered across ranks)."""
        self.mode = "eval"
        self.model = self.pipeline.initialize_model()
        if self.opt.get("WEIGHT") and os.path.isfile(self.opt.get("RESUME_FROM", "")):
            self.model.from_pretrained(self.opt["RESUME_FROM"], self.accel)
        proc = self.opt.get("PROCESSOR")
        if proc is not None:
            self.model.model.cullavo_processor = proc
        return self.pipeline.evaluate_model(self)

    def train(self):
        self.init_train()
        n_ep = int(self.opt["OPTIMIZER"]["EPOCH"])
        losses = []
        for epoch in range(n_ep):
            for batch in self.train_dataloaders:
                with self.accel.accumulate(self.model):
                    info, _, _ = self.train_step(batch)
                losses.append(info["loss_llm"])
        self.optimizer.synchronize()
        return losses


class CuLLaVO_Trainer(DefaultTrainer):
    def create_optimizer_and_scheduler(self):
        """reference trainer/cullavo_trainer.py:12-14: AdamW(lr, wd) + CosineAnnealingLR."""
        o = self.opt["OPTIMIZER"]
        cm = self.model.cullavo_model if hasattr(self.model, "cullavo_model") else self.model
        # OVERLAP: the update runs on a side stream under the next step's forward (optim.py). Off by
        # default since round 3: the HBM-bound update kernels refill every CU they touch, so the
        # 8-wave GEMMs (one whole-CU workgroup each) of the next forward starve beside them and
        # the step gains nothing (config 3: 351.5 / 352.4 ms with, 351.7 / 351.7 without,
        # alternating on one box; the ViT GEMMs ran at 138 TF/s beside it, 380 without).
        self.optimizer = FusedAdamW(list(cm.arenas.values()), lr=float(o["LR"]), weight_decay=float(o["WEIGHT_DECAY"]),
                                    overlap=bool(o.get("OVERLAP", False)))
        self.lr_scheduler = torch.optim.lr_scheduler.CosineAnnealingLR(
            optimizer=self.optimizer, T_max=max(1, len(self.train_dataloaders) * int(o["EPOCH"])),
            eta_min=float(o["LAST_LR"]))


def cosine_lr(step: int, total: int, lr: float, last_lr: float) -> float:
    return last_lr + (lr - last_lr) * (1 + math.cos(math.pi * step / max(1, total))) / 2
