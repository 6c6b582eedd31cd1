"""Synthetic, pre-tokenised CuLLaVO batches (SURVEY.md §8(d) recipes).

The reference builds each batch on the CPU from COCO/ShareGPT4V images with detectron2 drawing,
the llava tokenizer and CLIPImageProcessor (reference cullavo/arch_cullavo.py:96-339, 397-543;
out of scope: real tokenizer/images are unavailable offline). What reaches the hot path is
fixed tensors: input_ids [B, S] with one <image> id per row, attention_mask, pixel_values
[B, 3, 336, 336] and labels at the merged length [B, S + P - 1] (-100 on the prompt).
Batches are generated directly in HBM so the timed step starts with resident inputs.
"""
from __future__ import annotations

import torch

from .config import CuLLaVOConfig


def synthetic_batch(cfg: CuLLaVOConfig, batch: int, text_len: int = 513, image_col: int = 35, *,
                    label_from: int | None = None, seed: int = 1234, device="cuda"):
    """Config-3 recipe: BOS at 0, <image> at image_col, text U[2, image_token); pixels N(0,1);
    labels = next-token ids for merged positions >= label_from (default: 611 at the 7B shapes,
    i.e. the prompt + image block is masked), -100 before."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    v = cfg.vision_config
    P = v.num_patches
    ids = torch.randint(2, cfg.image_token_index, (batch, text_len), generator=g, device=device)
    ids[:, 0] = 1
    ids[:, image_col] = cfg.image_token_index
    mask = torch.ones_like(ids)
    pix = torch.randn(batch, v.num_channels, v.image_size, v.image_size, generator=g, device=device)
    L = text_len + P - 1
    if label_from is None:  # -100 for merged positions < image_col + P (611 at 7B)
        label_from = min(L - 1, image_col + P)
    labels = torch.full((batch, L), cfg.ignore_index, dtype=torch.long, device=device)
    labels[:, label_from:] = torch.randint(2, cfg.image_token_index, (batch, L - label_from), generator=g,
                                           device=device)
    return {"input_ids": ids, "attention_mask": mask, "pixel_values": pix, "labels": labels}


class SyntheticLoader:
    """A fixed-length iterable of synthetic batches (stands in for build_train_dataloader,
    reference datasets/build.py:354-409); rank-sharded by seed like accel.prepare would."""

    def __init__(self, cfg: CuLLaVOConfig, batch: int, steps: int, *, text_len: int = 513, image_col: int = 35,
                 rank: int = 0, device="cuda", seed: int = 1234, reuse: bool = True):
        self.cfg, self.batch, self.steps = cfg, batch, steps
        self.kw = dict(text_len=text_len, image_col=image_col, device=device)
        self.seed = seed + rank
        self.reuse = reuse
        self._fixed = None

    def __len__(self):
        return self.steps

    def __iter__(self):
        for i in range(self.steps):
            if self.reuse:
                if self._fixed is None:
                    self._fixed = synthetic_batch(self.cfg, self.batch, seed=self.seed, **self.kw)
                yield self._fixed
            else:
                yield synthetic_batch(self.cfg, self.batch, seed=self.seed + 1000 * i, **self.kw)
