"""Deterministic stand-in for the llava-1.5 tokenizer (the real one is unavailable offline).

Words are whitespace-delimited; '<image>' -> 32000, '</s>' -> 2, BOS 1 with special tokens,
pad 32001; other words hash (crc32) into [3, 31993). Used by tests/golden/make_golden_data.py
(through the REFERENCE's prompt builders) and by tests/test_prompting.py (through ours), so the
fixtures pin label / padding logic, not the tokenizer.
"""
from __future__ import annotations

import re
import zlib
from types import SimpleNamespace

import torch


class ToyTokenizer:
    pad_token_id = 32001
    bos_token_id = 1
    eos_token_id = 2
    image_token_id = 32000

    def __init__(self, padding_side: str = "right"):
        self.padding_side = padding_side

    def encode(self, text: str, add_special_tokens: bool = True) -> list[int]:
        ids = [self.bos_token_id] if add_special_tokens else []
        for part in re.split(r"(<image>|</s>)", text):
            if part == "<image>":
                ids.append(self.image_token_id)
            elif part == "</s>":
                ids.append(self.eos_token_id)
            else:
                ids += [3 + zlib.crc32(w.encode()) % 31990 for w in part.split()]
        return ids

    def __call__(self, text, return_tensors="pt", add_special_tokens=True, **kw):
        return SimpleNamespace(input_ids=torch.tensor([self.encode(text, add_special_tokens)], dtype=torch.long))
