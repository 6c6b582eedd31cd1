"""CPU oracle for the data step — TEST INFRASTRUCTURE ONLY.

The checker ``tests/test_imageprep.py`` and ``tests/test_prompting.py`` compare the product
path against; ``cullavo_amd`` never imports it.

* ``resample_coeffs`` / ``pil_resize_bicubic`` — Pillow's separable resampler, restated in
  numpy from libImaging/Resample.c (Pillow is a third-party dependency of the reference's
  transformers image processor; installed here as Pillow 12.2): precompute_coeffs (double),
  bicubic_filter (a = -0.5, support 2), normalize_coeffs_8bpc (22-bit fixed point, round half
  away from zero), ImagingResampleHorizontal_8bpc then ImagingResampleVertical_8bpc with clip8.
  ``Image.resize`` returns a copy when the size is unchanged; the fixed-point passes are the
  identity then too, so the restatement needs no special case.
* ``clip_preprocess`` — transformers' CLIPImageProcessor steps as the reference calls them
  (cullavo/arch_cullavo.py:82,313,516 -> image_transforms: get_resize_output_image_size with
  default_to_square=False, center_crop offsets (orig - crop) // 2, rescale
  float32(float64(u) * scale), normalize float32((x - mean) / std)).
* ``make_system_prompt`` / ``make_and_add_prompt_and_label`` / ``conversation_prompt`` —
  cullavo/arch_cullavo.py:28-61 and the conversation loop of step2_process (:424-436), over a
  tokenizer callable returning token id lists.

Pinning: tests/golden/make_golden_data.py runs transformers' CLIPImageProcessorPil (and through
it Pillow) on seeded images, and the REFERENCE's own make_system_prompt /
make_and_add_prompt_and_label / step2_process (imported from /root/reference with the
detectron2 stub of make_golden.py) over a deterministic toy tokenizer; the outputs are
committed under tests/golden/ and tests/test_imageprep.py / tests/test_prompting.py check this
restatement against them.
"""
from __future__ import annotations

import math

import numpy as np

PRECISION_BITS = 32 - 8 - 2
OPENAI_CLIP_MEAN = (0.48145466, 0.4578275, 0.40821073)
OPENAI_CLIP_STD = (0.26862954, 0.26130258, 0.27577711)


def _bicubic(x: float) -> float:
    """Pillow Resample.c bicubic_filter, a = -0.5"""
    a = -0.5
    if x < 0.0:
        x = -x
    if x < 1.0:
        return ((a + 2.0) * x - (a + 3.0)) * x * x + 1
    if x < 2.0:
        return (((x - 5) * x + 8) * x - 4) * a
    return 0.0


def resample_coeffs(in_size: int, out_size: int):
    """Pillow precompute_coeffs (box 0..in_size) + normalize_coeffs_8bpc.
    Returns (bounds [out, 2] int32: first source index, tap count; kk [out, ksize] int32)."""
    scale = float(np.float32(in_size)) / out_size
    filterscale = max(scale, 1.0)
    support = 2.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), np.int32)
    kk = np.zeros((out_size, ksize), np.int32)
    for xx in range(out_size):
        center = 0.0 + (xx + 0.5) * scale
        ss = 1.0 / filterscale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        w = [_bicubic((x + xmin - center + 0.5) * ss) for x in range(xmax)]
        ww = 0.0
        for v in w:
            ww += v
        if ww != 0.0:
            w = [v / ww for v in w]
        for x, v in enumerate(w):
            kk[xx, x] = int(-0.5 + v * (1 << PRECISION_BITS)) if v < 0 else int(0.5 + v * (1 << PRECISION_BITS))
        bounds[xx] = (xmin, xmax)
    return bounds, kk


def _pass(src: np.ndarray, bounds, kk, axis: int) -> np.ndarray:
    """one 8-bit resampling pass along axis (0 = rows of an [H, W, C] image, 1 = columns)"""
    src = np.moveaxis(src, axis, 0).astype(np.int64)
    out = np.empty((len(bounds),) + src.shape[1:], np.uint8)
    for i, (lo, n) in enumerate(bounds):
        ss = np.full(src.shape[1:], 1 << (PRECISION_BITS - 1), np.int64)
        for t in range(n):
            ss += src[lo + t] * int(kk[i, t])
        out[i] = np.clip(ss >> PRECISION_BITS, 0, 255)
    return np.moveaxis(out, 0, axis)


def pil_resize_bicubic(img_hwc: np.ndarray, out_h: int, out_w: int) -> np.ndarray:
    """Image.fromarray(img).resize((out_w, out_h), BICUBIC) for a uint8 [H, W, C] image"""
    H, W = img_hwc.shape[:2]
    tmp = _pass(img_hwc, *resample_coeffs(W, out_w), axis=1)  # horizontal first
    return _pass(tmp, *resample_coeffs(H, out_h), axis=0)


def resize_output_size(H: int, W: int, shortest_edge: int):
    """image_transforms.get_resize_output_image_size(default_to_square=False) -> (h, w)"""
    short, long = (W, H) if W <= H else (H, W)
    new_short, new_long = shortest_edge, int(shortest_edge * long / short)
    return (new_long, new_short) if W <= H else (new_short, new_long)


def clip_preprocess_u8(img_chw: np.ndarray, shortest_edge: int = 336, crop=(336, 336)) -> np.ndarray:
    """resize + center crop of one uint8 [C, H, W] image -> uint8 [C, crop_h, crop_w]"""
    C, H, W = img_chw.shape
    rh, rw = resize_output_size(H, W, shortest_edge)
    r = pil_resize_bicubic(np.ascontiguousarray(img_chw.transpose(1, 2, 0)), rh, rw)
    top, left = (rh - crop[0]) // 2, (rw - crop[1]) // 2
    return np.ascontiguousarray(r[top:top + crop[0], left:left + crop[1]].transpose(2, 0, 1))


def normalize_table(mean=OPENAI_CLIP_MEAN, std=OPENAI_CLIP_STD, rescale: float = 1 / 255) -> np.ndarray:
    """f32 [C, 256]: normalized value of every uint8 level per channel (rescale then normalize)"""
    u = (np.arange(256, dtype=np.float64) * rescale).astype(np.float32)
    m = np.asarray(mean, np.float32)[:, None]
    s = np.asarray(std, np.float32)[:, None]
    return ((u[None, :] - m) / s).astype(np.float32)


def clip_preprocess(images_bchw: np.ndarray, shortest_edge: int = 336, crop=(336, 336)) -> np.ndarray:
    """pixel_values f32 [B, C, crop_h, crop_w] of a uint8 [B, C, H, W] batch"""
    tab = normalize_table()
    out = []
    for img in images_bchw:
        u8 = clip_preprocess_u8(img, shortest_edge, crop)
        out.append(np.stack([tab[c][u8[c]] for c in range(u8.shape[0])]))
    return np.stack(out)


# ---- prompt / label construction (cullavo/arch_cullavo.py:28-61, 424-436) ----------------------
SYSTEM_PROMPT = ("A chat between a curious human and an artificial intelligence assistant. "
                 "The assistant gives helpful, detailed, and polite answers to the human's questions. ")


def make_system_prompt(tokenize, ignore_index=-100, n_patches=576):
    """arch_cullavo.py:29-40: label = ignore * (len(tokens(system + '<image>', specials)) + 575)"""
    prompt = SYSTEM_PROMPT + "<image>"
    n = len(tokenize(prompt, True))
    return prompt, [ignore_index] * (n + n_patches - 1)


def make_and_add_prompt_and_label(prompt_so_far, label_so_far, prompt, answer, tokenize, ignore_index=-100):
    """arch_cullavo.py:42-61"""
    prompt = " USER: " + prompt + " ASSISTANT:"
    n = len(tokenize(prompt, False))
    prompt = prompt + " " + str(answer) + "</s>"
    ids = list(tokenize(prompt, False))
    ids[:n] = [ignore_index] * min(n, len(ids))
    return prompt_so_far + prompt, list(label_so_far) + ids


def conversation_prompt(conversations, tokenize, ignore_index=-100, n_patches=576):
    """step2_process's per-sample loop (arch_cullavo.py:424-436), conversation turns only"""
    p, lab = make_system_prompt(tokenize, ignore_index, n_patches)
    for k in range(len(conversations) // 2):
        q = conversations[2 * k]["value"]
        if k == 0:
            q = q.replace("<image>", "").strip()
        p, lab = make_and_add_prompt_and_label(p, lab, q, conversations[2 * k + 1]["value"], tokenize,
                                               ignore_index)
    return p, lab
