"""The data step: lbk.json records -> prompts, labels and pixel_values.

Drop-ins for the reference's prompt builders and the processor call they end in:

* ``make_system_prompt`` / ``make_and_add_prompt_and_label`` — reference
  cullavo/arch_cullavo.py:28-61 (same signatures; the label of the system prompt covers the 575
  extra image slots the merge inserts).
* ``step1_process`` — reference :96-339: detectron2-style instance records -> boxes drawn into
  the image, object / colour / box question-answer prompts.
* ``step2_process`` / ``eval_process`` — reference :397-543 / :63-94; records carrying ``boxes``
  get them drawn into the image plus the colour / box prompts (:436-499).
* ``overlay_boxes`` — detectron2's ``Visualizer(img).overlay_instances(boxes, assigned_colors)
  .get_image()`` as the reference calls it (:149-153, :441-448), on the GPU
  (csrc/boxdraw.hip: pixel-identical to matplotlib's Agg rendering of that figure).
  Random draws (colour shuffle, dice, permutations) use Python's ``random`` and torch's global
  generator in the reference's order, so a seeded call reproduces the reference's prompts.
* ``CuLLaVOProcessor`` — the LlavaProcessor call ``processor(text=..., images=..., padding=True,
  return_tensors="pt")``: the caller's tokenizer (any object with HF's ``__call__`` /
  ``pad_token_id`` / ``padding_side``; the real llava tokenizer is not available offline) pads
  the text, and ``ClipImageProcessorHIP`` turns the uint8 images into pixel_values on the GPU
  (csrc/imageprep.hip: PIL-bicubic shortest-edge resize, center crop, rescale, normalise,
  bit-identical to transformers' CLIPImageProcessor).
* ``load_lbk_records`` — reference datasets/registration/register_lbkllava_datasets.py:25-73
  (``lbk.json`` ShareGPT4V conversations; image records kept only when the file exists).
"""
from __future__ import annotations

import json
import os
import random
from dataclasses import dataclass

import numpy as np
import torch

from . import ops

SYSTEM_PROMPT = ("A chat between a curious human and an artificial intelligence assistant. "
                 "The assistant gives helpful, detailed, and polite answers to the human's questions. ")
OPENAI_CLIP_MEAN = (0.48145466, 0.4578275, 0.40821073)
OPENAI_CLIP_STD = (0.26862954, 0.26130258, 0.27577711)
N_IMAGE_SLOTS = 576


def _token_ids(tokenizer, text: str, add_special_tokens: bool) -> torch.Tensor:
    return tokenizer(text, return_tensors="pt", add_special_tokens=add_special_tokens).input_ids[0]


def make_system_prompt(processor, device, ignore_index):
    """reference cullavo/arch_cullavo.py:29-40"""
    prompt = SYSTEM_PROMPT + "<image>"
    length = _token_ids(processor.tokenizer, prompt, True).shape[0]
    label = torch.full((length + N_IMAGE_SLOTS - 1,), ignore_index, dtype=torch.long, device=device)
    return prompt, label


def make_and_add_prompt_and_label(cullavo_prompt, cullavo_label, prompt, answer, processor, device, ignore_index):
    """reference cullavo/arch_cullavo.py:42-61: the ' USER: ... ASSISTANT:' tokens are masked,
    the answer and its '</s>' are supervised"""
    prompt = " USER: " + prompt + " ASSISTANT:"
    length = _token_ids(processor.tokenizer, prompt, False).shape[0]
    prompt = prompt + " " + str(answer) + "</s>"
    label_ids = _token_ids(processor.tokenizer, prompt, False).clone().long()
    label_ids[:length] = ignore_index
    label = torch.cat([torch.as_tensor(cullavo_label, dtype=torch.long).cpu(), label_ids]).to(device)
    return cullavo_prompt + prompt, label


def list2string(_list) -> str:
    """reference cullavo/utils/utils.py:69-75"""
    return ", ".join(str(x) for x in _list)


def box2string(box) -> str:
    """reference cullavo/utils/utils.py:77-83: '[x0, y0, x1, y1]' with 3 decimals"""
    return "[" + ", ".join(f"{round(float(x), 3):.3f}" for x in box) + "]"


def boxes2string(boxes) -> str:
    """reference cullavo/utils/utils.py:85-91"""
    return "[" + ", ".join(box2string(b) for b in boxes) + "]"


def _numbered(classes, values, fmt) -> str:
    count = {}
    out = []
    for x, y in zip(classes, values):
        count[x] = count.get(x, 0) + 1
        out.append(fmt(count[x], x, y))
    return ", ".join(out)


def classescolors2string(classes, colors) -> str:
    """reference cullavo/utils/utils.py:93-103: '(#1 person) red, (#2 person) blue'"""
    return _numbered(classes, colors, lambda n, x, y: f"(#{n} {x}) {y}")


def classesboxes2string(classes, boxes) -> str:
    """reference cullavo/utils/utils.py:106-116: '(#1 person) [x0, y0, x1, y1], ...'"""
    return _numbered(classes, boxes, lambda n, x, y: f"(#{n} {x}) {box2string(y)}")


def classes2string(classes) -> str:
    """reference cullavo/utils/utils.py:118-128: '(#1) person, (#2) person'"""
    return _numbered(classes, classes, lambda n, x, y: f"(#{n}) {x}")


# reference cullavo/utils/utils.py:14-33 and the matplotlib (CSS4) colours those names draw with
COLOR_LIST = ["white", "red", "orange", "coral", "yellow", "green", "blue", "navy", "gold", "pink", "purple",
              "brown", "violet", "olive", "lime", "cyan", "magenta", "silver", "gray", "black"]
COLOR_RGB = {
    "white": (255, 255, 255), "red": (255, 0, 0), "orange": (255, 165, 0), "coral": (255, 127, 80),
    "yellow": (255, 255, 0), "green": (0, 128, 0), "blue": (0, 0, 255), "navy": (0, 0, 128),
    "gold": (255, 215, 0), "pink": (255, 192, 203), "purple": (128, 0, 128), "brown": (165, 42, 42),
    "violet": (238, 130, 238), "olive": (128, 128, 0), "lime": (0, 255, 0), "cyan": (0, 255, 255),
    "magenta": (255, 0, 255), "silver": (192, 192, 192), "gray": (128, 128, 128), "black": (0, 0, 0),
}
# reference utils/constants.py:1 (COCO panoptic: 80 thing + 53 stuff classes)
COCO_PANOPTIC_CLASSES = [
    'person', 'bicycle', 'car', 'motorcycle', 'airplane', 'bus', 'train', 'truck', 'boat',
    'traffic light', 'fire hydrant', 'stop sign', 'parking meter', 'bench', 'bird', 'cat', 'dog',
    'horse', 'sheep', 'cow', 'elephant', 'bear', 'zebra', 'giraffe', 'backpack', 'umbrella', 'handbag',
    'tie', 'suitcase', 'frisbee', 'skis', 'snowboard', 'sports ball', 'kite', 'baseball bat',
    'baseball glove', 'skateboard', 'surfboard', 'tennis racket', 'bottle', 'wine glass', 'cup',
    'fork', 'knife', 'spoon', 'bowl', 'banana', 'apple', 'sandwich', 'orange', 'broccoli', 'carrot',
    'hot dog', 'pizza', 'donut', 'cake', 'chair', 'couch', 'potted plant', 'bed', 'dining table',
    'toilet', 'tv', 'laptop', 'mouse', 'remote', 'keyboard', 'cell phone', 'microwave', 'oven',
    'toaster', 'sink', 'refrigerator', 'book', 'clock', 'vase', 'scissors', 'teddy bear', 'hair drier',
    'toothbrush', 'banner', 'blanket', 'bridge', 'cardboard', 'counter', 'curtain', 'door-stuff',
    'floor-wood', 'flower', 'fruit', 'gravel', 'house', 'light', 'mirror-stuff', 'net', 'pillow',
    'platform', 'playingfield', 'railroad', 'river', 'road', 'roof', 'sand', 'sea', 'shelf', 'snow',
    'stairs', 'tent', 'towel', 'wall-brick', 'wall-stone', 'wall-tile', 'wall-wood', 'water-other',
    'window-blind', 'window-other', 'tree-merged', 'fence-merged', 'ceiling-merged',
    'sky-other-merged', 'cabinet-merged', 'table-merged', 'floor-other-merged', 'pavement-merged',
    'mountain-merged', 'grass-merged', 'dirt-merged', 'paper-merged', 'food-other-merged',
    'building-other-merged', 'rock-merged', 'wall-other-merged', 'rug-merged',
]
VISUALIZER_FONT_SIZE = 16  # vis._default_font_size = 16 (reference :150, :444)


def overlay_boxes(images, boxes, colors, device=None):
    """Visualizer(img); _default_font_size = 16; overlay_instances(boxes=boxes,
    assigned_colors=colors).get_image() for each image (reference :149-153, :441-448).

    images: uint8 [3, H, W] tensors (a [B, 3, H, W] batch or a list of any sizes); boxes: per
    image an [n, 4] float32 (x0, y0, x1, y1) pixel array; colors: per image n colour names of
    COLOR_RGB. Returns uint8 [3, H, W] tensors on ``device`` (the GPU), one per image."""
    if isinstance(images, torch.Tensor) and images.dim() == 3:
        images, boxes, colors = [images], [boxes], [colors]
    imgs = list(images)
    dev = device or torch.device("cuda", torch.cuda.current_device())
    out = [None] * len(imgs)
    groups = {}
    for i, im in enumerate(imgs):
        groups.setdefault(tuple(im.shape), []).append(i)
    for shape, idx in groups.items():
        batch = torch.stack([torch.as_tensor(imgs[i]) for i in idx]).to(dev)
        res = ops.draw_boxes(batch, [np.asarray(boxes[i], np.float32).reshape(-1, 4) for i in idx],
                             [[COLOR_RGB[c] for c in colors[i]] for i in idx], font_size=VISUALIZER_FONT_SIZE)
        for j, i in enumerate(idx):
            out[i] = res[j]
    return out


# ---- images ------------------------------------------------------------------------------------
def resize_output_size(H: int, W: int, shortest_edge: int):
    """transformers get_resize_output_image_size(default_to_square=False) -> (h, w)"""
    short, long = (W, H) if W <= H else (H, W)
    new_short, new_long = shortest_edge, int(shortest_edge * long / short)
    return (new_long, new_short) if W <= H else (new_short, new_long)


class ClipImageProcessorHIP:
    """CLIPImageProcessor (llava-1.5 / CLIP-L/14-336 settings) on the GPU.

    __call__(images) takes uint8 images — a [B, C, H, W] tensor (the reference stacks CHW
    tensors, cullavo/arch_cullavo.py:313,516), a [C, H, W] tensor, or a list of them with
    different sizes — and returns pixel_values [B, C, crop, crop] (f32 by default, like the
    processor; bf16 on request for the vision tower)."""

    def __init__(self, shortest_edge: int = 336, crop_size: int = 336, rescale_factor: float = 1 / 255,
                 image_mean=OPENAI_CLIP_MEAN, image_std=OPENAI_CLIP_STD, device=None):
        self.shortest_edge = int(shortest_edge)
        self.crop = (int(crop_size), int(crop_size))
        self.rescale_factor = float(rescale_factor)
        self.mean = tuple(float(np.float32(m)) for m in image_mean)
        self.std = tuple(float(np.float32(s)) for s in image_std)
        self.device = device
        self._tables = {}

    def _coeffs(self, in_size: int, out_size: int, device):
        key = (in_size, out_size, str(device))
        if key not in self._tables:
            L = ops.lib()
            ksize = L.cullavo_resample_coeffs(in_size, out_size, None, None, 0)
            bounds = np.zeros(2 * out_size, np.int32)
            kk = np.zeros(out_size * ksize, np.int32)
            rc = L.cullavo_resample_coeffs(in_size, out_size, bounds.ctypes.data, kk.ctypes.data, ksize)
            if rc != ksize:
                raise ValueError(f"cullavo_resample_coeffs({in_size}, {out_size}) failed ({rc})")
            self._tables[key] = (torch.from_numpy(bounds).to(device), torch.from_numpy(kk).to(device), ksize)
        return self._tables[key]

    def preprocess_batch(self, images: torch.Tensor, out_dtype=torch.float32, out=None) -> torch.Tensor:
        """images: uint8 [B, C, H, W] on the GPU (any strides) -> pixel_values [B, C, ch, cw]"""
        if images.dtype != torch.uint8 or images.dim() != 4:
            raise ValueError("images must be a uint8 [B, C, H, W] tensor")
        B, C, H, W = images.shape
        if C > 3:
            raise ValueError(f"expected at most 3 channels, got {C}")
        dev = images.device
        Hr, Wr = resize_output_size(H, W, self.shortest_edge)
        ch, cw = self.crop
        if ch > Hr or cw > Wr:
            raise ValueError(f"crop {self.crop} larger than the resized image {(Hr, Wr)}")
        top, left = (Hr - ch) // 2, (Wr - cw) // 2
        hb, hk, hks = self._coeffs(W, Wr, dev)
        vb, vk, vks = self._coeffs(H, Hr, dev)
        tmp = torch.empty(B * C * H * cw, dtype=torch.uint8, device=dev)
        if out is None:
            out = torch.empty((B, C, ch, cw), dtype=out_dtype, device=dev)
        ops.clip_image_preprocess(images, Hr, Wr, hb, hk, hks, vb, vk, vks, top, left, ch, cw,
                                  self.rescale_factor, self.mean, self.std, tmp, out)
        return out

    def __call__(self, images, out_dtype=torch.float32, device=None):
        device = device or self.device or torch.device("cuda", torch.cuda.current_device())
        if isinstance(images, np.ndarray):
            images = torch.from_numpy(images)
        if isinstance(images, torch.Tensor):
            if images.dim() == 3:
                images = images[None]
            return self.preprocess_batch(images.to(device), out_dtype)
        imgs = [torch.as_tensor(im) for im in images]
        out = torch.empty((len(imgs), imgs[0].shape[0]) + self.crop, dtype=out_dtype, device=device)
        shapes = {}
        for i, im in enumerate(imgs):  # one launch per distinct image size
            shapes.setdefault(tuple(im.shape), []).append(i)
        for shape, idx in shapes.items():
            batch = torch.stack([imgs[i] for i in idx]).to(device)
            res = self.preprocess_batch(batch, out_dtype)
            out[torch.tensor(idx, device=device)] = res
        return out


@dataclass
class BatchEncoding:
    input_ids: torch.Tensor
    attention_mask: torch.Tensor
    pixel_values: torch.Tensor | None = None

    def __getitem__(self, k):
        return getattr(self, k)


class CuLLaVOProcessor:
    """LlavaProcessor's __call__ as the reference uses it (text + images, padding=True, 'pt')"""

    def __init__(self, tokenizer, image_processor: ClipImageProcessorHIP | None = None):
        self.tokenizer = tokenizer
        self.image_processor = image_processor or ClipImageProcessorHIP()

    def __call__(self, text=None, images=None, padding=True, return_tensors="pt", **kw):
        texts = [text] if isinstance(text, str) else list(text)
        seqs = [list(_token_ids(self.tokenizer, t, True).tolist()) for t in texts]
        n = max(len(s) for s in seqs)
        pad = self.tokenizer.pad_token_id
        left = getattr(self.tokenizer, "padding_side", "right") == "left"
        ids = torch.full((len(seqs), n), pad, dtype=torch.long)
        mask = torch.zeros((len(seqs), n), dtype=torch.long)
        for i, s in enumerate(seqs):
            sl = slice(n - len(s), n) if left else slice(0, len(s))
            ids[i, sl] = torch.tensor(s, dtype=torch.long)
            mask[i, sl] = 1
        pix = self.image_processor(images) if images is not None else None
        return BatchEncoding(ids, mask, pix)

    def batch_decode(self, sequences, skip_special_tokens=True, **kw):
        """LlavaProcessor.batch_decode -> the tokenizer's"""
        return self.tokenizer.batch_decode(sequences, skip_special_tokens=skip_special_tokens, **kw)


# ---- step-2-pre labelling (reference cullavo/arch_cullavo.py:341-395) -----------------------------
STEP2_PRE_PROMPT = ("provide multiple object names with their numbering index and the objects' bounding box "
                    "coordinates in the image.")
STEP2_PRE_GENERATE = dict(do_sample=True, temperature=0.9, top_k=50, top_p=0.95, max_new_tokens=1000, use_cache=True)


def find(s: str, ch: str) -> list[int]:
    """reference cullavo/utils/utils.py:66-67"""
    return [i for i, c in enumerate(s) if c == ch]


def box_and_class_parser(decoded_text: str):
    """reference cullavo/utils/utils.py:46-64: '(... name)' / '[x0, y0, x1, y1]' pairs of the
    generated text -> (box tensor [n, 4], class names, flag); flag = True when the brackets do
    not pair up. The box literal is read with ast.literal_eval instead of the reference's eval()
    (generated text is untrusted; literal_eval accepts exactly the list literals eval() parses
    here and raises on anything else, which the caller's except branch handles like the
    reference's)."""
    import ast
    sb, eb = find(decoded_text, "["), find(decoded_text, "]")
    sc, ec = find(decoded_text, "("), find(decoded_text, ")")
    if len(sb) != len(eb) or len(sc) != len(ec) or len(sc) != len(sb):
        return None, None, True
    boxes, classes = [], []
    for b0, b1, c0, c1 in zip(sb, eb, sc, ec):
        boxes.append(ast.literal_eval(decoded_text[b0:b1 + 1]))
        classes.append(decoded_text[c0 + 1:c1].split(" ")[-1])
        if len(boxes[-1]) != 4:
            boxes.pop(-1)
            classes.pop(-1)
    return torch.tensor(boxes), classes, False


def step2_preprocess(model, batched_inputs, processor, device, *, dice=None, generate_kwargs=None, on_generate=None,
                     vis_dir=None):
    """reference cullavo/arch_cullavo.py:341-395: for one record in ~50 (torch.randint(0, 50) == 0)
    generate an object/box description of its image with the reference's sampling settings
    (T 0.9, top-k 50, top-p 0.95, 1000 new tokens, KV cache), parse boxes and classes, and emit
    the new lbk.json entry; every other record passes through. With vis_dir the image with the
    boxes (x 336) and class names is written to vis_dir/<question_id>.png like the reference's
    debugging render (:376-386, visualize.render_boxes_and_labels); a failing render emits the
    record without boxes, as the reference's bare except does. dice(record) replaces
    the random roll, generate_kwargs override the sampling settings (tests: greedy),
    on_generate(record, generate_ids, decoded_text) observes each generation."""
    gk = dict(STEP2_PRE_GENERATE, **(generate_kwargs or {}))
    new = []
    for batch in batched_inputs:
        if "image" not in batch:
            new.append({"id": batch["question_id"], "conversations": batch["question"]})
            continue
        roll = int(torch.randint(high=50, low=0, size=(1,)).item()) if dice is None else int(dice(batch))
        base = {"id": batch["question_id"], "image": batch.get("image_id"), "conversations": batch["question"]}
        if roll != 0:
            new.append(base)
            continue
        inputs = eval_process(images=batch["image"], prompt=STEP2_PRE_PROMPT, processor=processor, device=device,
                              ignore_index=model.config.ignore_index)
        with torch.inference_mode():
            ids = model.generate(**inputs, **gk)
        text = processor.batch_decode(ids, skip_special_tokens=True)[0]
        if on_generate is not None:
            on_generate(batch, ids, text)
        try:
            boxes, classes, flag = box_and_class_parser(text)
            if flag:
                continue  # the reference drops the record (:372-373)
            if len(classes) > len(COLOR_LIST):
                # the reference draws box_tensor[:len(color_list)] with labels=class_list at full
                # length: detectron2's overlay_instances asserts len(labels) == num_instances
                # (utils/visualizer.py:673) and the bare except emits the record without boxes
                new.append(base)
                continue
            if vis_dir is not None:
                import os

                from PIL import Image

                from .visualize import render_boxes_and_labels
                n = boxes.shape[0]
                img = render_boxes_and_labels(batch["image"], boxes[:len(COLOR_LIST)] * 336, classes,
                                              COLOR_LIST[:n])
                Image.fromarray(img).save(os.path.join(vis_dir, f"{batch['question_id']}.png"))
            new.append(dict(base, boxes=boxes.cpu().tolist(), classes=classes))
        except Exception:  # the reference's bare except (:387-388)
            new.append(base)
    return new


def _outputs(input_ids, pixel_values, attention_mask, labels=None):
    out = dict.fromkeys(["input_ids", "pixel_values", "attention_mask", "position_ids", "past_key_values",
                         "inputs_embeds", "vision_feature_layer", "vision_feature_select_strategy", "labels",
                         "use_cache", "output_attentions", "output_hidden_states", "return_dict"])
    out.update(input_ids=input_ids, pixel_values=pixel_values, attention_mask=attention_mask, labels=labels)
    return out


def _draw_default(image, boxes, colors):
    """one image through overlay_boxes (GPU)"""
    return overlay_boxes([torch.as_tensor(image)], [boxes], [colors])[0]


def _stack(images):
    """torch.stack on one device (the GPU when any image is there), or the list for mixed sizes"""
    dev = next((im.device for im in images if im.is_cuda), torch.device("cpu"))
    images = [im.to(dev) for im in images]
    if len({tuple(im.shape) for im in images}) == 1:
        return torch.stack(images)
    return images


def _finish(prompts, labels, images, processor, device, ignore_index):
    enc = processor(text=prompts, images=_stack(images), padding=True, return_tensors="pt")
    lab = torch.nn.utils.rnn.pad_sequence([x.cpu() for x in labels], batch_first=True, padding_value=ignore_index)
    return _outputs(enc.input_ids.to(device), enc.pixel_values.to(device) if enc.pixel_values is not None else None,
                    enc.attention_mask.to(device), lab.to(device))


def step2_process(batched_inputs, processor, device, ignore_index=-100, image_size=336, draw=None):
    """reference cullavo/arch_cullavo.py:397-543: per record the system prompt, then each
    (question, answer) turn ('<image>' stripped from the first question); a record with
    ``boxes`` (normalised x0 y0 x1 y1) gets them drawn into its image (x 336, colours from a
    fresh shuffle of COLOR_LIST; the record's image is replaced like the reference's :448) and
    the colour prompt plus up to 5 colour <-> box prompts (:450-499); images stacked (zeros
    [3, 336, 336] for text-only records), one processor call, labels right-padded with
    ignore_index. ``draw(image, boxes_px, colour_names)`` replaces the GPU drawing (tests)."""
    draw = draw or _draw_default
    images, prompts, labels = [], [], []
    for batch in batched_inputs:
        p, lab = make_system_prompt(processor, device, ignore_index)
        q = batch["question"]
        for k in range(len(q) // 2):
            text = q[2 * k]["value"] if k != 0 else q[2 * k]["value"].replace("<image>", "").strip()
            p, lab = make_and_add_prompt_and_label(p, lab, text, q[2 * k + 1]["value"], processor, device,
                                                   ignore_index)
        if "boxes" in batch:
            cl = list(COLOR_LIST)
            random.shuffle(cl)
            bt = torch.tensor(batch["boxes"])
            n = len(batch["boxes"])
            batch["image"] = draw(batch["image"], (bt * 336).numpy(), cl[:n])
            colors = cl[:n]
            answer = (f"Sure, it is {list2string(colors)} color. There is a bounding box in the image." if n == 1
                      else f"Sure, it is {list2string(colors)} color. There are {n} bounding boxes in the image.")
            p, lab = make_and_add_prompt_and_label(p, lab, "provide multiple bounding box colors in the image.",
                                                   answer, processor, device, ignore_index)
            for r_int in torch.randperm(n)[:5]:
                box, color = bt[r_int], cl[r_int]
                if torch.randint(high=2, low=0, size=(1,)).item() == 0:
                    qa = (f"provide a bounding box coordinate of {color} bounding box color.",
                          f"Sure, it is {box2string(box)}. There is a {color} bounding box color")
                else:
                    qa = (f"provide a bounding box color of bounding box coordinate {box2string(box)}.",
                          f"Sure, it is {color} color.")
                p, lab = make_and_add_prompt_and_label(p, lab, *qa, processor, device, ignore_index)
        if "image" in batch:
            images.append(torch.as_tensor(batch["image"]))
        else:
            images.append(torch.zeros(3, image_size, image_size, dtype=torch.uint8))
        prompts.append(p)
        labels.append(lab)
    return _finish(prompts, labels, images, processor, device, ignore_index)


def _class_name(c) -> str:
    return COCO_PANOPTIC_CLASSES[int(c)].replace("-merged", "").replace("-other", "").replace("-stuff", "")


def _box_tensor(gt_boxes) -> torch.Tensor:
    return gt_boxes.tensor if hasattr(gt_boxes, "tensor") else torch.as_tensor(gt_boxes)


def step1_process(inputs, processor, device, ignore_index=-100, fix_num=5, draw=None):
    """reference cullavo/arch_cullavo.py:96-339 (step 1: object understanding).

    inputs: detectron2-style records {"image": uint8 [3, H, W], "instances": object with
    ``is_things``, ``gt_classes`` (COCO panoptic ids) and ``gt_boxes`` (Boxes or an [n, 4]
    pixel tensor)}. For each record with thing instances (at most 20, one per colour): the boxes
    drawn into the image in a shuffled colour order, then the prompts — objects with their
    boxes, the box colours, one class -> colours / boxes question picked by a die, and up to
    ``fix_num`` colour <-> box and box / colour -> class questions — with the reference's
    random draws in its order (one ``random.shuffle`` per call, ``torch.randint`` /
    ``torch.randperm`` per record). Returns the model inputs, or {"input_ids": None} when no
    record has a thing instance (:309). The reference scales the record's Boxes in place
    (:145); this leaves the record untouched. Its drawing multiplies both coordinates by the
    image height (:151), reproduced as is."""
    draw = draw or _draw_default
    cl = list(COLOR_LIST)
    random.shuffle(cl)
    images, prompts, labels = [], [], []
    for inp in inputs:
        inst = inp["instances"]
        things = [i for i, t in enumerate(inst.is_things) if t]
        idx = torch.tensor(things, dtype=torch.long)[:len(cl)]
        if len(idx) == 0:
            continue
        cls_ids = torch.as_tensor(inst.gt_classes)[idx]
        names = [_class_name(c) for c in cls_ids]
        uniq = cls_ids.unique()
        uniq_names = [_class_name(c) for c in uniq]
        _, H, W = inp["image"].shape
        gt = _box_tensor(inst.gt_boxes).clone()
        gt[:, 0::2] *= 1 / W
        gt[:, 1::2] *= 1 / H
        boxes = gt[idx]
        colors = cl[:len(idx)]
        boxed = draw(inp["image"], (boxes * H).cpu().numpy(), colors)
        p, lab = make_system_prompt(processor, device, ignore_index)
        n = len(names)
        answer = (f"Sure, it is {classesboxes2string(names, boxes)}. There is an object in the image." if n == 1
                  else f"Sure, it is {classesboxes2string(names, boxes)}. There are {n} objects in the image.")
        p, lab = make_and_add_prompt_and_label(
            p, lab, "provide multiple object names with their numbering index and the objects' bounding box "
                    "coordinates in the image.", answer, processor, device, ignore_index)
        answer = (f"Sure, it is {list2string(colors)} color. There is a bounding box in the image." if n == 1
                  else f"Sure, it is {list2string(colors)} color. There are {n} bounding boxes in the image.")
        p, lab = make_and_add_prompt_and_label(p, lab, "provide multiple bounding box colors in the image.", answer,
                                               processor, device, ignore_index)
        dice = torch.randint(high=2, low=0, size=(1,)).item()
        pick = torch.randint(high=len(uniq), low=0, size=(1,)).item()
        sel_cls = uniq_names[pick]
        sel = torch.where(cls_ids == uniq[pick])[0]
        sel_names = [names[i.item()] for i in sel]
        sel_boxes = boxes[sel]
        sel_colors = [cl[i.item()] for i in sel]
        m = len(sel_names)
        tail = "There is a bounding box in the image." if m == 1 else f"There are {m} bounding boxes in the image."
        if dice == 0:
            qa = (f"provide multiple bounding box colors corresponding {sel_cls} in the image.",
                  f"Sure, it is {classescolors2string(sel_names, sel_colors)} color. {tail}")
        else:
            qa = (f"provide multiple bounding box coordinates for {sel_cls} in the image.",
                  f"Sure, it is {classesboxes2string(sel_names, sel_boxes)} color. {tail}")
        p, lab = make_and_add_prompt_and_label(p, lab, *qa, processor, device, ignore_index)
        for r_int in torch.randperm(len(boxes))[:fix_num]:
            name, box, color = names[r_int], boxes[r_int], cl[r_int]
            if torch.randint(high=2, low=0, size=(1,)).item() == 0:
                qa = (f"provide a bounding box coordinate of {color} bounding box color.",
                      f"Sure, it is {box2string(box)}. There is a {color} bounding box color")
            else:
                qa = (f"provide a bounding box color of bounding box coordinate {box2string(box)}.",
                      f"Sure, it is {color} color.")
            p, lab = make_and_add_prompt_and_label(p, lab, *qa, processor, device, ignore_index)
            if torch.randint(high=2, low=0, size=(1,)).item() == 0:
                qa = (f"provide an object name for bounding box coordinate {box2string(box)}.", f"Sure, it is {name}.")
            else:
                qa = (f"provide an object name for {color} bounding box.", f"Sure, it is {name}.")
            p, lab = make_and_add_prompt_and_label(p, lab, *qa, processor, device, ignore_index)
        images.append(boxed)
        prompts.append(p)
        labels.append(lab)
    if not prompts:
        return {"input_ids": None}
    return _finish(prompts, labels, images, processor, device, ignore_index)


def eval_process(images, aux_prompt=None, prompt=None, processor=None, device=None, ignore_index=-100):
    """reference cullavo/arch_cullavo.py:63-94"""
    p, _ = make_system_prompt(processor, device, ignore_index)
    p += f" {aux_prompt} USER: {prompt} ASSISTANT:" if aux_prompt else f" USER: {prompt} ASSISTANT:"
    enc = processor(text=p, images=images, padding=True, return_tensors="pt")
    return {"input_ids": enc.input_ids.to(device), "pixel_values": enc.pixel_values.to(device),
            "attention_mask": enc.attention_mask.to(device)}


def load_lbk_records(json_path: str, image_root: str | None = None):
    """reference register_lbkllava_datasets.py:25-73 (load_pretrain_arrows + load_pretrain_data):
    image records are kept only when image_root/<image> exists; boxes are carried through"""
    with open(json_path) as f:
        questions = json.load(f)
    ret = []
    for q in questions:
        rec = {"question": q["conversations"], "question_id": q["id"]}
        if "image" in q:
            if image_root is None or not os.path.isfile(os.path.join(image_root, q["image"])):
                continue
            rec = {"image_id": q["image"], **rec}
            if "boxes" in q:
                rec["boxes"] = q["boxes"]
        ret.append(rec)
    if not ret:
        raise AssertionError("No images found in pretraining")
    return ret
