"""Box drawing of the step-1 / step-2 prompts (reference
cullavo/arch_cullavo.py:96-339 step1_process, :436-499 step-2 records with boxes).

Parity chain: tests/golden/make_golden_boxes.py renders with matplotlib (the renderer
detectron2's Visualizer drives; detectron2 itself is absent, its wrapper is restated there) and
runs the REFERENCE's own step1_process / step2_process. Here:
* CPU: oracle/boxdraw_oracle.py reproduces those rasters bit-exactly; the host geometry of
  libcullavo_hip.so (imshow maps, transData) equals the oracle's; prompting.step1_process /
  step2_process with the oracle's drawing reproduce the reference's ids, labels and images.
* GPU: cullavo_draw_boxes reproduces the fixtures and the oracle bit-exactly (random boxes of
  every kind, large images, strided inputs); step1_process / step2_process with the GPU drawing
  reproduce the reference's outputs.
"""
import json
import os
import random

import numpy as np
import pytest
import torch

from oracle import boxdraw_oracle as BO
from tests.golden.make_golden_boxes import (COLORS, STEP2_RECORDS, PassProcessor, case_boxes, case_image,
                                            step1_records)
from tests.toy_tokenizer import ToyTokenizer

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def fx():
    return np.load(os.path.join(GOLD, "boxdraw.npz"))


@pytest.fixture(scope="module")
def prompts_fx():
    with open(os.path.join(GOLD, "boxdraw_prompts.json")) as f:
        return json.load(f)


def oracle_draw(image, boxes, colors):
    """prompting's draw hook through the oracle (CPU)"""
    img = torch.as_tensor(image).cpu().permute(1, 2, 0).numpy()
    return torch.from_numpy(BO.overlay_boxes(img, boxes, colors).transpose(2, 0, 1).copy())


def test_oracle_matches_matplotlib(fx):
    for seed, H, W, n in fx["cases"]:
        img = case_image(int(seed), int(H), int(W))
        out = BO.overlay_boxes(img.transpose(1, 2, 0), fx[f"c{seed}_boxes"], [COLORS[i] for i in fx[f"c{seed}_colors"]])
        assert np.array_equal(out.transpose(2, 0, 1), fx[f"c{seed}_out"]), (seed, H, W)


def test_host_geometry_matches_oracle():
    import cullavo_amd.ops as ops
    L = ops.lib()
    rng = np.random.default_rng(0)
    sizes = [(255, 236), (29, 60), (100, 37), (336, 336), (480, 640), (1, 1), (2, 3000)]
    sizes += [tuple(int(v) for v in s) for s in rng.integers(1, 2000, (40, 2))]
    for H, W in sizes:
        rows, cols, td = np.zeros(H, np.int32), np.zeros(W, np.int32), np.zeros(4)
        assert L.cullavo_visimage_geometry(H, W, rows.ctypes.data, cols.ctypes.data, td.ctypes.data) == 0
        r, c = BO.visimage_maps(H, W)
        assert np.array_equal(rows, r) and np.array_equal(cols, c), (H, W)
        assert tuple(td) == BO.axes_transform(H, W)[0], (H, W)


def _check_prompt_outputs(res, ref, images):
    assert res["input_ids"].tolist() == ref["input_ids"]
    assert res["attention_mask"].tolist() == ref["attention_mask"]
    assert res["labels"].tolist() == ref["labels"]
    assert np.array_equal(res["pixel_values"].cpu().numpy().astype(np.uint8), images)


def _step2_images(fx, k, seed):
    rows, cols = BO.visimage_maps(336, 336)
    base = np.stack([case_image(seed * 10 + j, 336, 336)[:, rows][:, :, cols] for j in range(len(STEP2_RECORDS))])
    np.put(base, fx[f"step2_{k}_diff_idx"], fx[f"step2_{k}_diff_val"])
    return base


def _run_step1(seed, draw):
    from cullavo_amd.prompting import step1_process
    random.seed(seed)
    torch.manual_seed(seed)
    return step1_process(step1_records(seed), PassProcessor(ToyTokenizer()), "cpu", draw=draw)


def _run_step2(seed, draw, device="cpu"):
    from cullavo_amd.prompting import step2_process
    random.seed(seed)
    torch.manual_seed(seed)
    recs = [dict(r, question=list(r["question"]), image=torch.from_numpy(case_image(seed * 10 + j, 336, 336)))
            for j, r in enumerate(STEP2_RECORDS)]
    return step2_process(recs, PassProcessor(ToyTokenizer()), device, draw=draw)


def test_step1_process_matches_reference(fx, prompts_fx):
    for k, ref in enumerate(prompts_fx["step1"]):
        _check_prompt_outputs(_run_step1(ref["seed"], oracle_draw), ref, fx[f"step1_{k}_images"])


def test_step2_box_records_match_reference(fx, prompts_fx):
    for k, ref in enumerate(prompts_fx["step2"]):
        _check_prompt_outputs(_run_step2(ref["seed"], oracle_draw), ref, _step2_images(fx, k, ref["seed"]))


def test_step1_without_things_returns_none():
    from cullavo_amd.prompting import step1_process
    recs = step1_records(3)
    for r in recs:
        r["instances"].is_things = [False] * len(r["instances"].is_things)
    assert step1_process(recs, PassProcessor(ToyTokenizer()), "cpu", draw=oracle_draw) == {"input_ids": None}


def test_box_strings():
    from cullavo_amd import prompting as P
    b = torch.tensor([[0.1234, 0.5, 0.98765, 1.0], [0.0, 0.25, 0.5, 0.75]])
    assert P.classesboxes2string(["cat", "cat"], b) == \
        "(#1 cat) [0.123, 0.500, 0.988, 1.000], (#2 cat) [0.000, 0.250, 0.500, 0.750]"
    assert P.classescolors2string(["dog", "cat", "dog"], ["red", "blue", "gold"]) == \
        "(#1 dog) red, (#1 cat) blue, (#2 dog) gold"
    assert P.classes2string(["a", "a"]) == "(#1) a, (#2) a"
    assert P.boxes2string(b[:1]) == "[[0.123, 0.500, 0.988, 1.000]]"
    assert len(P.COCO_PANOPTIC_CLASSES) == 133 and P.COCO_PANOPTIC_CLASSES[0] == "person"
    assert set(P.COLOR_LIST) == set(P.COLOR_RGB) == set(BO.COLOR_RGB) and P.COLOR_RGB == BO.COLOR_RGB


# ---- GPU ------------------------------------------------------------------------------------------
def _gpu_draw(img_chw, boxes, colors, **kw):
    import cullavo_amd.ops as ops
    t = torch.from_numpy(np.ascontiguousarray(img_chw))[None].cuda()
    return ops.draw_boxes(t, [boxes], [[BO.COLOR_RGB[c] for c in colors]], **kw)[0].cpu().numpy()


@pytest.mark.gpu
def test_draw_boxes_matches_matplotlib_fixtures(fx):
    import cullavo_amd.ops as ops
    for seed, H, W, n in fx["cases"]:
        img = case_image(int(seed), int(H), int(W))
        out = _gpu_draw(img, fx[f"c{seed}_boxes"], [COLORS[i] for i in fx[f"c{seed}_colors"]])
        assert np.array_equal(out, fx[f"c{seed}_out"]), (seed, H, W)
    # a batch of same-size images in one launch, with a different box count per image
    imgs = [case_image(s, 64, 80) for s in (21, 22, 23)]
    boxes = [case_boxes(21, 64, 80, 7), case_boxes(22, 64, 80, 0), case_boxes(23, 64, 80, 13)]
    cols = [[COLORS[(i * 7 + j) % 20] for j in range(len(b))] for i, b in enumerate(boxes)]
    out = ops.draw_boxes(torch.from_numpy(np.stack(imgs)).cuda(), boxes,
                         [[BO.COLOR_RGB[c] for c in cs] for cs in cols]).cpu().numpy()
    for i in range(3):
        ref = BO.overlay_boxes(imgs[i].transpose(1, 2, 0), boxes[i], cols[i]).transpose(2, 0, 1)
        assert np.array_equal(out[i], ref), i


@pytest.mark.gpu
def test_draw_boxes_random_vs_oracle():
    rng = np.random.default_rng(5)
    for t in range(12):
        H, W = (336, 336) if t < 3 else (int(rng.integers(4, 700)), int(rng.integers(4, 700)))
        if t == 3:
            H, W = 480, 640
        img = case_image(100 + t, H, W)
        boxes = case_boxes(100 + t, H, W, int(rng.integers(1, 21)))
        cols = [COLORS[int(i)] for i in rng.integers(0, 20, len(boxes))]
        out = _gpu_draw(img, boxes, cols)
        ref = BO.overlay_boxes(img.transpose(1, 2, 0), boxes, cols).transpose(2, 0, 1)
        assert np.array_equal(out, ref), (t, H, W)


@pytest.mark.gpu
def test_draw_boxes_strided_input_and_alpha():
    import cullavo_amd.ops as ops
    img = case_image(7, 90, 120)
    boxes = case_boxes(7, 90, 120, 10)
    cols = [COLORS[i % 20] for i in range(10)]
    hwc = torch.from_numpy(img.transpose(1, 2, 0).copy()).cuda()
    out = ops.draw_boxes(hwc.permute(2, 0, 1)[None], [boxes], [[BO.COLOR_RGB[c] for c in cols]])[0].cpu().numpy()
    assert np.array_equal(out, BO.overlay_boxes(img.transpose(1, 2, 0), boxes, cols).transpose(2, 0, 1))
    out1 = _gpu_draw(img, boxes, cols, alpha=1.0)  # opaque colour: full-cover pixels are copied
    assert np.array_equal(out1, BO.overlay_boxes(img.transpose(1, 2, 0), boxes, cols, alpha=1.0).transpose(2, 0, 1))
    with pytest.raises(RuntimeError):
        ops.draw_boxes(torch.from_numpy(img)[None], [boxes], [[(0, 0, 0)] * 10])  # CPU tensor: no CPU path
    with pytest.raises(ValueError):
        ops.draw_boxes(torch.from_numpy(img)[None, :2].cuda(), [boxes], [[(0, 0, 0)] * 10])


@pytest.mark.gpu
def test_step1_step2_prompts_gpu_drawing_match_reference(fx, prompts_fx):
    for k, ref in enumerate(prompts_fx["step1"]):
        _check_prompt_outputs(_run_step1(ref["seed"], None), ref, fx[f"step1_{k}_images"])
    for k, ref in enumerate(prompts_fx["step2"]):
        _check_prompt_outputs(_run_step2(ref["seed"], None, "cuda"), ref, _step2_images(fx, k, ref["seed"]))


@pytest.mark.gpu
def test_forward_step1_pipeline_on_records():
    """CuLLaVO.forward in the step-1 config (reference cullavo_model.py:45-71): records ->
    step1_process (GPU drawing + preprocessing) -> model -> loss, equal to running the two halves
    by hand with the same random state; a batch without things gives loss 0"""
    from cullavo_amd.arch_cullavo import CuLLaVOModel
    from cullavo_amd.config import tiny_gpu
    from cullavo_amd.pipeline import CuLLaVO
    from cullavo_amd.prompting import ClipImageProcessorHIP, CuLLaVOProcessor
    from tests.test_eval_pipeline import TinyVocabTokenizer
    cfg = tiny_gpu()
    cfg.vision_config.image_size = 336  # the prompt builders' labels cover 576 image slots (336 px / 14)
    m = CuLLaVOModel(cfg, device="cuda", trainable="none", init="random", seed=3)
    proc = CuLLaVOProcessor(TinyVocabTokenizer(), ClipImageProcessorHIP(shortest_edge=336, crop_size=336))
    net = CuLLaVO({"NAME": "cullavo_step1.yaml"}, m, proc)
    net.train()
    seen = {}
    fwd = net.forward_step

    def spy(b):
        seen.update({k: v.clone() for k, v in b.items() if torch.is_tensor(v)})
        return fwd(b)
    net.forward_step = spy
    random.seed(1)
    torch.manual_seed(1)
    with torch.no_grad():
        loss = net(step1_records(3))["loss_llm"]
    random.seed(1)
    torch.manual_seed(1)
    inputs = m.step1_process(step1_records(3), proc, torch.device("cuda"))
    assert inputs["pixel_values"].shape == (3, 3, 336, 336) and inputs["labels"].shape[0] == 3
    for k, v in seen.items():
        assert torch.equal(v, inputs[k]), k
    with torch.no_grad():
        ref = m(**inputs).loss
    assert torch.isfinite(loss).all() and float(loss) == float(ref)
    recs = step1_records(3)
    for r in recs:
        r["instances"].is_things = [False] * len(r["instances"].is_things)
    assert net(recs)["loss_llm"].tolist() == [0]
    # labels built for 576 image slots on a 224 px tower (256 slots): the reference's masked
    # indexing raises; so does the model (no out-of-range read of the mask)
    m224 = CuLLaVOModel(tiny_gpu(), device="cuda", trainable="none", init="random", seed=3)
    proc224 = CuLLaVOProcessor(TinyVocabTokenizer(), ClipImageProcessorHIP(shortest_edge=224, crop_size=224))
    bad = m224.step1_process(step1_records(3), proc224, torch.device("cuda"))
    with pytest.raises(IndexError):
        m224(**bad)
