"""Eval / step-2-pre entry points (SURVEY.md §3.4, §8(b) entry points; reference
modeling/architectures/cullavo_model.py:53-58,73-76, cullavo/arch_cullavo.py:341-395,
pipeline/CuLLaVOPipeline.py:95-133, trainer/default_trainer.py:51-71).

CPU: the box/class parser (reference cullavo/utils/utils.py:46-64) and the pass-through records of
step2_preprocess. GPU: greedy step2_preprocess generates the oracle's argmax tokens (full
recompute per step), and DefaultTrainer.eval -> evaluate_model writes the gathered entries.
"""
import json
import re
import zlib
from types import SimpleNamespace

import pytest
import torch

from oracle import cullavo_oracle as O


class TinyVocabTokenizer:
    """Words -> ids in the tiny configs' 1024-entry vocabulary: '<image>' 1000, pad 1001, BOS 1,
    '</s>' 2; decode writes 't<id>' words (skipping special ids)."""
    pad_token_id = 1001
    padding_side = "right"

    def encode(self, text, add_special_tokens=True):
        ids = [1] if add_special_tokens else []
        for part in re.split(r"(<image>|</s>)", text):
            if part == "<image>":
                ids.append(1000)
            elif part == "</s>":
                ids.append(2)
            else:
                ids += [3 + zlib.crc32(w.encode()) % 990 for w in part.split()]
        return ids

    def __call__(self, text, return_tensors="pt", add_special_tokens=True, **kw):
        return SimpleNamespace(input_ids=torch.tensor([self.encode(text, add_special_tokens)], dtype=torch.long))

    def batch_decode(self, seqs, skip_special_tokens=True, **kw):
        out = []
        for s in seqs:
            out.append(" ".join(f"t{int(i)}" for i in s if not (skip_special_tokens and int(i) in (1, 2, 1000, 1001))))
        return out


def test_box_and_class_parser():
    from cullavo_amd.prompting import box_and_class_parser
    txt = "Sure, it is person (#1) [0.100, 0.200, 0.300, 0.400], tv (#1) [0.5, 0.5, 0.9, 1.0]."
    boxes, classes, flag = box_and_class_parser(txt)
    assert not flag and classes == ["#1", "#1"]
    assert torch.allclose(boxes, torch.tensor([[0.1, 0.2, 0.3, 0.4], [0.5, 0.5, 0.9, 1.0]]))
    assert box_and_class_parser("person (#1) [0.1, 0.2")[2] is True  # unpaired bracket
    b, c, f = box_and_class_parser("a (x) [0.1, 0.2, 0.3]")  # 3 numbers: dropped like the reference
    assert not f and c == [] and b.numel() == 0
    with pytest.raises((ValueError, SyntaxError)):
        box_and_class_parser("a (x) [os.system, 1, 2, 3]")  # literal_eval: names are not evaluated


def test_step2_preprocess_passthrough_records():
    from cullavo_amd.prompting import step2_preprocess
    recs = [{"question_id": "q0", "question": [{"from": "human", "value": "hi"}]},
            {"question_id": "q1", "image_id": "a.jpg", "image": torch.zeros(3, 8, 8, dtype=torch.uint8),
             "question": [{"from": "human", "value": "<image> what?"}]}]
    out = step2_preprocess(None, recs, None, "cpu", dice=lambda r: 1)
    assert out == [{"id": "q0", "conversations": recs[0]["question"]},
                   {"id": "q1", "image": "a.jpg", "conversations": recs[1]["question"]}]


@pytest.mark.parametrize("n_boxes", [20, 21])
def test_step2_preprocess_more_boxes_than_colors(monkeypatch, n_boxes):
    """More parsed boxes than the reference's 20 colours: its overlay_instances call trips the
    labels-length assert and the bare except emits the record without boxes/classes
    (reference cullavo/arch_cullavo.py:376-389); 20 boxes still produce a box entry."""
    from cullavo_amd import prompting as P
    text = "Sure. " + ", ".join(f"obj{i} (#{i}) [0.{i:02d}0, 0.100, 0.500, 0.900]" for i in range(n_boxes))
    monkeypatch.setattr(P, "eval_process", lambda **kw: {})
    model = SimpleNamespace(config=SimpleNamespace(ignore_index=-100), generate=lambda **kw: torch.zeros(1, 3))
    proc = SimpleNamespace(batch_decode=lambda ids, skip_special_tokens=True: [text])
    rec = {"question_id": "q", "image_id": "a.jpg", "image": torch.zeros(3, 8, 8, dtype=torch.uint8),
           "question": [{"from": "human", "value": "<image>"}]}
    out = P.step2_preprocess(model, [rec], proc, "cpu", dice=lambda r: 0)
    base = {"id": "q", "image": "a.jpg", "conversations": rec["question"]}
    if n_boxes > len(P.COLOR_LIST):
        assert out == [base]
    else:
        assert out[0]["classes"] == [f"#{i}" for i in range(n_boxes)] and len(out[0]["boxes"]) == n_boxes


def test_step2_preprocess_visualisation_png(monkeypatch, tmp_path):
    """vis_dir: the record's image with its generated boxes (x 336) and class names is written to
    <vis_dir>/<question_id>.png (reference cullavo/arch_cullavo.py:376-386): right size, the
    box edges drawn in their colours, the labels on black boxes; the entry carries the boxes."""
    import numpy as np
    from PIL import Image
    from cullavo_amd import prompting as P
    text = "Sure. cat (#1) [0.100, 0.100, 0.600, 0.700], dog (#2) [0.500, 0.550, 0.950, 0.950]"
    monkeypatch.setattr(P, "eval_process", lambda **kw: {})
    model = SimpleNamespace(config=SimpleNamespace(ignore_index=-100), generate=lambda **kw: torch.zeros(1, 3))
    proc = SimpleNamespace(batch_decode=lambda ids, skip_special_tokens=True: [text])
    img = torch.full((3, 336, 336), 128, dtype=torch.uint8)
    rec = {"question_id": "q7", "image_id": "a.jpg", "image": img, "question": [{"from": "human", "value": "<image>"}]}
    out = P.step2_preprocess(model, [rec], proc, "cpu", dice=lambda r: 0, vis_dir=str(tmp_path))
    assert out[0]["classes"] == ["#1", "#2"] and len(out[0]["boxes"]) == 2
    png = np.asarray(Image.open(tmp_path / "q7.png").convert("RGB"))
    assert png.shape == (336, 336, 3)
    assert (png != 128).any(axis=2).mean() > 0.01          # boxes and labels were drawn
    assert (png[200, 33:36] != 128).any()                   # cat's left edge (x = 33.6) in white/red
    assert (png[:, :, :] < 60).all(axis=2).any()            # the labels' black boxes
    # a render that fails (here: an unreadable image) falls back to the record without boxes
    bad = dict(rec, question_id="q8", image=object())
    out = P.step2_preprocess(model, [bad], proc, "cpu", dice=lambda r: 0, vis_dir=str(tmp_path))
    assert out == [{"id": "q8", "image": "a.jpg", "conversations": rec["question"]}]


def _processor(size):
    from cullavo_amd.prompting import ClipImageProcessorHIP, CuLLaVOProcessor
    return CuLLaVOProcessor(TinyVocabTokenizer(), ClipImageProcessorHIP(shortest_edge=size, crop_size=size))


def _records(n, size=224, seed=0):
    g = torch.Generator().manual_seed(seed)
    return [{"question_id": f"q{i}", "image_id": f"{i}.jpg",
             "image": torch.randint(0, 256, (3, size + 16 * i, size), generator=g, dtype=torch.uint8),
             "question": [{"from": "human", "value": "<image>\ndescribe"}, {"from": "gpt", "value": "ok"}]}
            for i in range(n)]


@pytest.mark.gpu
def test_step2_preprocess_greedy_matches_oracle_argmax(monkeypatch):
    from cullavo_amd.arch_cullavo import CuLLaVOModel
    from cullavo_amd.config import tiny_gpu
    cfg = O.config_small_gpu()
    W = O.make_weights(cfg, 8)
    m = CuLLaVOModel(tiny_gpu(), device="cuda", trainable="none", init="none")
    m.load_state_dict(W)
    m.eval()
    proc = _processor(224)
    seen = []
    recs = _records(2)
    out = m.step2_preprocess(recs, proc, torch.device("cuda"), dice=lambda r: 0,
                             generate_kwargs=dict(do_sample=False, max_new_tokens=6),
                             on_generate=lambda rec, ids, text: seen.append((rec, ids.cpu(), text)))
    assert len(seen) == 2
    for rec, ids, text in seen:
        inputs = m.eval_process(images=rec["image"], prompt="x", processor=proc, device="cuda")
        S = ids.shape[1] - 6
        pix = proc.image_processor(rec["image"]).cpu()
        for i in range(6):  # each greedy token = the oracle's argmax of the full recompute
            prefix = ids[:, :S + i]
            _, lg, _ = O.forward(W, cfg, prefix, pix, torch.ones_like(prefix), None)
            last = lg[0, -1]
            tok = int(ids[0, S + i])
            top = torch.topk(last, 2).values
            assert tok == int(last.argmax()) or (last.max() - last[tok]).item() <= 2e-2 * (top[0] - last.min()).item()
        assert text == proc.batch_decode(ids)[0]
        del inputs
    # random weights write no brackets at all: nothing to pair, so (as in the reference) each
    # record is kept with empty boxes/classes; a generation that parses is kept with its boxes
    assert [(e["id"], e["boxes"], e["classes"]) for e in out] == [("q0", [], []), ("q1", [], [])]
    monkeypatch.setattr(proc, "batch_decode",
                        lambda ids, skip_special_tokens=True: ["bed (#1) [0.000, 0.580, 0.607, 1.000]"])
    out = m.step2_preprocess(recs[:1], proc, torch.device("cuda"), dice=lambda r: 0,
                             generate_kwargs=dict(do_sample=False, max_new_tokens=2))
    assert len(out) == 1 and out[0]["classes"] == ["#1"] and out[0]["id"] == "q0" and out[0]["image"] == "0.jpg"
    assert len(out[0]["boxes"]) == 1 and out[0]["boxes"][0] == pytest.approx([0.0, 0.58, 0.607, 1.0])


@pytest.mark.gpu
def test_trainer_eval_evaluate_model_writes_gathered_json(tmp_path):
    from cullavo_amd.trainer import CuLLaVO_Trainer
    recs = _records(3, seed=1)
    opt = {"NAME": "cullavo_step2_pre.yaml", "MODEL": {"NAME": "cullavo_model", "CONFIG": "tiny"},
           "LLM": {"TRAINABLE": "none"}, "DATASETS": {"TEST": ["lbk_pre"]},
           "DATA": {"BATCH_SIZE_PER_GPU": 2, "EVAL_RECORDS": {"lbk_pre": recs}},
           "EVAL_OUTPUT": str(tmp_path / "lbk_new_version.json"), "PROCESSOR": _processor(224)}
    tr = CuLLaVO_Trainer(opt)
    torch.manual_seed(0)
    out = tr.eval()
    ids = sorted(e["id"] for e in out)
    # the dice keeps ~1 in 50 records for generation; whatever it rolled, every record is
    # either passed through or (if generated and parsed) extended -- none is lost except flagged
    assert set(ids) <= {"q0", "q1", "q2"}
    assert json.load(open(tmp_path / "lbk_new_version.json")) == out
