"""Data step, text half: prompt / label construction and the lbk.json
records. Fixtures: the REFERENCE's own make_system_prompt / make_and_add_prompt_and_label /
step2_process over tests/toy_tokenizer.py (tests/golden/make_golden_data.py). CPU only: the
image processor is replaced by a pass-through here (it has its own tests in test_imageprep.py)."""
import json
import os
import sys

import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

from oracle import data_oracle as D  # noqa: E402
from tests.toy_tokenizer import ToyTokenizer  # noqa: E402

GOLD = json.load(open(os.path.join(HERE, "golden", "data_step.json")))


class _PassThroughImages:
    def __call__(self, images):
        return images.float()


def _processor(side="right"):
    from cullavo_amd.prompting import CuLLaVOProcessor
    return CuLLaVOProcessor(ToyTokenizer(side), image_processor=_PassThroughImages())


def test_system_prompt_and_turn_match_reference():
    from cullavo_amd import prompting as P
    g = GOLD["prompts"]["single"]
    proc = _processor()
    p, lab = P.make_system_prompt(proc, "cpu", -100)
    assert p == g["system_prompt"] and len(lab) == g["system_label_len"]
    p2, lab2 = P.make_and_add_prompt_and_label(p, lab, "What is it?", "A dog.", proc, "cpu", -100)
    assert p2 == g["prompt"] and lab2.tolist() == g["label"]


@pytest.mark.parametrize("side", ["right", "left"])
def test_step2_process_matches_reference(side):
    from cullavo_amd import prompting as P
    g = GOLD["prompts"][side]
    batch = [dict(r, image=torch.zeros(3, 8, 8, dtype=torch.uint8)) for r in GOLD["records"]]
    out = P.step2_process(batch, _processor(side), "cpu")
    assert out["input_ids"].tolist() == g["input_ids"]
    assert out["attention_mask"].tolist() == g["attention_mask"]
    assert out["labels"].tolist() == g["labels"]
    assert out["pixel_values"].shape == (3, 3, 8, 8)
    assert set(out) >= {"position_ids", "past_key_values", "use_cache", "return_dict"}


def test_oracle_restatement_matches_reference_labels():
    tok = ToyTokenizer()
    g = GOLD["prompts"]["right"]
    for rec, labels in zip(GOLD["records"], g["labels"]):
        _, lab = D.conversation_prompt(rec["question"], tok.encode)
        assert labels[:len(lab)] == lab and all(x == -100 for x in labels[len(lab):])


def test_supervised_tokens_follow_the_answers():
    """every supervised label is an answer token or '</s>'; the image slots and prompts are -100"""
    from cullavo_amd import prompting as P
    tok = ToyTokenizer()
    rec = GOLD["records"][1]
    out = P.step2_process([dict(rec, image=torch.zeros(3, 8, 8, dtype=torch.uint8))], _processor(), "cpu")
    sup = [x for x in out["labels"][0].tolist() if x != -100]
    answers = []
    for k in range(len(rec["question"]) // 2):
        answers += tok.encode(str(rec["question"][2 * k + 1]["value"]) + "</s>", False)
    assert sup == answers
    # merged length = text tokens + 575 image slots
    assert out["labels"].shape[1] == out["input_ids"].shape[1] + 575


def test_box_records_need_an_image_and_helpers():
    from cullavo_amd import prompting as P
    # a record with boxes but no image fails like the reference's batch['image'] (:442)
    with pytest.raises(KeyError):
        P.step2_process([dict(GOLD["records"][0], boxes=[[0, 0, 1, 1]])], _processor(), "cpu",
                        draw=lambda img, b, c: img)
    assert P.list2string(["red", "blue", 3]) == "red, blue, 3"
    assert P.box2string(torch.tensor([0.12345, 0.5, 1.0, 0.0004])) == "[0.123, 0.500, 1.000, 0.000]"


def test_load_lbk_records(tmp_path):
    from cullavo_amd import prompting as P
    (tmp_path / "img").mkdir()
    (tmp_path / "img" / "a.jpg").write_bytes(b"x")
    recs = [{"id": 1, "image": "a.jpg", "conversations": GOLD["records"][0]["question"]},
            {"id": 2, "image": "missing.jpg", "conversations": []},
            {"id": 3, "image": "a.jpg", "boxes": [[0, 0, 1, 1]], "conversations": []},
            {"id": 4, "conversations": GOLD["records"][1]["question"]}]
    path = tmp_path / "lbk.json"
    path.write_text(json.dumps(recs))
    out = P.load_lbk_records(str(path), str(tmp_path / "img"))
    assert [r["question_id"] for r in out] == [1, 3, 4]
    assert out[0]["image_id"] == "a.jpg" and "boxes" in out[1] and "image_id" not in out[2]
    path.write_text(json.dumps(recs[1:2]))
    with pytest.raises(AssertionError):
        P.load_lbk_records(str(path), str(tmp_path / "img"))


@pytest.mark.gpu
def test_step2_process_on_gpu_with_hip_image_processor():
    """records with real uint8 images -> step2_process on the GPU: ids / labels as the reference,
    pixel_values bit-identical to transformers' processor"""
    import hashlib
    import numpy as np
    from cullavo_amd import prompting as P
    sys.path.insert(0, os.path.join(HERE, "golden"))
    from make_golden_data import case_image
    c = next(x for x in json.load(open(os.path.join(HERE, "golden", "data_step.json")))["images"]
             if x["H"] == 480)
    img = torch.from_numpy(case_image(c["seed"], c["H"], c["W"]))
    proc = P.CuLLaVOProcessor(ToyTokenizer(), P.ClipImageProcessorHIP(device="cuda"))
    batch = [dict(r, image=img) for r in GOLD["records"]]
    out = P.step2_process(batch, proc, "cuda")
    g = GOLD["prompts"]["right"]
    assert out["input_ids"].tolist() == g["input_ids"] and out["labels"].tolist() == g["labels"]
    for pv in out["pixel_values"]:
        assert hashlib.sha256(pv.cpu().numpy().astype(np.float32).tobytes()).hexdigest() == c["sha256"]


def test_pipeline_forward_step_on_raw_step2_records():
    """CuLLaVOPipeline.forward_step on the reference's collate=list batches (raw lbk records):
    the records go through step2_process, the loss is backpropagated and num_samples is
    len(batch) (reference pipeline/CuLLaVOPipeline.py:76-93, :85). The model is a host stub
    (the GPU model has its own tests); this pins the pipeline plumbing."""
    import types
    from torch import nn
    from cullavo_amd import prompting as P
    from cullavo_amd.pipeline import CuLLaVO, CuLLaVOPipeline

    class _StubModel(nn.Module):
        def __init__(self):
            super().__init__()
            self.w = nn.Parameter(torch.ones(()))
            self.arenas = {}
            self.seen = None

        def step2_process(self, batch, processor, device):
            return P.step2_process(batch, processor, device)

        def forward(self, input_ids=None, labels=None, **kw):
            self.seen = input_ids
            return types.SimpleNamespace(loss=self.w * (labels != -100).sum().float())

    stub = _StubModel()
    model = CuLLaVO({"NAME": "cullavo_step2.yaml"}, stub, cullavo_processor=_processor())
    model.train()
    calls = []
    accel = types.SimpleNamespace(device=torch.device("cpu"), sync_gradients=True,
                                  clip_grad_norm_=lambda p, m: calls.append(("clip", m)))
    trainer = types.SimpleNamespace(model=types.SimpleNamespace(cullavo_model=stub), accel=accel)
    trainer.compute_loss = lambda f, b: f(trainer, b)
    trainer.backward_loss = lambda loss: (loss.backward(), calls.append("backward"))
    trainer.update_model = lambda: calls.append("update")
    pipe = CuLLaVOPipeline({"OPTIMIZER": {"GRAD_MAX": 10.0}})
    pipe.forward_func = lambda tr, b: model(b, tr.accel)  # instance attribute: not bound
    batch = [dict(r, image=torch.zeros(3, 8, 8, dtype=torch.uint8)) for r in GOLD["records"]]
    loss_info, size_info, _ = pipe.forward_step(trainer, batch)
    assert size_info == {"num_samples": len(batch)}
    assert stub.seen.tolist() == GOLD["prompts"]["right"]["input_ids"]
    n_sup = sum(x != -100 for row in GOLD["prompts"]["right"]["labels"] for x in row)
    assert float(loss_info["loss_llm"]) == n_sup and float(stub.w.grad) == n_sup
    assert calls == ["backward", ("clip", 10.0), "update"]
