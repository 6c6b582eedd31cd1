"""The CPU oracle (oracle/cullavo_oracle.py) against golden vectors produced by the
reference's own CuLLaVOModel.forward (tests/golden/make_golden.py). This pins the oracle that
every GPU parity test uses as its checker."""
import os

import numpy as np
import pytest
import torch

from oracle import cullavo_oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")

CASES = {
    "config1": (O.config1, dict(batch=2, text_len=32, image_col=5, seed=0)),
    "config1_pad": (O.config1, dict(batch=2, text_len=32, image_col=5, seed=1, pad_tail=[0, 7])),
    "small_gpu": (O.config_small_gpu, dict(batch=2, text_len=40, image_col=4, seed=2)),
}


def _run(name):
    mk, kw = CASES[name]
    cfg = mk()
    W = {k: v.clone().requires_grad_(True) for k, v in O.make_weights(cfg, kw["seed"]).items()}
    ids, mask, pix, labels = O.make_inputs(cfg, kw["batch"], kw["text_len"], kw["image_col"], kw["seed"],
                                           pad_tail=kw.get("pad_tail"))
    loss, logits, aux = O.forward(W, cfg, ids, pix, mask, labels)
    loss.backward()
    return cfg, W, loss, logits, aux


@pytest.mark.parametrize("name", list(CASES))
def test_oracle_matches_reference_forward(name):
    g = np.load(os.path.join(GOLD, name + ".npz"))
    cfg, W, loss, logits, aux = _run(name)
    assert tuple(logits.shape) == tuple(g["logits_shape"])
    # fp32 vs fp32: only summation order differs
    assert abs(loss.item() - float(g["loss"][0])) < 1e-4 * max(1.0, abs(float(g["loss"][0])))
    rows = g["logits_rows"]
    sample = logits[:, rows].detach().numpy()
    ref = g["logits_sample"]
    valid = aux["attention_mask"][:, rows].numpy().astype(bool)
    err = np.abs(sample - ref)[valid].max()
    assert err < 2e-4 * np.abs(ref).max(), err
    np.testing.assert_allclose(logits.detach().norm(dim=-1).numpy(), g["logits_rownorm"], rtol=2e-5, atol=1e-4)


@pytest.mark.parametrize("name", list(CASES))
def test_oracle_grads_match_reference(name):
    g = np.load(os.path.join(GOLD, name + ".npz"))
    cfg, W, loss, logits, aux = _run(name)
    n = 0
    for key in g.files:
        if key.startswith("gradnorm/"):
            k = key[len("gradnorm/"):]
            ours = W[k].grad.norm().item() if W[k].grad is not None else 0.0
            ref = float(g[key][0])
            assert abs(ours - ref) <= 1e-4 * max(ref, 1e-6) + 1e-7, (k, ours, ref)
            n += 1
        if key.startswith("grad/"):
            k = key[len("grad/"):]
            stride = int(g["gradstride/" + k][0])
            ours = W[k].grad.reshape(-1)[::stride].numpy()
            np.testing.assert_allclose(ours, g[key], rtol=1e-3, atol=1e-6 * np.abs(g[key]).max())
    assert n > 10
