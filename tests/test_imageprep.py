"""Data step, image half: CLIP image preprocessing.

CPU: the oracle's Pillow/transformers restatement against the fixtures made with transformers'
CLIPImageProcessorPil (tests/golden/make_golden_data.py), and the C-ABI's host coefficient
builder (cullavo_resample_coeffs, no GPU) against the oracle's. GPU: csrc/imageprep.hip through
the C-ABI against the same fixtures, bit for bit (sha256 of the f32 pixel_values), batched,
strided (HWC views) and bf16.
"""
import ctypes
import hashlib
import json
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(HERE, "golden"))

from make_golden_data import case_image  # noqa: E402
from oracle import data_oracle as D  # noqa: E402

GOLD = json.load(open(os.path.join(HERE, "golden", "data_step.json")))
CASES = GOLD["images"]


def _sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.float32).tobytes()).hexdigest()


@pytest.mark.parametrize("c", CASES, ids=lambda c: f"{c['H']}x{c['W']}->{c['crop']}")
def test_oracle_matches_transformers_processor(c):
    img = case_image(c["seed"], c["H"], c["W"])
    pv = D.clip_preprocess(img[None], c["shortest_edge"], (c["crop"], c["crop"]))[0]
    assert _sha(pv) == c["sha256"]


@pytest.mark.parametrize("n_in,n_out", [(336, 336), (640, 448), (427, 336), (300, 504), (1024, 336),
                                        (91, 162), (50, 64), (5000, 336), (1, 7)])
def test_host_resample_coeffs_match_oracle(n_in, n_out):
    from cullavo_amd import _lib
    L = _lib.lib()
    ks = L.cullavo_resample_coeffs(n_in, n_out, None, None, 0)
    bounds = np.zeros(2 * n_out, np.int32)
    kk = np.zeros(n_out * ks, np.int32)
    assert L.cullavo_resample_coeffs(n_in, n_out, bounds.ctypes.data_as(ctypes.c_void_p),
                                     kk.ctypes.data_as(ctypes.c_void_p), ks) == ks
    rb, rk = D.resample_coeffs(n_in, n_out)
    assert rk.shape[1] == ks
    np.testing.assert_array_equal(bounds.reshape(-1, 2), rb)
    np.testing.assert_array_equal(kk.reshape(n_out, ks), rk)
    assert L.cullavo_resample_coeffs(0, n_out, None, None, 0) == 1  # CULLAVO_EINVAL


def test_resize_output_size_matches_oracle():
    from cullavo_amd.prompting import resize_output_size
    for H, W in [(336, 336), (480, 640), (640, 427), (1000, 336), (37, 91), (91, 37)]:
        assert resize_output_size(H, W, 336) == D.resize_output_size(H, W, 336)


# ---- GPU ---------------------------------------------------------------------------------------
def _proc(c, **kw):
    from cullavo_amd.prompting import ClipImageProcessorHIP
    return ClipImageProcessorHIP(shortest_edge=c["shortest_edge"], crop_size=c["crop"], device="cuda", **kw)


@pytest.mark.gpu
@pytest.mark.parametrize("c", CASES, ids=lambda c: f"{c['H']}x{c['W']}->{c['crop']}")
def test_gpu_preprocess_bit_exact(c):
    img = torch.from_numpy(case_image(c["seed"], c["H"], c["W"]))
    batch = torch.stack([img, img.flip(-1)]).cuda()  # second image: a mirrored copy
    pv = _proc(c)(batch)
    torch.cuda.synchronize()
    assert pv.shape == (2, 3, c["crop"], c["crop"]) and pv.dtype == torch.float32
    assert _sha(pv[0].cpu().numpy()) == c["sha256"]
    ref1 = D.clip_preprocess(img.flip(-1).numpy()[None], c["shortest_edge"], (c["crop"], c["crop"]))[0]
    assert torch.equal(pv[1].cpu(), torch.from_numpy(ref1))


@pytest.mark.gpu
def test_gpu_preprocess_strided_hwc_bf16_and_ragged_list():
    c = CASES[1]
    img = case_image(c["seed"], c["H"], c["W"])
    hwc = torch.from_numpy(np.ascontiguousarray(img.transpose(1, 2, 0))).cuda()
    view = hwc.permute(2, 0, 1)[None]  # [1, 3, H, W] with channel stride 1
    p = _proc(c)
    f32 = p(view)
    assert _sha(f32[0].cpu().numpy()) == c["sha256"]
    bf = p.preprocess_batch(view, out_dtype=torch.bfloat16)
    assert torch.equal(bf, f32.to(torch.bfloat16))
    # a list of differently sized images -> one launch per size, order kept
    imgs = [torch.from_numpy(case_image(x["seed"], x["H"], x["W"])) for x in CASES[:5]]
    out = p([imgs[1], imgs[0], imgs[3], imgs[1]])
    for got, src in zip(out, [1, 0, 3, 1]):
        assert _sha(got.cpu().numpy()) == CASES[src]["sha256"]


@pytest.mark.gpu
def test_gpu_preprocess_empty_and_bad_crop():
    from cullavo_amd.prompting import ClipImageProcessorHIP
    p = ClipImageProcessorHIP(device="cuda")
    assert p(torch.zeros(0, 3, 400, 500, dtype=torch.uint8, device="cuda")).shape == (0, 3, 336, 336)
    bad = ClipImageProcessorHIP(shortest_edge=64, crop_size=96, device="cuda")
    with pytest.raises(ValueError):
        bad(torch.zeros(1, 3, 64, 64, dtype=torch.uint8, device="cuda"))
