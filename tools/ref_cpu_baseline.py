"""The REFERENCE's own CPU path timed on this host (VERDICT r05 "What's missing" item 3): the
reference's CuLLaVOModel.forward (/root/reference/cullavo/arch_cullavo.py:546-677, run unmodified
through the shim of tests/golden/make_golden.py) + loss.backward() at config-3 widths
(ViT-L/14-336 + Vicuna-7B, one sample: 336 px image + 513 text tokens -> L = 1088), the full
fine-tune's trainable set (vision frozen: no vision gradients are requested, as in the step).

The whole 7B model does not fit this 64 GiB container in fp32 with gradients, so the per-sample
time is assembled from the reference's own code at reduced depth: the same model with 1 and with 2
decoder layers (their difference is one decoder layer's forward + backward), and the vision tower's
own forward (no autograd: the tower is frozen) with 2 and 3 CLIP layers (one CLIP layer), then
  t_sample = t(1 LM, 2 ViT) + 31 x d_LM + 22 x d_ViT   (32 LM layers, the 23 ViT layers the step runs).
Run here, in the build container (the reference is not on the GPU box): writes the record to
profiles/r06/ref_cpu_baseline.json. bench.py's cpu_baseline (kind "port") is the oracle timed on the
GPU box's host; this record is the reference itself on this container's cores.

  python tools/ref_cpu_baseline.py [--threads 8] [--dtype fp32|bf16|both]
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))

from oracle import cullavo_oracle as O  # noqa: E402


def timed_step(n_lm: int, n_vit: int, dtype: torch.dtype, reps: int, vit_only: bool = False) -> float:
    import make_golden as MG  # the reference shim (imports /root/reference)
    cfg = O.config_7b()
    cfg.text.num_hidden_layers = n_lm
    cfg.vision.num_hidden_layers = n_vit
    W = O.make_weights(cfg, 0)
    if dtype != torch.float32:
        W = {k: v.to(dtype) for k, v in W.items()}
    ids, mask, pix, labels = O.make_inputs(cfg, 1, 513, 35, 0)
    model = MG.build_reference_model(cfg, W)
    if dtype != torch.float32:
        model = model.to(dtype)
        pix = pix.to(dtype)
    for n, p_ in model.named_parameters():  # the step's trainable set: vision tower frozen
        p_.requires_grad_(not n.startswith("model.vision_tower."))
    del W

    def step():
        model.zero_grad(set_to_none=True)
        out = model(input_ids=ids, pixel_values=pix, attention_mask=mask, labels=labels, return_dict=True)
        out.loss.backward()

    def vit():  # the reference's vision call (arch_cullavo.py:586-597), frozen: no autograd
        with torch.no_grad():
            model.vision_tower(pix, output_hidden_states=True)

    fn = vit if vit_only else step
    fn()  # warm
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    del model
    return sorted(ts)[len(ts) // 2]  # median


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    ap.add_argument("--dtype", default="both", choices=["fp32", "bf16", "both"])
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    out = {"what": "reference CuLLaVOModel.forward + backward (vision frozen), one config-3 sample "
                   "(336 px + 513 tokens, L = 1088), timed at reduced depth and assembled per layer",
           "threads": a.threads, "cpu": platform.processor() or platform.machine(),
           "torch": torch.__version__, "results": {}}
    try:
        out["cpu_model"] = [ln.split(":", 1)[1].strip() for ln in open("/proc/cpuinfo") if ln.startswith("model name")][0]
    except (OSError, IndexError):
        pass
    dts = {"fp32": [torch.float32], "bf16": [torch.bfloat16], "both": [torch.float32, torch.bfloat16]}[a.dtype]
    for dt in dts:
        name = "fp32" if dt == torch.float32 else "bf16"
        t11 = timed_step(1, 2, dt, a.reps)
        t21 = timed_step(2, 2, dt, a.reps)
        # one CLIP layer from the vision tower's own forward at 2 and 3 layers (5 reps: it is short)
        d_vit = timed_step(1, 3, dt, 5, vit_only=True) - timed_step(1, 2, dt, 5, vit_only=True)
        d_lm = t21 - t11
        sample = t11 + 31 * d_lm + 22 * d_vit
        out["results"][name] = {"t_1lm_1vit_s": round(t11, 3), "lm_layer_fwd_bwd_s": round(d_lm, 3),
                                "vit_layer_fwd_s": round(d_vit, 3), "sample_s": round(sample, 2),
                                "samples_per_s": 1.0 / sample}
        print(name, out["results"][name], flush=True)
    path = os.path.join(REPO, "profiles", "r06", "ref_cpu_baseline.json")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(path)


if __name__ == "__main__":
    main()
