"""Where do images 0-1 of a ViT-L bs-64 batch stop matching the same images run alone? Compares
the attention forward bitwise at B = 64 vs B = 2, and the encoder's hidden states layer by layer
(rel-L2), with random weights (diagnostic for test_full_size's per-image independence check)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cullavo_amd import ops  # noqa: E402
from cullavo_amd.arena import ParamArena  # noqa: E402
from cullavo_amd.config import CLIPVisionConfig  # noqa: E402
from cullavo_amd.modeling import CLIPVisionTransformer, clip_specs  # noqa: E402


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


g = torch.Generator(device="cuda").manual_seed(1)
L, H, D = 577, 16, 64
for B in (64, 3):
    q, k, v = (torch.randn(B * L, 3 * H * D, device="cuda", generator=g).bfloat16() for _ in range(3))
    kw = dict(H=H, Lq=L, Lk=L, D=D, scale=D ** -0.5, causal=False)
    o_all, lse_all = ops.attn_fwd(q[:, :H * D], k[:, :H * D], v[:, :H * D], B=B, **kw)
    o_two, lse_two = ops.attn_fwd(q[:2 * L, :H * D].contiguous(), k[:2 * L, :H * D].contiguous(),
                                  v[:2 * L, :H * D].contiguous(), B=2, **kw)
    print(f"attn B={B} vs B=2 (strided vs contiguous): O max|d| {(o_all[:2 * L].float() - o_two.float()).abs().max().item():.3e}"
          f" lse {(lse_all[:2] - lse_two).abs().max().item():.3e}", flush=True)

vc = CLIPVisionConfig()
pre = "vision_tower.vision_model."
ar = ParamArena("vision", clip_specs(vc, pre), device="cuda", dtype=torch.bfloat16, trainable=False)
with torch.no_grad():
    ar.flat.normal_(0, 0.02, generator=torch.Generator(device="cuda").manual_seed(3))
vt = CLIPVisionTransformer(vc, ar.params, pre, ar)
pix = torch.randn(64, 3, 336, 336, device="cuda", generator=torch.Generator(device="cuda").manual_seed(4))
with torch.no_grad():
    for n in (0, 1, 2, 4, 8, 23):
        a = vt.hidden_state(pix, n)
        b = vt.hidden_state(pix[:2].contiguous(), n)
        print(f"layers {n:2d}: rel-L2 batch-64 vs alone {rel(b, a[:2]):.3e}  max|d| {(a[:2].float() - b.float()).abs().max().item():.3e}",
              flush=True)
