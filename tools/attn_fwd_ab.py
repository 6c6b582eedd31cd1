"""Forward-only A/B of the attention staging modes (cullavo_attn_set_stage) at the 7B layer and
ViT bs-64 shapes, alternating modes over several rounds (HIP-event timing, 20 launches each).

  python tools/attn_fwd_ab.py [rounds] [stage ...]      (default: 4 rounds, stages 4 7)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cullavo_amd import _lib, ops  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
stages = [int(x) for x in sys.argv[2:]] or [4, 7]
L_ = _lib.lib()
shapes = [("LM causal D128", 8, 1088, 32, 128, True), ("ViT D64", 64, 577, 16, 64, False)]
data = {}
for name, B, L, H, D, causal in shapes:
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = (torch.randn(B * L, 3 * H * D, device="cuda", generator=g) * 0.5).bfloat16()
    data[name] = (qkv, B, L, H, D, causal)
res = {(n, st): [] for n in data for st in stages}
for r in range(rounds):
    for st in stages:
        L_.cullavo_attn_set_stage(st)
        for name, (qkv, B, L, H, D, causal) in data.items():
            q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
            kw = dict(B=B, H=H, Lq=L, Lk=L, D=D, scale=D ** -0.5, causal=causal)
            for _ in range(3):
                ops.attn_fwd(q, k, v, **kw)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(20):
                ops.attn_fwd(q, k, v, **kw)
            e.record()
            e.synchronize()
            res[(name, st)].append(s.elapsed_time(e) / 20 * 1e3)
L_.cullavo_attn_set_stage(-1)
for (name, st), ts in res.items():
    print(f"{name:16s} stage {st}: " + " ".join(f"{t:6.1f}" for t in ts) + f"  min {min(ts):6.1f} us", flush=True)
