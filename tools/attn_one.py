"""LM causal attention backward at the 7B step's shape (B=8, H=32, L=1088, D=128) in one
backward tile mode, a few launches: the program the attention PMC passes profile.

  python tools/attn_one.py [mode ...]     (default: 4 6)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cullavo_amd import _lib, ops  # noqa: E402

B, H, L, D = 8, 32, 1088, 128
modes = [int(m) for m in sys.argv[1:]] or [4, 6]
g = torch.Generator(device="cuda").manual_seed(0)
qkv = (torch.randn(B * L, 3 * H * D, device="cuda", generator=g) * 0.5).bfloat16()
q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
kw = dict(B=B, H=H, Lq=L, Lk=L, D=D, scale=D ** -0.5, causal=True)
o, lse = ops.attn_fwd(q, k, v, **kw)
do = torch.randn(o.shape, device="cuda", generator=g).bfloat16()
dqkv = torch.empty_like(qkv)
for mode in modes:
    _lib.lib().cullavo_attn_set_bwd_tiles(mode)
    for _ in range(int(os.environ.get("REPS", "2"))):
        ops.attn_bwd(q, k, v, o, do, lse, dq=dqkv[:, :H * D], dk=dqkv[:, H * D:2 * H * D], dv=dqkv[:, 2 * H * D:], **kw)
torch.cuda.synchronize()
print("ok")
