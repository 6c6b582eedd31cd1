"""Flash attention forward / backward at the production shapes (HIP-event timing):
LM causal D=128 (B=8, L=1088, H=32) and CLIP non-causal D=64 (B=64, T=577, H=16).
Algorithmic FLOPs: fwd 4*B*H*Lq*Lk*D (x1/2 causal), bwd 2.5x fwd."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cullavo_amd import _lib, ops  # noqa: E402


def timeit(fn, iters=10):
    for _ in range(2):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


STAGES = [int(x) for x in os.environ.get("ATTN_STAGE_AB", "2").split(",")]  # e.g. 2,4,2,4
ref_out = {}
for stage in STAGES:
  if len(STAGES) > 1:
    _lib.lib().cullavo_attn_set_stage(stage % 10)
    _lib.lib().cullavo_attn_set_bwd_stage(stage // 10)  # e.g. 14 = forward stage 4 + dK/dV DMA
  for name, B, L, H, D, causal in [("LM causal D128", 8, 1088, 32, 128, True), ("ViT D64", 64, 577, 16, 64, False)]:
    torch.manual_seed(0)
    qkv = (torch.randn(B * L, 3 * H * D, device="cuda") * 0.5).bfloat16()
    q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
    o, lse = ops.attn_fwd(q, k, v, B=B, H=H, Lq=L, Lk=L, D=D, scale=D ** -0.5, causal=causal)
    do = torch.randn_like(o)
    dqkv = torch.empty_like(qkv)
    fl = 4.0 * B * H * L * L * D * (0.5 if causal else 1.0)
    tf = timeit(lambda: ops.attn_fwd(q, k, v, B=B, H=H, Lq=L, Lk=L, D=D, scale=D ** -0.5, causal=causal))
    res = []
    outs = {}
    for mode in (4, 7, 8, 1, 2):  # 4 = 8-wave dK/dV + 4-wave dQ, 7 = 8-wave dK/dV storing dS + dQ from it, 8 = 7 with the pipelined dK/dV, 1 / 2 = 4-wave
        _lib.lib().cullavo_attn_set_bwd_tiles(mode)
        tb = timeit(lambda: ops.attn_bwd(q, k, v, o, do, lse, B=B, H=H, Lq=L, Lk=L, D=D, scale=D ** -0.5,
                                         causal=causal, dq=dqkv[:, :H * D], dk=dqkv[:, H * D:2 * H * D],
                                         dv=dqkv[:, 2 * H * D:]))
        outs[mode] = dqkv.float().clone()
        res.append(f"m{mode} {tb * 1e3:7.1f} us {2.5 * fl / tb / 1e9:6.1f} TF")
    diff = ((outs[4] - outs[1]).norm() / outs[1].norm()).item()
    res.append(f"rel(m4, m1) {diff:.1e} rel(m7, m1) {((outs[7] - outs[1]).norm() / outs[1].norm()).item():.1e} "
               f"rel(m8, m1) {((outs[8] - outs[1]).norm() / outs[1].norm()).item():.1e}")
    key = name
    cur = (o.float().clone(), outs[7])
    if key in ref_out:
        res.append(f"bitwise equal across staging: {torch.equal(ref_out[key][0], cur[0]) and torch.equal(ref_out[key][1], cur[1])}")
    else:
        ref_out[key] = cur
    _lib.lib().cullavo_attn_set_bwd_tiles(-1)
    tag = f"stage {stage} " if len(STAGES) > 1 else ""
    print(f"{tag}{name:16s} fwd {tf * 1e3:8.1f} us {fl / tf / 1e9:7.1f} TF | bwd " + " | ".join(res), flush=True)
