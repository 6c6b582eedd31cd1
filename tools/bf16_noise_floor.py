"""bf16 noise floor of the parity gates: the bf16-faithful oracle run twice with the SAME rounding
points but a different accumulation order inside every bf16 product (the oracle's f32-accumulate
/ round-once GEMM arithmetic vs torch's native CPU bf16 matmul). A kernel/oracle gap of that size
is accumulation order, not a rounding-point or indexing error.

  python tools/bf16_noise_floor.py small   # smoke()'s config (tests/test_model_gpu.py gates)
  python tools/bf16_noise_floor.py vit     # 23-layer CLIP ViT-L/14-336 (tests/test_full_size.py)

Measured (this container's Xeon): small -- f32 vs f64 accumulation inside every Linear (same
rounding points, only which bf16 outputs flip by one ulp differs) moves the logits by rel-L2
7.0e-3 (|dloss| 9.9e-4); torch's native CPU bf16 matmul by 8.2e-3; the bf16-faithful oracle vs
fp32 is 1.06e-2. The GPU's smoke() distance to the bf16-faithful oracle, 9.2e-3 (MI355X), sits
at 1.1-1.3x these floors. vit -- 1.09e-2 after 23 layers (native vs f32 accumulation).
"""
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import cullavo_oracle as O  # noqa: E402


def native_linear(x, w, b=None):
    return F.linear(x, w, b)


def f64_linear(x, w, b=None):
    if x.dtype == torch.bfloat16:
        return F.linear(x.double(), w.double(), None if b is None else b.double()).to(torch.bfloat16)
    return F.linear(x, w, b)


def rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm()).item()


def small():
    cfg = O.config_small_gpu()
    W = O.make_weights(cfg, 2)
    ids, mask, pix, labels = O.make_inputs(cfg, 2, 40, 4, 2)
    Wb = O.to_bf16(W)
    la, a, _ = O.forward(Wb, cfg, ids, pix, mask, labels)
    acc = O.linear
    for name, fn in (("f64-accumulated Linear", f64_linear), ("native CPU bf16 Linear", native_linear)):
        O.linear = fn
        lb, b, _ = O.forward(Wb, cfg, ids, pix, mask, labels)
        O.linear = acc
        print(f"small_gpu: {name} vs the oracle's f32 accumulation: logits rel-L2 {rel(a.float(), b.float()):.3e} "
              f"|dloss| {abs(la.item() - lb.item()):.3e}")
    lf, f, _ = O.forward(W, cfg, ids, pix, mask, labels)
    print(f"small_gpu: bf16-faithful vs fp32 logits {rel(a.float(), f.float()):.3e} |dloss| {abs(la.item() - lf.item()):.3e}")


def vit():
    cfg = O.config_7b()
    v = cfg.vision
    W = {k: O.init_tensor(k, shp, kind, 3) for k, (shp, kind) in O.weight_shapes(cfg).items()
         if k.startswith("vision_tower")}
    Wb = O.to_bf16(W)
    pix = torch.randn(2, 3, 336, 336, generator=torch.Generator().manual_seed(4)).bfloat16()
    t = time.time()
    a = O.vision_hidden_states(pix, Wb, v, 23)[23]
    print("bf16 run", time.time() - t)
    acc = O.linear
    O.linear = native_linear
    b = O.vision_hidden_states(pix, Wb, v, 23)[23]
    O.linear = acc
    f = O.vision_hidden_states(pix.float(), W, v, 23)[23]
    print(f"vit-L 23 layers: accumulation-order-only rel-L2 {rel(a, b):.3e}; bf16 vs fp32 {rel(a, f):.3e}")


if __name__ == "__main__":
    {"small": small, "vit": vit}[sys.argv[1] if len(sys.argv) > 1 else "small"]()
