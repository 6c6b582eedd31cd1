"""bf16 noise floor of the 23-layer CLIP ViT-L/14-336 forward (tests/test_full_size.py's gate):
the bf16-faithful oracle run twice with the SAME rounding points but a different accumulation
order inside every Linear (native bf16 matmul vs f32 matmul rounded to bf16). The two differ by
rel-L2 ~1.1e-2 after 23 layers (measured: 1.09e-2; bf16 vs fp32: 1.14e-2), so a kernel/oracle
gap of that size is accumulation order, not a rounding-point or indexing error.

  python tools/bf16_noise_floor.py
"""
import sys, torch, time
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from oracle import cullavo_oracle as O
import torch.nn.functional as F
cfg = O.config_7b(); v = cfg.vision
W = {}
for k,(shp,kind) in O.weight_shapes(cfg).items():
    if k.startswith('vision_tower'): W[k] = O.init_tensor(k, shp, kind, 3)
Wb = O.to_bf16(W)
g = torch.Generator().manual_seed(4)
pix = torch.randn(2,3,336,336, generator=g).bfloat16()
t=time.time()
a = O.vision_hidden_states(pix, Wb, v, 23)[23]
print('bf16 run', time.time()-t)
# same rounding points, different accumulation: F.linear via f32 math rounded to bf16
orig = F.linear
def lin32(x, w, b=None):
    y = orig(x.float(), w.float(), None if b is None else b.float())
    return y.to(x.dtype)
O.F.linear = lin32
b = O.vision_hidden_states(pix, Wb, v, 23)[23]
O.F.linear = orig
rel = ((a.double()-b.double()).norm()/b.double().norm()).item()
f = O.vision_hidden_states(pix.float(), W, v, 23)[23]
print('accum-order-only rel-L2', rel, ' bf16 vs fp32', ((a.double()-f.double()).norm()/f.double().norm()).item())
