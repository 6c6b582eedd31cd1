"""CLIP image preprocessing (csrc/imageprep.hip) at the data-step shape: B=8 uint8 [3, 480, 640]
photos -> pixel_values [8, 3, 336, 336] f32, and a 64-image batch (HIP-event timing).
Algorithmic bytes: input read + tmp (uint8 [B, 3, H, 336]) write and read + output write."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cullavo_amd.prompting import ClipImageProcessorHIP  # noqa: E402

p = ClipImageProcessorHIP(device="cuda")
for B, H, W, dt in [(8, 480, 640, torch.float32), (64, 480, 640, torch.bfloat16), (64, 1024, 768, torch.bfloat16)]:
    x = torch.randint(0, 256, (B, 3, H, W), dtype=torch.uint8, device="cuda")
    out = torch.empty((B, 3, 336, 336), dtype=dt, device="cuda")
    for _ in range(3):
        p.preprocess_batch(x, out=out)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        p.preprocess_batch(x, out=out)
    e.record()
    e.synchronize()
    us = s.elapsed_time(e) / 20 * 1e3
    byt = x.numel() + 2 * B * 3 * H * 336 + out.numel() * out.element_size()
    print(f"B={B:3d} {H}x{W} -> 336 {str(dt):15s} {us:8.1f} us  {byt / us / 1e3:7.1f} GB/s  "
          f"{B / us * 1e6:10.0f} images/s")
