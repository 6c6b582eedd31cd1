"""RMSNorm forward/backward at the config-3 shape (8704 x 4096 bf16) with HIP-event timing:
effective HBM rate of each kernel against ~6 TB/s achievable."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cullavo_amd import _lib, ops  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


rows, cols = 8704, 4096
x = torch.randn(rows, cols, device="cuda").bfloat16()
dy = torch.randn_like(x)
dres = torch.randn_like(x)
w = torch.ones(cols, device="cuda").bfloat16()
y, rstd = ops.rmsnorm_fwd(x, w, 1e-5)
dw = torch.empty(cols, device="cuda", dtype=torch.bfloat16)
nb = rows * cols * 2
ms = timeit(lambda: ops.rmsnorm_fwd(x, w, 1e-5))
print(f"rmsnorm fwd          {ms * 1e3:8.1f} us  {2 * nb / ms / 1e9:6.2f} TB/s")
L = _lib.lib()
for mode in (1, 0, 1, 0):  # cullavo_rmsnorm_set_bwd: 1 pipelined (default), 0 round-1 kernel
    prev = L.cullavo_rmsnorm_set_bwd(mode)
    for name, fn, nbytes in [("bwd", lambda: ops.rmsnorm_bwd(dy, x, w, rstd), 3 * nb),
                             ("bwd+dres", lambda: ops.rmsnorm_bwd(dy, x, w, rstd, dres=dres), 4 * nb),
                             ("bwd+dres+dw", lambda: ops.rmsnorm_bwd(dy, x, w, rstd, dres=dres, dw=dw), 4 * nb)]:
        ms = timeit(fn)
        print(f"rmsnorm {name:12s} mode {mode} {ms * 1e3:8.1f} us  {nbytes / ms / 1e9:6.2f} TB/s")
    L.cullavo_rmsnorm_set_bwd(prev)
