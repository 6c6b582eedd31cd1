"""Fused AdamW + global-norm clipping over the flat gradient arenas.

Semantics of the reference's update (reference pipeline/CuLLaVOPipeline.py:88-92,
trainer/cullavo_trainer.py:12-14, trainer/default_trainer.py:86-90): clip_grad_norm_ to
GRAD_MAX over all trainable parameters, then torch.optim.AdamW(lr, weight_decay) and a
CosineAnnealingLR schedule. Here the clip coefficient never leaves the GPU: the sum of squares
of every gradient arena accumulates into one device scalar, cullavo_clip_coef turns it into
min(1, max_norm/(norm+1e-6)) and cullavo_adamw multiplies it into the gradient as it reads it
— no host sync, no extra pass over 13.5 GB of gradients.

overlap=True (the trainer's default on the GPU): the update kernels go to a side HIP stream,
one launch per decoder layer in forward order, each followed by an event the arena keeps
(ParamArena.defer); the next step's forward waits per layer (ParamArena.wait_update) instead of
for the whole update, so the HBM-bound AdamW (~17 ms of a 7B full fine-tune step) runs under
the compute-bound forward GEMMs of the layers before it. Same kernels on the same data in the
same order: bitwise equal to overlap=False (tests/test_model_gpu.py).
"""
from __future__ import annotations

import torch

from . import ops
from .arena import ParamArena


class FusedAdamW(torch.optim.Optimizer):
    """torch.optim.Optimizer subclass (so torch LR schedulers drive param_groups[0]['lr'])."""

    # the order the forward consumes the arenas in (side-stream launch order)
    FORWARD_ORDER = ("embed", "vision", "lora", "projector", "layers", "head")

    def __init__(self, arenas: list[ParamArena], lr: float = 2e-5, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, state_dtype=torch.bfloat16, overlap: bool = False):
        # state dtype defaults to the parameter dtype, as torch.optim.AdamW does for the
        # reference's bf16-cast parameters (reference cullavo/load_cullavo.py:123-126);
        # pass torch.float32 for f32 moments
        self.arenas = [a for a in arenas if a.trainable]
        params = [p for a in self.arenas for p in a.params.values()]
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.flat_state = [(torch.zeros(a.numel, dtype=state_dtype, device=a.device),
                            torch.zeros(a.numel, dtype=state_dtype, device=a.device)) for a in self.arenas]
        self.step_count = 0
        # per-key step counts (torch keeps state['step'] per parameter): a key skipped in a
        # cycle (no gradient, arena.skipped) neither moves nor advances its bias correction
        self.key_steps = [{k: 0 for k in a.offsets} for a in self.arenas]
        dev = self.arenas[0].device if self.arenas else torch.device("cpu")
        self._sumsq = torch.zeros(1, dtype=torch.float32, device=dev)
        self._coef = torch.ones(1, dtype=torch.float32, device=dev)
        self._norm = torch.zeros(1, dtype=torch.float32, device=dev)
        self._clip_pending = False
        self.overlap = bool(overlap) and dev.type == "cuda"
        self._stream = torch.cuda.Stream(device=dev) if self.overlap else None

    def synchronize(self):
        """Make the current stream wait for every pending side-stream update (before reading
        parameters outside a forward: evaluation, checkpoints, comparisons)."""
        for a in self.arenas:
            a.wait_update()

    @staticmethod
    def _layer_prefix(key: str) -> str:
        head, tail = key.split(".layers.", 1)
        return f"{head}.layers.{tail.split('.', 1)[0]}."

    def _chunks(self, a, lo, hi):
        """split [lo, hi) at decoder-layer boundaries (per-layer events for the layers arena)"""
        if a.name != "layers":
            return [(lo, hi)]
        cuts = getattr(a, "_layer_cuts", None)
        if cuts is None:
            cuts = a._layer_cuts = sorted({a.span(self._layer_prefix(k))[0] for k in a.offsets if ".layers." in k})
        out, cur = [], lo
        for c in cuts:
            if cur < c < hi:
                out.append((cur, c))
                cur = c
        out.append((cur, hi))
        return out

    def clip_grad_norm_(self, max_norm: float) -> torch.Tensor:
        """Global L2 norm over every trainable gradient (device scalar); the clip factor is
        applied inside the next step()."""
        self._sumsq.zero_()
        for a in self.arenas:
            ops.sumsq(a.grad_flat, self._sumsq)
        ops.clip_coef(self._sumsq, float(max_norm), self._coef, self._norm)
        self._clip_pending = True
        return self._norm

    @torch.no_grad()
    def step(self, closure=None):
        self.step_count += 1
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        scale = self._coef if self._clip_pending else None
        order = sorted(range(len(self.arenas)), key=lambda i: self.FORWARD_ORDER.index(self.arenas[i].name)
                       if self.arenas[i].name in self.FORWARD_ORDER else len(self.FORWARD_ORDER))
        if self.overlap:
            self.synchronize()
            self._stream.wait_stream(torch.cuda.current_stream(self._stream.device))
        for i in order:
            a, (m, v), steps = self.arenas[i], self.flat_state[i], self.key_steps[i]
            for lo, hi, st in self._runs(a, steps):
                for clo, chi in (self._chunks(a, lo, hi) if self.overlap else [(lo, hi)]):
                    if self.overlap:
                        with torch.cuda.stream(self._stream):
                            ops.adamw(a.flat[clo:chi], a.grad_flat[clo:chi], m[clo:chi], v[clo:chi], lr=g["lr"],
                                      beta1=b1, beta2=b2, eps=g["eps"], weight_decay=g["weight_decay"], step=st,
                                      grad_scale=scale)
                            ev = torch.cuda.Event()
                            ev.record(self._stream)
                        a.defer(clo, chi, ev)
                    else:
                        ops.adamw(a.flat[clo:chi], a.grad_flat[clo:chi], m[clo:chi], v[clo:chi], lr=g["lr"], beta1=b1,
                                  beta2=b2, eps=g["eps"], weight_decay=g["weight_decay"], step=st, grad_scale=scale)
            a.note_written()
        self._clip_pending = False

    @staticmethod
    def _runs(a, steps):
        """Advance the per-key step counts of the keys with a gradient and return the maximal
        contiguous element ranges (lo, hi, step) sharing one step count: one launch per arena
        when every key has a gradient and the same history (the training step)."""
        runs = []
        for k, (o, n, _) in sorted(a.offsets.items(), key=lambda kv: kv[1][0]):
            if k in a.skipped:
                continue
            steps[k] += 1
            if runs and runs[-1][1] == o and runs[-1][2] == steps[k]:
                runs[-1][1] = o + n
            else:
                runs.append([o, o + n, steps[k]])
        return runs

    def zero_grad(self, set_to_none: bool = False):
        for a in self.arenas:
            a.zero_grad()

    def state_dict(self):
        self.synchronize()
        return {"step": self.step_count, "lr": self.param_groups[0]["lr"], "key_steps": [dict(s) for s in self.key_steps],
                "exp_avg": [m for m, _ in self.flat_state], "exp_avg_sq": [v for _, v in self.flat_state]}

    def load_state_dict(self, sd):
        self.step_count = sd["step"]
        self.param_groups[0]["lr"] = sd["lr"]
        if "key_steps" in sd:
            self.key_steps = [dict(s) for s in sd["key_steps"]]
        else:
            self.key_steps = [{k: self.step_count for k in a.offsets} for a in self.arenas]
        for (m, v), m2, v2 in zip(self.flat_state, sd["exp_avg"], sd["exp_avg_sq"]):
            m.copy_(m2)
            v.copy_(v2)
