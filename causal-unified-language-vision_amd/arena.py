"""Flat parameter / gradient arenas.

Every parameter group (vision tower, projector, token embedding, decoder layers, lm_head) lives
in ONE contiguous bf16 buffer, with the parameters as views into it, laid out so that
the q|k|v projections of a layer and its gate|up projections are adjacent: the fused
[3d, d] / [2F, d] weight of a single GEMM is then just another view (no copies, no
re-packing). Trainable groups own a matching flat gradient buffer; the backward GEMMs write
dW straight into it (beta = 0 on the first write of an accumulation cycle, 1 after), the DP
all-reduce works on contiguous slices of it, and AdamW runs over the whole buffer in one
kernel. 288 GB of HBM makes this trade (no compaction, everything resident) the right one.
"""
from __future__ import annotations

import math

import torch
from torch import nn


class ParamArena:
    def __init__(self, name: str, specs: list[tuple[str, tuple[int, ...]]], *, device, dtype=torch.bfloat16,
                 trainable: bool = False):
        self.name = name
        self.dtype = dtype
        self.device = torch.device(device)
        self.offsets: dict[str, tuple[int, int, tuple[int, ...]]] = {}
        off = 0
        for key, shape in specs:
            n = int(math.prod(shape))
            self.offsets[key] = (off, n, tuple(shape))
            off += n
        self.numel = off
        self.flat = torch.empty(off, dtype=dtype, device=self.device)
        self.params: dict[str, nn.Parameter] = {}
        for key, (o, n, shape) in self.offsets.items():
            p = nn.Parameter(self.flat[o:o + n].view(shape), requires_grad=trainable)
            p._cv_arena = self
            p._cv_key = key
            self.params[key] = p
        self.trainable = trainable
        self.grad_flat = None
        self._written: set[str] = set()
        # keys with no gradient this cycle (zeroed by finalize_grads): the optimizer skips them
        # like torch.optim.AdamW skips parameters whose .grad is None
        self.skipped: set[str] = set()
        self._write_hooks: list = []  # called with the keys whose gradient write is enqueued
        self._writes = 0  # writes torch's version counter cannot see (kernels on raw pointers)
        self._kmajor: dict[str, list] = {}  # first_key -> [buffer [K, N], state made from, pending event]
        # (lo, hi, event): parameter updates of elements [lo, hi) still running on the
        # optimizer's side stream (FusedAdamW(overlap=True)); consumers call wait_update
        self._pending: list = []
        self._spans: dict[str, tuple[int, int]] = {}
        if trainable:
            self.grad_flat = torch.zeros(off, dtype=dtype, device=self.device)
            self._attach_grads()

    # -- K-major weight copies for the dX GEMMs -------------------------------------------------
    # dx = dy @ W reads W [N, K] along N; from a [K, N] copy both GEMM operands are
    # reduction-contiguous (mode (0,0): +5-18 % on the 7B dX shapes, bitwise-equal results).
    # A copy is re-made when the arena was written since it was made: in-place torch writes
    # through any view bump flat._version, kernel writes (AdamW, RCCL broadcast) call note_written.
    def note_written(self):
        self._writes += 1

    def _state(self):
        return (self.flat._version, self._writes)

    def _kmajor_entry(self, first_key: str, shape: tuple[int, int]):
        ent = self._kmajor.get(first_key)
        if ent is None or ent[0].shape != (shape[1], shape[0]):
            ent = [torch.empty((shape[1], shape[0]), dtype=self.dtype, device=self.device), None, None]
            self._kmajor[first_key] = ent
        return ent

    def prefetch_transposed(self, first_key: str, shape: tuple[int, int], stream=None):
        """Enqueue the refresh of a stale K-major copy on `stream` (after the current stream's
        pending work, e.g. the previous AdamW step), so it overlaps the layer's forward GEMMs;
        transposed() makes the consumer wait on it."""
        from . import ops

        ent = self._kmajor_entry(first_key, shape)
        st = self._state()
        if ent[1] == st:
            return
        cur = torch.cuda.current_stream(self.device)
        if stream is None:
            ops.transpose2d(self.view(first_key, shape), ent[0])
            ent[2] = None
        else:
            stream.wait_stream(cur)
            with torch.cuda.stream(stream):
                ops.transpose2d(self.view(first_key, shape), ent[0])
                ev = torch.cuda.Event()
                ev.record(stream)
            ent[2] = ev
        ent[1] = st

    def transposed(self, first_key: str, shape: tuple[int, int]) -> torch.Tensor:
        """[K, N] copy of the fused weight view [N, K] at first_key, current with the arena."""
        ent = self._kmajor_entry(first_key, shape)
        if ent[1] != self._state():
            self.prefetch_transposed(first_key, shape)
        if ent[2] is not None:
            torch.cuda.current_stream(self.device).wait_event(ent[2])
            ent[2] = None
        return ent[0]

    # -- views -----------------------------------------------------------------------------
    def view(self, first_key: str, n_keys_shape: tuple[int, ...], *, grad: bool = False) -> torch.Tensor:
        """A view starting at first_key spanning prod(shape) elements (fused weights)."""
        o = self.offsets[first_key][0]
        n = int(math.prod(n_keys_shape))
        buf = self.grad_flat if grad else self.flat
        return buf[o:o + n].view(n_keys_shape)

    def check_adjacent(self, keys: list[str]):
        for a, b in zip(keys, keys[1:]):
            oa, na, _ = self.offsets[a]
            if self.offsets[b][0] != oa + na:
                raise RuntimeError(f"arena {self.name}: {a} and {b} are not adjacent")

    def span(self, prefix: str) -> tuple[int, int]:
        """element range [lo, hi) of the keys starting with prefix (one layer's parameters)"""
        sp = self._spans.get(prefix)
        if sp is None:
            sp = self._spans[prefix] = self.slice_of([k for k in self.offsets if k.startswith(prefix)])
        return sp

    # -- deferred optimizer updates ------------------------------------------------------------
    def defer(self, lo: int, hi: int, event):
        self._pending.append((lo, hi, event))

    def wait_update(self, lo: int | None = None, hi: int | None = None):
        """Make the current stream wait for the pending side-stream updates of elements [lo, hi)
        (all of them when lo is None). Forward consumers call it per layer, so the next step's
        forward overlaps the optimizer update of the layers it has not reached yet."""
        if not self._pending:
            return
        cur = torch.cuda.current_stream(self.device)
        keep = []
        for a, b, ev in self._pending:
            if lo is None or (a < hi and lo < b):
                cur.wait_event(ev)
            else:
                keep.append((a, b, ev))
        self._pending = keep

    def slice_of(self, keys: list[str]) -> tuple[int, int]:
        lo = min(self.offsets[k][0] for k in keys)
        hi = max(self.offsets[k][0] + self.offsets[k][1] for k in keys)
        return lo, hi

    # -- gradients ---------------------------------------------------------------------------
    def _attach_grads(self):
        for key, (o, n, shape) in self.offsets.items():
            self.params[key].grad = self.grad_flat[o:o + n].view(shape)

    def grad_slot(self, key: str, span: tuple[int, ...] | None = None) -> tuple[torch.Tensor, float]:
        """(gradient view to write, beta): beta=0 on the first write in this accumulation
        cycle, 1 afterwards. `span` widens the view over adjacent keys (fused weights)."""
        if not self.trainable:
            raise RuntimeError(f"arena {self.name} is frozen")
        self.wait_update()  # the optimizer's side stream may still read last step's gradients
        if self.params[key].grad is None:  # e.g. optimizer.zero_grad(set_to_none=True)
            self._attach_grads()
        beta = 1.0 if key in self._written else 0.0
        self._written.add(key)
        if span is None:
            o, n, shape = self.offsets[key]
            return self.grad_flat[o:o + n].view(shape), beta
        return self.view(key, span, grad=True), beta

    def mark_written(self, keys: list[str]):
        self._written.update(keys)

    def commit(self, keys: list[str]):
        """The kernels writing these keys' gradients are enqueued on the current stream
        (DP bucket hooks may now launch their all-reduce behind them)."""
        for h in self._write_hooks:
            h(keys)

    def zero_grad(self):
        """Start a new accumulation cycle. Buffers are not cleared: the first backward write
        uses beta = 0. Parameters that were never written last cycle are zeroed explicitly."""
        if self.trainable:
            unwritten = [k for k in self.offsets if k not in self._written]
            if unwritten:
                self.wait_update()  # a side-stream optimizer update may still read these gradients
            for k in unwritten:
                o, n, _ = self.offsets[k]
                self.grad_flat[o:o + n].zero_()
            self._attach_grads()
        self._written = set()
        self.skipped = set()

    def finalize_grads(self):
        """Zero the gradient of every parameter that received no write this cycle, record it as
        skipped for this cycle's optimizer step and commit it (so DP buckets holding it can be
        reduced: their all-reduce is issued behind the zeroing)."""
        if self.trainable:
            zeroed = []
            for k, (o, n, _) in self.offsets.items():
                if k not in self._written:
                    self.grad_flat[o:o + n].zero_()
                    self._written.add(k)
                    zeroed.append(k)
            self.skipped.update(zeroed)
            if zeroed:
                self.commit(zeroed)


def grad_slot(p: nn.Parameter, span=None):
    return p._cv_arena.grad_slot(p._cv_key, span)


def commit(*ps):
    for p in ps:
        if p is not None and p.requires_grad:
            p._cv_arena.commit([p._cv_key])


def trainable(p) -> bool:
    return p is not None and p.requires_grad
