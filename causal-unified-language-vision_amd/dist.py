"""Data-parallel gradient exchange: bucketed all-reduce of the flat gradient arenas over RCCL
(torch.distributed backend "nccl" on ROCm), launched on a side HIP stream while the rest of the
backward is still running.

Why not DDP: the reference wraps with DistributedDataParallel through Accelerate and then
unwraps to .module (reference trainer/utils_trainer.py:32-37), which bypasses DDP's reducer.
Here every trainable parameter's gradient already lives in one contiguous arena, written once
per step by the fused backward Functions, so a bucket is just a slice of that buffer:
 * buckets are built in backward-production order (lm_head/final norm, decoder layer L-1 ... 0,
   embeddings, projector) and sized for xGMI (default 256 MiB: large enough that each ring
   step runs at link bandwidth, small enough to start while most of the backward remains);
 * when the last parameter of a bucket has been written (arena write hook, i.e. its dW kernel
   is enqueued), an event is recorded on the compute stream, the comm stream waits on it and
   the all-reduce (average) is issued there; compute continues on the next layer;
 * finish() launches whatever is left and makes the compute stream wait for the comm stream,
   so the optimizer sees reduced gradients. Mean-of-rank-means = DDP semantics.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .arena import ParamArena


class GradReducer:
    def __init__(self, arenas: list[ParamArena], order: list[list[str]] | None = None, *,
                 bucket_bytes: int = 256 << 20, group=None, use_side_stream: bool = True):
        """arenas: trainable arenas; order: parameter keys grouped in the order backward
        produces them (defaults to reverse offset order per arena, arenas as given)."""
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.buckets: list[dict] = []
        self._key_bucket: dict[tuple[int, str], int] = {}
        backend = dist.get_backend(group) if dist.is_initialized() else None
        self.avg_supported = backend == "nccl"
        for ai, ar in enumerate(arenas):
            keys = sorted(ar.offsets, key=lambda k: -ar.offsets[k][0])
            cur: list[str] = []
            cur_bytes = 0
            for k in keys:
                cur.append(k)
                cur_bytes += ar.offsets[k][1] * ar.flat.element_size()
                if cur_bytes >= bucket_bytes:
                    self._add_bucket(ai, ar, cur)
                    cur, cur_bytes = [], 0
            if cur:
                self._add_bucket(ai, ar, cur)
            ar._write_hooks = getattr(ar, "_write_hooks", [])
            ar._write_hooks.append(self._on_write(ai))
        self.arenas = arenas
        dev = arenas[0].flat.device if arenas else torch.device("cpu")
        self.stream = torch.cuda.Stream(device=dev) if (use_side_stream and dev.type == "cuda") else None
        self.enabled = self.world > 1
        self.reset()

    def _add_bucket(self, ai, ar, keys):
        lo, hi = ar.slice_of(keys)
        b = {"arena": ai, "keys": set(keys), "lo": lo, "hi": hi, "pending": set(keys), "work": None,
             "launched": False}
        for k in keys:
            self._key_bucket[(ai, k)] = len(self.buckets)
        self.buckets.append(b)

    def reset(self):
        for b in self.buckets:
            b["pending"] = set(b["keys"])
            b["work"] = None
            b["launched"] = False
        self.launched = []

    def _on_write(self, ai):
        def hook(keys):
            if not self.enabled:
                return
            for k in keys:
                bi = self._key_bucket.get((ai, k))
                if bi is None:
                    continue
                b = self.buckets[bi]
                b["pending"].discard(k)
                if not b["pending"] and not b["launched"]:
                    self._launch(bi)
        return hook

    def _launch(self, bi):
        b = self.buckets[bi]
        b["launched"] = True
        ar = self.arenas[b["arena"]]
        view = ar.grad_flat[b["lo"]:b["hi"]]
        if self.stream is not None:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(view.device))
            with torch.cuda.stream(self.stream):
                self.stream.wait_event(ev)
                b["work"] = self._allreduce(view)
        else:
            b["work"] = self._allreduce(view)
        self.launched.append(bi)

    def _allreduce(self, view):
        if self.avg_supported:
            return dist.all_reduce(view, op=dist.ReduceOp.AVG, group=self.group, async_op=True)
        w = dist.all_reduce(view, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        w.wait()
        view.div_(self.world)
        return None

    def finish(self):
        """Launch every bucket not yet reduced; make the current stream wait for all of them."""
        if not self.enabled:
            return
        for bi, b in enumerate(self.buckets):
            if not b["launched"]:
                self._launch(bi)
        if self.stream is not None:
            with torch.cuda.stream(self.stream):
                for b in self.buckets:
                    if b["work"] is not None:
                        b["work"].wait()
            torch.cuda.current_stream(self.stream.device).wait_stream(self.stream)
        else:
            for b in self.buckets:
                if b["work"] is not None:
                    b["work"].wait()
        self.reset()
