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
   the all-reduce is issued there; compute continues on the next layer;
 * buckets are issued in ONE fixed global order (bucket i only after buckets 0..i-1), so every
   rank pairs the same buffers in the same collective sequence even when their backward
   passes write parameters in different orders (a rank whose batch has no image writes the
   projector only when its unwritten gradients are zeroed at the end of the backward);
 * weight-gradient GEMMs may run on their own side stream (functions.DW_STREAM): the comm
   stream also waits for that stream before each bucket;
 * finish() zero-commits what the backward did not write (arena.finalize_grads), launches
   the remaining buckets and makes the compute stream wait for the comm stream, so the
   optimizer sees reduced gradients. Mean-of-rank-means = DDP semantics;
 * which keys the optimizer skips is agreed across ranks: a per-key "written on this rank"
   mask is MAX-reduced over a host (gloo) group (started asynchronously before the last buckets
   are issued, waited for after; this is a per-step host rendezvous, not a GPU barrier), so a key no rank wrote (e.g. the projector
   when no rank's batch holds an image) stays skipped exactly as on one GPU (DDP leaves such a
   gradient None and torch AdamW skips it); a key written by any rank gets the averaged
   gradient and a step. The mask is host-side control flow, so the exchange never waits on
   the GPU.
The same asynchronous code runs on every backend: RCCL reduces with ReduceOp.AVG; gloo (the
CPU tests) sums and the 1/N scale is applied in finish() after the waits.
"""
from __future__ import annotations

import time

import torch
import torch.distributed as dist

from .arena import ParamArena

_HOST_GROUPS: dict = {}


def host_group(group=None):
    """A gloo group over the ranks of `group` for the written-key mask, created once per process
    group (new_group is collective over the default group: every rank of it reaches the first
    enabled finish() at the same point of the step, so the lazy creation is matched)."""
    if dist.get_backend(group) == "gloo":
        return group
    key = id(group)
    if key not in _HOST_GROUPS:
        ranks = dist.get_process_group_ranks(group) if group is not None else None
        _HOST_GROUPS[key] = dist.new_group(ranks=ranks, backend="gloo")
    return _HOST_GROUPS[key]


class GradReducer:
    def __init__(self, arenas: list[ParamArena], order: list[list[str]] | None = None, *,
                 bucket_bytes: int = 256 << 20, group=None, use_side_stream: bool = True,
                 enabled: bool | None = None):
        """arenas: trainable arenas, in the order backward produces them; each arena's keys in
        reverse offset order (decoder layer L-1 first). enabled: None = only when the group has
        more than one rank; True runs the exchange at world size 1 too (tests of the RCCL path)."""
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self._elem = [ar.flat.element_size() for ar in arenas]
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
        self.enabled = self.world > 1 if enabled is None else (bool(enabled) and dist.is_initialized())
        self.timing = None  # a list: record when each bucket becomes ready (overlap analysis)
        # per finish(): (backward-end event, exchange-done event, host ms in the mask agreement)
        # on the compute stream when `measure` is set (bench.py's exposed-exchange figure)
        self.measure = False
        self.exposure: list[tuple] = []
        self.bytes_per_step = sum((b["hi"] - b["lo"]) * self._elem[b["arena"]] for b in self.buckets)
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
        self._next = 0  # the next bucket in the global issue order

    def _on_write(self, ai):
        def hook(keys):
            if not self.enabled:
                return
            for k in keys:
                bi = self._key_bucket.get((ai, k))
                if bi is not None:
                    self.buckets[bi]["pending"].discard(k)
            self._issue_ready()
        return hook

    def _issue_ready(self):
        """Issue the longest ready prefix of the global bucket order."""
        while self._next < len(self.buckets) and not self.buckets[self._next]["pending"]:
            self._launch(self._next)
            self._next += 1

    def _launch(self, bi):
        b = self.buckets[bi]
        b["launched"] = True
        ar = self.arenas[b["arena"]]
        view = ar.grad_flat[b["lo"]:b["hi"]]
        from .functions import dw_join, dw_wait
        if self.stream is not None:
            ev = torch.cuda.Event(enable_timing=self.timing is not None)
            ev.record(torch.cuda.current_stream(view.device))
            if self.timing is not None:  # (bucket, bytes, ready event) for tools/dp_overlap.py
                self.timing.append((bi, view.numel() * view.element_size(), ev))
            with torch.cuda.stream(self.stream):
                self.stream.wait_event(ev)
                dw_wait(self.stream)  # weight gradients of the bucket may be on the dW side stream
                b["work"] = self._allreduce(view)
        else:
            if view.is_cuda:
                dw_join(view.device)
            b["work"] = self._allreduce(view)
        self.launched.append(bi)

    def _allreduce(self, view):
        op = dist.ReduceOp.AVG if self.avg_supported else dist.ReduceOp.SUM
        return dist.all_reduce(view, op=op, group=self.group, async_op=True)

    def _start_agree_skipped(self):
        """Start the MAX of the per-rank written masks on the host group (asynchronous: the
        buckets are issued while gloo exchanges the mask). This is the exchange's one host
        rendezvous per step; the GPU never waits on it unless the host falls behind the GPU."""
        keys = [(ar, k) for ar in self.arenas for k in ar.offsets]
        written = torch.tensor([0 if k in ar.skipped else 1 for ar, k in keys], dtype=torch.uint8)
        work = dist.all_reduce(written, op=dist.ReduceOp.MAX, group=host_group(self.group), async_op=True)
        return keys, written, work

    def _finish_agree_skipped(self, pending):
        """ar.skipped := the keys no rank wrote this cycle."""
        keys, written, work = pending
        work.wait()
        for ar in self.arenas:
            ar.skipped = set()
        for (ar, k), w in zip(keys, written.tolist()):
            if not w:
                ar.skipped.add(k)

    def finish(self):
        """Zero-commit unwritten gradients, issue every bucket not yet reduced (in order) and
        make the current stream wait for all of them (sum backends: scale by 1/N after)."""
        if not self.enabled:
            return
        cur = torch.cuda.current_stream(self.stream.device) if self.stream is not None else None
        ev_bwd = None
        if self.measure and cur is not None:
            ev_bwd = torch.cuda.Event(enable_timing=True)
            ev_bwd.record(cur)
        for ar in self.arenas:
            ar.finalize_grads()  # commits the keys it zeroes -> hooks issue their buckets
        pending = self._start_agree_skipped()
        for b in self.buckets:
            b["pending"].clear()
        self._issue_ready()
        assert self._next == len(self.buckets)
        scale = 1.0 / self.world

        def _complete():
            for b in self.buckets:
                b["work"].wait()
                if not self.avg_supported:
                    self.arenas[b["arena"]].grad_flat[b["lo"]:b["hi"]].mul_(scale)

        # every bucket's completion is queued on the GPU before the host waits for the written-key
        # agreement (needed only by the optimizer step that follows: which keys move)
        ev_done = None
        if self.stream is not None:
            with torch.cuda.stream(self.stream):
                _complete()
            cur.wait_stream(self.stream)
            if ev_bwd is not None:
                ev_done = torch.cuda.Event(enable_timing=True)
                ev_done.record(cur)
        else:
            _complete()
        t0 = time.perf_counter()
        self._finish_agree_skipped(pending)
        host_ms = (time.perf_counter() - t0) * 1e3
        if ev_done is not None:
            self.exposure.append((ev_bwd, ev_done, host_ms))
        self.reset()

    def exposure_stats(self) -> dict | None:
        """Mean over the measured steps: exposed exchange = backward end (the compute stream's
        last gradient write) -> the compute stream may start clip + AdamW (all buckets reduced);
        host_ms = the host time spent waiting for the written-key agreement."""
        if not self.exposure:
            return None
        torch.cuda.synchronize()
        exp = [a.elapsed_time(b) for a, b, _ in self.exposure]
        host = [h for _, _, h in self.exposure]
        return {"exposed_ms": sum(exp) / len(exp), "host_rendezvous_ms": sum(host) / len(host),
                "steps": len(exp)}
