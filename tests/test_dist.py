"""Data-parallel gradient exchange.

CPU (gloo, world_size 2): GradReducer buckets the flat gradient arena in backward order,
launches each bucket's all-reduce as soon as its last gradient is committed, and finish()
leaves every rank with the mean of the per-rank gradients (DDP mean-of-rank-means).

GPU (gloo over 2 processes sharing the one MI355X): a full CuLLaVOModel DP step on per-rank
batches yields the same reduced gradients as the average of single-process gradients on the
same two batches.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _reducer_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, REPO)
    try:
        _init(rank, world, port)
        from cullavo_amd.arena import ParamArena
        from cullavo_amd.dist import GradReducer
        specs = [(f"layers.{i}.w", (16, 8)) for i in range(6)] + [("norm.w", (8,))]
        ar = ParamArena("layers", specs, device="cpu", dtype=torch.float32, trainable=True)
        red = GradReducer([ar], bucket_bytes=2 * 16 * 8 * 4)  # 2 layers per bucket
        launched_at = []
        orig = red._launch

        def spy(bi):
            launched_at.append((bi, len(written)))
            orig(bi)
        red._launch = spy
        written = []
        g = torch.Generator().manual_seed(100 + rank)
        expect = {}
        # backward order: norm, layer 5 ... layer 0
        for key in ["norm.w"] + [f"layers.{i}.w" for i in reversed(range(6))]:
            slot, beta = ar.grad_slot(key)
            val = torch.randn(slot.shape, generator=g)
            slot.copy_(val)
            expect[key] = val
            written.append(key)
            ar.commit([key])
        red.finish()
        res = {k: ar.params[k].grad.clone().numpy() for k in expect}  # by value through the queue
        expect = {k: v.numpy() for k, v in expect.items()}
        q.put((rank, res, expect, launched_at, len(red.buckets)))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - surfaced by the parent
        q.put((rank, repr(e), None, None, None))


def test_grad_reducer_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_reducer_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = {}
    for _ in ps:
        rank, res, expect, launched, nb = q.get(timeout=120)
        assert expect is not None, res
        out[rank] = (res, expect, launched, nb)
    for p in ps:
        p.join(timeout=60)
    for k in out[0][0]:
        mean = torch.from_numpy((out[0][1][k] + out[1][1][k]) / 2)
        torch.testing.assert_close(torch.from_numpy(out[0][0][k]), mean)
        torch.testing.assert_close(torch.from_numpy(out[1][0][k]), mean)
    res, expect, launched, nb = out[0]
    assert nb >= 3
    # buckets are launched during the backward, before all gradients were written, in the
    # fixed global order
    assert launched and launched[0][1] < len(expect)
    assert [b for b, _ in launched] == list(range(nb))


def _ragged_worker(rank, world, port, q):
    """Rank 0 writes every key in backward order; rank 1 writes them in another order and never
    writes 'proj.w' (a rank whose batch has no image: the projector gets no gradient)."""
    import sys
    sys.path.insert(0, REPO)
    try:
        _init(rank, world, port)
        from cullavo_amd.arena import ParamArena
        from cullavo_amd.dist import GradReducer
        specs = [(f"layers.{i}.w", (16, 8)) for i in range(4)] + [("proj.w", (8, 8))]
        ar = ParamArena("layers", specs, device="cpu", dtype=torch.float32, trainable=True)
        red = GradReducer([ar], bucket_bytes=16 * 8 * 4)  # one key per bucket
        issued = []
        orig = red._launch

        def spy(bi):
            issued.append(bi)
            orig(bi)
        red._launch = spy
        g = torch.Generator().manual_seed(7 + rank)
        order = ["proj.w"] + [f"layers.{i}.w" for i in reversed(range(4))]
        if rank == 1:
            order = ["layers.0.w", "layers.2.w", "layers.3.w", "layers.1.w"]
        vals = {}
        for key in order:
            slot, _ = ar.grad_slot(key)
            vals[key] = torch.randn(slot.shape, generator=g)
            slot.copy_(vals[key])
            ar.commit([key])
        red.finish()
        res = {k: ar.params[k].grad.clone().numpy() for k in ar.offsets}
        q.put((rank, res, {k: v.numpy() for k, v in vals.items()}, issued, sorted(ar.skipped)))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc(), None, None, None))


def test_grad_reducer_ragged_ranks_gloo_world2():
    """Ranks that write their gradients in different orders, one of them missing a parameter:
    the same buckets are reduced in the same global order (no mismatched collectives), the
    missing gradient contributes zeros, and every rank ends with the mean."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_ragged_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = {}
    for _ in ps:
        rank, res, vals, issued, skipped = q.get(timeout=120)
        assert vals is not None, res
        out[rank] = (res, vals, issued, skipped)
    for p in ps:
        p.join(timeout=60)
    import numpy as np
    for k in out[0][0]:
        mean = (out[0][1].get(k, 0) + out[1][1].get(k, np.zeros_like(out[0][1][k]))) / 2
        for r in range(2):
            np.testing.assert_allclose(out[r][0][k], mean, rtol=1e-6, atol=1e-7)
    assert out[0][2] == out[1][2] == list(range(len(out[0][2]))) and len(out[0][2]) >= 4
    assert out[0][3] == out[1][3] == []  # DP: every key steps on the averaged gradient


def _world_worker(rank, world, port, q):
    """N ranks, each writing its gradients in its own (seeded) order. 'proj.w' is written only by
    even ranks (odd ranks: a batch with no image), 'unused.w' by no rank, and 'layers.1.w' only by
    the last rank (a ragged batch that alone reaches a parameter)."""
    import sys
    sys.path.insert(0, REPO)
    try:
        _init(rank, world, port)
        from cullavo_amd.arena import ParamArena
        from cullavo_amd.dist import GradReducer
        from cullavo_amd.optim import FusedAdamW
        specs = [(f"layers.{i}.w", (16, 8)) for i in range(6)] + [("proj.w", (8, 8)), ("unused.w", (4, 8))]
        ar = ParamArena("layers", specs, device="cpu", dtype=torch.float32, trainable=True)
        red = GradReducer([ar], bucket_bytes=2 * 16 * 8 * 4)
        issued = []
        orig = red._launch

        def spy(bi):
            issued.append(bi)
            orig(bi)
        red._launch = spy
        keys = [f"layers.{i}.w" for i in range(6) if i != 1]
        if rank % 2 == 0:
            keys.append("proj.w")
        if rank == world - 1:
            keys.append("layers.1.w")
        g = torch.Generator().manual_seed(1000 + rank)
        order = [keys[i] for i in torch.randperm(len(keys), generator=g).tolist()]
        vals = {}
        for key in order:
            slot, _ = ar.grad_slot(key)
            vals[key] = torch.randn(slot.shape, generator=g)
            slot.copy_(vals[key])
            ar.commit([key])
        red.finish()
        res = {k: ar.params[k].grad.clone().numpy() for k in ar.offsets}
        steps = {k: 0 for k in ar.offsets}
        runs = FusedAdamW._runs(ar, steps)  # the element ranges the optimizer would update
        q.put((rank, res, {k: v.numpy() for k, v in vals.items()}, issued, sorted(ar.skipped), runs))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc(), None, None, None, None))


@pytest.mark.parametrize("world", [2, 4, 8])
def test_grad_reducer_worlds_ragged_and_unused(world):
    """DP protocol at the world sizes the scaling run uses: every rank issues the same bucket
    sequence in the fixed global order whatever order its backward wrote in; the result is the
    mean over ranks with zeros from ranks that did not reach a parameter; a parameter that no
    rank wrote stays skipped on every rank (no AdamW step, like torch AdamW on a None grad under
    DDP), while one written by a single rank is stepped everywhere."""
    import numpy as np
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_world_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = {}
    for _ in ps:
        rank, res, vals, issued, skipped, runs = q.get(timeout=240)
        assert vals is not None, res
        out[rank] = (res, vals, issued, skipped, runs)
    for p in ps:
        p.join(timeout=60)
    for k in out[0][0]:
        tot = sum(out[r][1].get(k, np.zeros_like(out[0][0][k])) for r in range(world))
        for r in range(world):
            np.testing.assert_allclose(out[r][0][k], tot / world, rtol=1e-5, atol=1e-6)
    nb = len(out[0][2])
    assert nb >= 3
    for r in range(world):
        assert out[r][2] == list(range(nb)), (r, out[r][2])
        assert out[r][3] == ["unused.w"], (r, out[r][3])
        assert out[r][4] == out[0][4]
    # the optimizer's ranges stop before 'unused.w' (the last key) and cover everything else
    lo, hi = out[0][4][0][0], out[0][4][-1][1]
    assert lo == 0 and hi == 6 * 16 * 8 + 8 * 8


def _dp_worker(rank, world, port, q, text_only_rank=-1):
    import sys
    sys.path.insert(0, REPO)
    try:
        torch.cuda.set_device(0)
        _init(rank, world, port)
        from oracle import cullavo_oracle as O
        from cullavo_amd.arch_cullavo import CuLLaVOModel
        from cullavo_amd.config import tiny_gpu
        from cullavo_amd.dist import GradReducer
        cfg_o = O.config_small_gpu()
        W = O.make_weights(cfg_o, 5)
        batches = [O.make_inputs(cfg_o, 2, 40, 4, 50 + r) for r in range(world)]
        if text_only_rank >= 0:  # that rank's batch has no image: no pixel_values, no <image> id
            ids, mask, _, labels = batches[text_only_rank]
            ids = ids.clone()
            ids[ids == cfg_o.image_token_index] = 7
            batches[text_only_rank] = (ids, mask, None, labels[:, -ids.shape[1]:].clone())

        def model():
            m = CuLLaVOModel(tiny_gpu(), device="cuda", trainable="full", init="none")
            m.load_state_dict(W)
            return m

        def run(m, b):
            ids, mask, pix, labels = (t.cuda() if t is not None else None for t in b)
            m(input_ids=ids, pixel_values=pix, attention_mask=mask, labels=labels).loss.backward()

        m = model()
        arenas = [a for a in m.arenas.values() if a.trainable]
        red = GradReducer(arenas, bucket_bytes=64 << 10)
        run(m, batches[rank])
        red.finish()
        torch.cuda.synchronize()
        dp = {a.name: a.grad_flat.float().cpu().numpy() for a in arenas}
        ref = None
        if rank == 0:
            acc = {}
            for b in batches:
                m2 = model()
                run(m2, b)
                for a in m2.arenas.values():
                    a.finalize_grads()  # a parameter the batch did not reach has a zero gradient
                    if a.trainable:
                        acc[a.name] = acc.get(a.name, 0) + a.grad_flat.float().cpu() / world
            ref = {k: v.numpy() for k, v in acc.items()}
        q.put((rank, dp, ref))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc(), None))


@pytest.mark.gpu
@pytest.mark.parametrize("text_only_rank", [-1, 1], ids=["both_images", "rank1_text_only"])
def test_dp_step_equals_mean_of_single_gpu_grads(text_only_rank):
    """Both ranks run the production reducer code (async all-reduce on the side stream, fixed
    bucket order); with rank 1 holding a text-only batch its projector buckets are issued from
    finish() while rank 0 issues them from the backward hooks, and the result is still the mean."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_dp_worker, args=(r, 2, port, q, text_only_rank)) for r in range(2)]
    for p in ps:
        p.start()
    out = {}
    for _ in ps:
        rank, dp, ref = q.get(timeout=600)
        assert isinstance(dp, dict), dp
        out[rank] = (dp, ref)
    for p in ps:
        p.join(timeout=60)
    ref = {k: torch.from_numpy(v) for k, v in out[0][1].items()}
    for name in ref:
        for r in range(2):
            got = torch.from_numpy(out[r][0][name])
            # bf16 gradients: the all-reduce sums bf16 values (one rounding) vs an f32 mean
            err = (got - ref[name]).norm() / (ref[name].norm() + 1e-12)
            assert err < 1e-2, (name, r, err.item())
    torch.testing.assert_close(torch.from_numpy(out[0][0]["layers"]), torch.from_numpy(out[1][0]["layers"]))


def _rccl_worker(port, q):
    import sys
    sys.path.insert(0, REPO)
    try:
        torch.cuda.set_device(0)
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        from oracle import cullavo_oracle as O
        from cullavo_amd.arch_cullavo import CuLLaVOModel
        from cullavo_amd.config import tiny_gpu
        from cullavo_amd.dist import GradReducer
        cfg_o = O.config_small_gpu()
        W = O.make_weights(cfg_o, 5)
        ids, mask, pix, labels = (t.cuda() for t in O.make_inputs(cfg_o, 2, 40, 4, 50))
        grads = []
        for use_reducer in (False, True):
            m = CuLLaVOModel(tiny_gpu(), device="cuda", trainable="full", init="none")
            m.load_state_dict(W)
            arenas = [a for a in m.arenas.values() if a.trainable]
            red = GradReducer(arenas, bucket_bytes=64 << 10, enabled=True) if use_reducer else None
            m(input_ids=ids, pixel_values=pix, attention_mask=mask, labels=labels).loss.backward()
            if red is not None:
                assert red.avg_supported and red.stream is not None
                red.finish()
            else:
                for a in arenas:
                    a.finalize_grads()
            torch.cuda.synchronize()
            grads.append({a.name: a.grad_flat.float().cpu() for a in arenas})
        q.put(("ok", grads))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback
        q.put((traceback.format_exc(), None))


@pytest.mark.gpu
def test_rccl_reducer_path_world1_is_identity():
    """The reducer's RCCL branch (ReduceOp.AVG, async all-reduce on the side stream, fixed bucket
    order, stream join) on a real RCCL communicator: at world size 1 the averaged gradients must be
    bitwise the local ones (the multi-rank arithmetic is covered by the gloo tests above)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), q))
    p.start()
    status, grads = q.get(timeout=600)
    p.join(timeout=60)
    assert status == "ok", status
    plain, reduced = grads
    for name in plain:
        assert torch.equal(plain[name], reduced[name]), name
