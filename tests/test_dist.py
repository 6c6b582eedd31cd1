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
    # buckets are launched during the backward, before all gradients were written
    assert launched and launched[0][1] < len(expect)
    assert sorted(b for b, _ in launched) == list(range(nb))


def _dp_worker(rank, world, port, q):
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

        def model():
            m = CuLLaVOModel(tiny_gpu(), device="cuda", trainable="full", init="none")
            m.load_state_dict(W)
            return m

        def run(m, b):
            ids, mask, pix, labels = (t.cuda() for t in b)
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
                    if a.trainable:
                        acc[a.name] = acc.get(a.name, 0) + a.grad_flat.float().cpu() / world
            ref = {k: v.numpy() for k, v in acc.items()}
        q.put((rank, dp, ref))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc(), None))


@pytest.mark.gpu
def test_dp_step_equals_mean_of_single_gpu_grads():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_dp_worker, args=(r, 2, port, q)) for r in range(2)]
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
