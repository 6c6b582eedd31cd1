"""KV-cache decode / generate (reference cullavo/arch_cullavo.py:341-395,
605-636 and HF generate()).

Kernel level: kv_append is a copy (bit-exact); attn_decode against an fp32 softmax over the
visible key range (max|err| <= 1e-2 * scale, bf16 output). Model level: prefill logits equal
the training-path forward, and each cached decode step's logits match the CPU oracle's full
recompute of the whole sequence (relative-L2 <= 3e-2, the bf16 model-parity bar of
tests/test_model_gpu.py); greedy tokens are the oracle's argmax up to bf16 near-ties.
"""
import pytest
import torch

from oracle import cullavo_oracle as O

BF = torch.bfloat16


def rel_l2(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


# ---------------------------------------------------------------------------------------------
# CPU: sampling warpers (torch glue, no kernels)
# ---------------------------------------------------------------------------------------------
def test_sample_next_warpers():
    from cullavo_amd.generation import sample_next
    logits = torch.tensor([[0.0, 1.0, 2.0, 3.0, 4.0]])
    assert sample_next(logits, do_sample=False).item() == 4
    g = torch.Generator().manual_seed(0)
    assert sample_next(logits, do_sample=True, top_k=1, generator=g).item() == 4
    # top-p 0.5 keeps only the most likely token here (p(4) = 0.64)
    assert sample_next(logits, do_sample=True, top_p=0.5, generator=g).item() == 4
    draws = {sample_next(logits, do_sample=True, top_k=2, generator=g).item() for _ in range(200)}
    assert draws == {3, 4}


# ---------------------------------------------------------------------------------------------
# GPU kernels
# ---------------------------------------------------------------------------------------------
@pytest.mark.gpu
def test_kv_append_exact():
    from cullavo_amd import ops
    B, Lnew, hd, Lmax = 3, 5, 256, 16
    src = torch.randn(B * Lnew, 3 * hd).to(BF).cuda()
    k, v = src[:, hd:2 * hd], src[:, 2 * hd:]
    kc = torch.zeros(B, Lmax, hd, dtype=BF, device="cuda")
    vc = torch.zeros_like(kc)
    start = torch.tensor([0, 4, 11], dtype=torch.int32, device="cuda")
    ops.kv_append(k, v, kc, vc, start, B=B, Lnew=Lnew)
    for b in range(B):
        s = int(start[b])
        assert torch.equal(kc[b, s:s + Lnew], k[b * Lnew:(b + 1) * Lnew])
        assert torch.equal(vc[b, s:s + Lnew], v[b * Lnew:(b + 1) * Lnew])
        assert int((kc[b, :s] != 0).sum()) == 0


@pytest.mark.gpu
def test_attn_decode_matches_softmax():
    from cullavo_amd import ops
    B, H, D, Lmax = 3, 4, 128, 700
    g = torch.Generator().manual_seed(5)
    q = torch.randn(B, H * D, generator=g).to(BF)
    kc = torch.randn(B, Lmax, H * D, generator=g).to(BF)
    vc = torch.randn(B, Lmax, H * D, generator=g).to(BF)
    kv_len = torch.tensor([700, 513, 3], dtype=torch.int32)
    kv_start = torch.tensor([0, 17, 1], dtype=torch.int32)
    o = ops.attn_decode(q.cuda(), kc.cuda(), vc.cuda(), kv_len.cuda(), B=B, H=H, D=D, max_len=700,
                        scale=D ** -0.5, kv_start=kv_start.cuda())
    for b in range(B):
        lo, hi = int(kv_start[b]), int(kv_len[b])
        qh = q[b].float().view(H, D)
        kh = kc[b, lo:hi].float().view(-1, H, D).transpose(0, 1)
        vh = vc[b, lo:hi].float().view(-1, H, D).transpose(0, 1)
        p = torch.softmax((kh @ qh[:, :, None]).squeeze(-1) * D ** -0.5, -1)
        ref = (p[:, None, :] @ vh).squeeze(1).reshape(-1)
        err = (o[b].float().cpu() - ref).abs().max().item()
        assert err <= 1e-2 * ref.abs().max().item(), (b, err)


# ---------------------------------------------------------------------------------------------
# model: prefill + cached decode vs the oracle's full recompute
# ---------------------------------------------------------------------------------------------
def _model(seed=6):
    from cullavo_amd.arch_cullavo import CuLLaVOModel
    from cullavo_amd.config import tiny_gpu
    m = CuLLaVOModel(tiny_gpu(), device="cuda", trainable="none", init="none")
    m.load_state_dict(O.make_weights(O.config_small_gpu(), seed))
    m.eval()
    return m


@pytest.mark.gpu
def test_prefill_and_cached_decode_match_oracle():
    cfg = O.config_small_gpu()
    W = O.make_weights(cfg, 6)
    m = _model(6)
    ids, mask, pix, _ = O.make_inputs(cfg, 2, 24, 4, 11)
    out = m(input_ids=ids.cuda(), pixel_values=pix.cuda(), attention_mask=mask.cuda(), use_cache=True)
    cache = out.past_key_values
    ref_train = m(input_ids=ids.cuda(), pixel_values=pix.cuda(), attention_mask=mask.cuda())
    assert rel_l2(out.logits, ref_train.logits) <= 1e-2  # same kernels, no cache
    g = torch.Generator().manual_seed(1)
    seq = ids.clone()
    for step in range(3):
        tok = torch.randint(2, cfg.image_token_index, (2, 1), generator=g)
        out = m(input_ids=tok.cuda(), past_key_values=cache, use_cache=True)
        seq = torch.cat([seq, tok], 1)
        _, logits_ref, _ = O.forward(W, cfg, seq, pix, torch.ones_like(seq), None)
        err = rel_l2(out.logits[:, -1], logits_ref[:, -1])
        assert err <= 3e-2, (step, err)
    assert cache.get_seq_length() == 24 + cfg.vision.num_patches - 1 + 3
    k0, v0 = cache[0]
    assert k0.shape == (2, cfg.text.num_attention_heads, cache.get_seq_length(), cfg.text.head_dim)


@pytest.mark.gpu
def test_generate_greedy_and_sampling():
    cfg = O.config_small_gpu()
    W = O.make_weights(cfg, 6)
    m = _model(6)
    ids, mask, pix, _ = O.make_inputs(cfg, 1, 20, 3, 12)
    out = m.generate(input_ids=ids.cuda(), pixel_values=pix.cuda(), attention_mask=mask.cuda(), max_new_tokens=5)
    assert out.shape == (1, 25) and torch.equal(out[:, :20].cpu(), ids)
    # each greedy token is the oracle's argmax of the full recompute (up to bf16 near-ties)
    for i in range(5):
        prefix = out[:, :20 + i].cpu()
        _, lg, _ = O.forward(W, cfg, prefix, pix, torch.ones_like(prefix), None)
        last = lg[0, -1]
        tok = int(out[0, 20 + i])
        top = torch.topk(last, 2).values
        assert tok == int(last.argmax()) or (last.max() - last[tok]).item() <= 2e-2 * (top[0] - last.min()).item(), i
    # decoding is deterministic (greedy twice), sampling reproducible with a seeded generator
    again = m.generate(input_ids=ids.cuda(), pixel_values=pix.cuda(), attention_mask=mask.cuda(), max_new_tokens=5)
    assert torch.equal(again, out)
    kw = dict(input_ids=ids.cuda(), pixel_values=pix.cuda(), attention_mask=mask.cuda(), max_new_tokens=6,
              do_sample=True, temperature=0.9, top_k=50, top_p=0.95)  # the reference's step-2 settings
    a = m.generate(**kw, generator=torch.Generator(device="cuda").manual_seed(3))
    b = m.generate(**kw, generator=torch.Generator(device="cuda").manual_seed(3))
    assert torch.equal(a, b) and a.shape == (1, 26)


@pytest.mark.gpu
def test_left_padded_batch_matches_single():
    cfg = O.config_small_gpu()
    m = _model(6)
    ids, mask, pix, _ = O.make_inputs(cfg, 1, 20, 3, 13)
    pad = cfg.pad_token_id
    ids2 = torch.cat([torch.full((1, 5), pad), ids], 1)
    mask2 = torch.cat([torch.zeros(1, 5, dtype=mask.dtype), mask], 1)
    extra = torch.randint(2, cfg.image_token_index, (1, 5), generator=torch.Generator().manual_seed(2))
    batch_ids = torch.cat([ids2, torch.cat([extra, ids], 1)], 0)  # row 1: unpadded, longer prompt
    batch_mask = torch.cat([mask2, torch.ones_like(mask2)], 0)
    batch_pix = torch.cat([pix, pix], 0)
    one = m.generate(input_ids=ids.cuda(), pixel_values=pix.cuda(), attention_mask=mask.cuda(), max_new_tokens=4)
    two = m.generate(input_ids=batch_ids.cuda(), pixel_values=batch_pix.cuda(), attention_mask=batch_mask.cuda(),
                     max_new_tokens=4)
    assert torch.equal(two[0, 25:].cpu(), one[0, 20:].cpu())


@pytest.mark.gpu
def test_transformers_layout_cache_decode_matches_kvcache():
    """A decode step fed a transformers-layout cache (the legacy tuple of per-layer (key, value)
    [B, H, L, D] that the reference's decode branch indexes, arch_cullavo.py:605-636) with the
    caller's text-level attention_mask (left padding in row 0) gives bitwise the logits of the
    same step on the native KVCache, and the returned cache indexes like the legacy tuple."""
    from cullavo_amd.generation import KVCache
    cfg = O.config_small_gpu()
    m = _model(6)
    ids, mask, pix, _ = O.make_inputs(cfg, 2, 20, 3, 17)
    pad = cfg.pad_token_id
    ids = torch.cat([torch.full((2, 4), pad), ids], 1)
    ids[1, :4] = torch.randint(2, cfg.image_token_index, (4,), generator=torch.Generator().manual_seed(3))
    mask = torch.cat([torch.ones(2, 4, dtype=mask.dtype), mask], 1)
    mask[0, :4] = 0
    ids, mask, pix = ids.cuda(), mask.cuda(), pix.cuda()
    out = m(input_ids=ids, pixel_values=pix, attention_mask=mask, use_cache=True)
    native = out.past_key_values
    legacy = tuple((k.clone(), v.clone()) for k, v in native.to_legacy_cache())
    tok = torch.randint(2, cfg.image_token_index, (2, 1), generator=torch.Generator().manual_seed(4)).cuda()
    step_mask = torch.cat([mask, torch.ones(2, 1, dtype=mask.dtype, device=mask.device)], 1)
    a = m(input_ids=tok, past_key_values=legacy, attention_mask=step_mask, use_cache=True)
    b = m(input_ids=tok, past_key_values=native, attention_mask=step_mask, use_cache=True)
    assert torch.equal(a.logits, b.logits)
    assert isinstance(a.past_key_values, KVCache)
    first = a.past_key_values[0][0][:, :, :, 0]  # the reference's indexing (:611)
    assert first.shape == (2, cfg.text.num_attention_heads, native.get_seq_length())
    with pytest.raises(TypeError, match="legacy cache"):
        m(input_ids=tok, past_key_values=torch.zeros(3), attention_mask=step_mask, use_cache=True)


# ---------------------------------------------------------------------------------------------
# decode-step GEMV (gemv.hip) and the captured decode graph (generation.DecodeGraph)
# ---------------------------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(1, 4096, 4096), (8, 12288, 4096), (3, 776, 1000), (16, 4096, 11008),
                                   (8, 32064, 4096), (5, 264, 64)])
@pytest.mark.parametrize("epi", ["none", "residual", "addend_bias"])
def test_gemv_decode_rows_match_fp32(M, N, K, epi):
    """Y = X W^T for M = batch <= 16 rows goes through the weight-streaming kernel (plan tile 14)
    with the full GEMM epilogue; checked against fp32 on the same bf16 inputs (max|err| <= 8e-3 x
    scale, the GEMM tests' bar) and against the tiled kernel (forced tile 2: same products, other
    f32 summation order)."""
    from cullavo_amd import _lib, ops
    L = _lib.lib()
    assert L.cullavo_gemm_plan(M, N, K, 0, 0, None) == 14
    g = torch.Generator().manual_seed(M * 7 + N + K)
    X = torch.randn(M, K, generator=g).to(BF)
    W = (torch.randn(N, K, generator=g) * K ** -0.5).to(BF)
    bias = torch.randn(N, generator=g).to(BF) if epi == "addend_bias" else None
    add = torch.randn(M, N, generator=g).to(BF) if epi == "addend_bias" else None
    res = torch.randn(M, N, generator=g).to(BF) if epi == "residual" else None
    z = X.float() @ W.float().T
    if bias is not None:
        z = (z + bias.float()).to(BF).float() + add.float()
    if res is not None:
        z = z.to(BF).float() + res.float()
    dev = lambda t: t.cuda() if t is not None else None
    outs = []
    for tile in (-1, 2):
        prev = L.cullavo_gemm_set_tile(tile)
        try:
            C = torch.empty(M, N, dtype=BF, device="cuda")
            ops.gemm_ex(0, 0, M, N, K, dev(X), K, dev(W), K, C, N, bias=dev(bias), addend=dev(add),
                        ld_addend=N if add is not None else 0, residual=dev(res), ldr=N if res is not None else 0)
            torch.cuda.synchronize()
        finally:
            L.cullavo_gemm_set_tile(prev)
        outs.append(C.float().cpu())
    for o in outs:
        assert (o - z).abs().max().item() <= 8e-3 * z.abs().max().item()
    assert rel_l2(outs[0], outs[1]) <= 4e-3


@pytest.mark.gpu
def test_decode_graph_matches_eager_steps():
    """The captured decode step (HIP graph replay, attention sized for the cache capacity) gives
    bitwise the logits of the eager cached forward, step after step, and advances the cache the
    same way; generate() with and without the graph returns the same tokens."""
    from cullavo_amd.generation import DecodeGraph, KVCache
    cfg = O.config_small_gpu()
    m = _model(6)
    ids, mask, pix, _ = O.make_inputs(cfg, 2, 20, 3, 21)
    ids, mask, pix = ids.cuda(), mask.cuda(), pix.cuda()
    L0 = 20 + cfg.vision.num_patches - 1
    runs = []
    for use_graph in (False, True):
        out = m._forward_cached(ids, pix, mask, None, None, None, -2, "default", None, True, max_len=L0 + 8)
        cache = out.past_key_values
        graph = DecodeGraph(m, cache) if use_graph else None
        toks = torch.randint(2, cfg.image_token_index, (6, 2), generator=torch.Generator().manual_seed(9)).cuda()
        steps = []
        for i in range(6):
            if graph is not None:
                lg = graph.step(toks[i]).clone()
            else:
                lg = m(input_ids=toks[i][:, None], past_key_values=cache, use_cache=True).logits.clone()
            steps.append(lg)
        runs.append((steps, cache))
    for i, (a, b) in enumerate(zip(runs[0][0], runs[1][0])):
        assert torch.equal(a, b), i
    ca, cb = runs[0][1], runs[1][1]
    assert ca.length == cb.length == L0 + 6
    assert torch.equal(ca.k[:, :, :ca.length], cb.k[:, :, :cb.length])
    assert torch.equal(ca.next_pos, cb.next_pos)
    kw = dict(input_ids=ids, pixel_values=pix, attention_mask=mask, max_new_tokens=7)
    assert torch.equal(m.generate(**kw), m.generate(**kw, decode_graph=False))


@pytest.mark.gpu
@pytest.mark.parametrize("swiglu", [False, True])
def test_decode_fusions_bitwise(monkeypatch, swiglu):
    """The decode layer with its RMSNorms (and SwiGLU) folded into the weight-streaming products
    (CULLAVO_DECODE_FUSE) gives bitwise the logits of the separate kernels, step after step."""
    from cullavo_amd import generation
    cfg = O.config_small_gpu()
    m = _model(6)
    ids, mask, pix, _ = O.make_inputs(cfg, 2, 20, 3, 31)
    ids, mask, pix = ids.cuda(), mask.cuda(), pix.cuda()
    toks = torch.randint(2, cfg.image_token_index, (4, 2), generator=torch.Generator().manual_seed(5)).cuda()
    runs = []
    for fuse in (False, True):
        monkeypatch.setattr(generation, "FUSE_DECODE_NORMS", fuse)
        monkeypatch.setattr(generation, "FUSE_DECODE_SWIGLU", fuse and swiglu)
        cache = m(input_ids=ids, pixel_values=pix, attention_mask=mask, use_cache=True).past_key_values
        runs.append([m(input_ids=t[:, None], past_key_values=cache, use_cache=True).logits.clone() for t in toks])
    for i, (a, b) in enumerate(zip(*runs)):
        assert torch.equal(a, b), i


@pytest.mark.gpu
def test_generate_eos_stop_with_sparse_checks():
    """generate() tests 'all rows finished' every 16 tokens and trims the padding-only steps it ran
    past the stop: the result equals the per-step-checked loop (an eos that every row emits)."""
    cfg = O.config_small_gpu()
    m = _model(6)
    ids, mask, pix, _ = O.make_inputs(cfg, 2, 20, 3, 23)
    kw = dict(input_ids=ids.cuda(), pixel_values=pix.cuda(), attention_mask=mask.cuda(), max_new_tokens=40)
    free = m.generate(**kw)
    eos = int(free[0, 23])  # row 0's 4th new token: row 1 may finish later or never (then no stop)
    out = m.generate(**kw, eos_token_id=eos)
    gen = out[:, 20:].cpu()
    fin = torch.cumsum((gen == eos).long(), 1) > 0
    all_done = fin.all(0)
    if bool(all_done.any()):
        stop = int(all_done.long().argmax())
        assert gen.shape[1] == stop + 1  # stopped exactly where the per-step loop would
    else:
        assert gen.shape[1] == 40
    # rows that finished are padded after their eos
    for r in range(2):
        hit = (gen[r] == eos).nonzero()
        if len(hit):
            assert (gen[r, int(hit[0]) + 1:] == cfg.pad_token_id).all()


@pytest.mark.gpu
@pytest.mark.parametrize("M", [1, 3, 8, 16])
def test_decode_linear_fused_transforms_bitwise(M):
    """cullavo_decode_linear's fused input transforms give bitwise the unfused path's values:
    RMSNorm (cullavo_rmsnorm_fwd then the GEMV) and SwiGLU (cullavo_swiglu_fwd then the GEMV), with
    and without a residual; plus the plain GEMV against fp32."""
    from cullavo_amd import ops
    g = torch.Generator().manual_seed(40 + M)
    d, F = 4096, 11008
    h = (torch.randn(M, d, generator=g) * 3).to(BF).cuda()
    nw = (1 + 0.1 * torch.randn(d, generator=g)).to(BF).cuda()
    Wq = (torch.randn(3 * 1024, d, generator=g) * d ** -0.5).to(BF).cuda()
    gu = torch.randn(M, 2 * F, generator=g).to(BF).cuda()
    Wd = (torch.randn(d, F, generator=g) * F ** -0.5).to(BF).cuda()
    res = torch.randn(M, d, generator=g).to(BF).cuda()
    x1, _ = ops.rmsnorm_fwd(h, nw, 1e-5)
    norm_fits = M * (d + 8) * 2 <= 65536  # the normalised rows are staged in LDS
    if norm_fits:
        a = ops.decode_linear(h, Wq, transform=1, norm_w=nw, eps=1e-5)
        b = ops.decode_linear(x1, Wq)
        assert torch.equal(a, b)
    else:
        with pytest.raises(ValueError):
            ops.decode_linear(h, Wq, transform=1, norm_w=nw, eps=1e-5)
    act = ops.swiglu_fwd(gu)
    for r in (None, res):
        a = ops.decode_linear(gu, Wd, transform=2, residual=r)
        b = ops.decode_linear(act, Wd, residual=r)
        assert torch.equal(a, b)
    # the widest product (gate|up: 16-wave workgroups) and the plain linear's dispatch agree too
    Wgu = (torch.randn(2 * F, d, generator=g) * d ** -0.5).to(BF).cuda()
    if norm_fits:
        a = ops.decode_linear(h, Wgu, transform=1, norm_w=nw, eps=1e-5)
        assert torch.equal(a, ops.linear(x1, Wgu))
        # RMSNorm in, SwiGLU out (transform 4): the whole gate|up half of the decode MLP
        a = ops.decode_linear(h, Wgu, transform=4, norm_w=nw, eps=1e-5)
        assert torch.equal(a, ops.swiglu_fwd(ops.linear(x1, Wgu)))
    assert torch.equal(ops.decode_linear(act, Wd, residual=res), ops.linear(act, Wd, residual=res))
    z = x1.float() @ Wq.float().T
    y = ops.decode_linear(x1, Wq)
    assert (y.float() - z).abs().max().item() <= 8e-3 * z.abs().max().item()
    with pytest.raises(ValueError):
        ops.decode_linear(torch.zeros(17, d, dtype=BF, device="cuda"), Wq)


@pytest.mark.gpu
@pytest.mark.parametrize("Lnew", [1, 2])
def test_rope_kv_append_bitwise(Lnew):
    """cullavo_rope_kv_append (the decode step's RoPE + cache append in one launch) leaves q and
    the caches bitwise as cullavo_rope followed by cullavo_kv_append: q / k / v as column blocks of
    one fused projection output, per-sequence cache rows start[b], ragged positions."""
    import torch
    from cullavo_amd import ops
    B, H, D, Lmax = 3, 4, 128, 40
    d = H * D
    g = torch.Generator().manual_seed(5)
    qkv = torch.randn(B * Lnew, 3 * d, generator=g).bfloat16().cuda()
    pos = torch.tensor([7, 19, 33, 2, 5, 30][:B * Lnew], dtype=torch.int64).cuda()
    start = torch.tensor([3, 0, 17], dtype=torch.int32).cuda()
    caches = [torch.randn(B, Lmax, d, generator=g).bfloat16().cuda() for _ in range(2)]
    a = qkv.clone()
    ka, va = caches[0].clone(), caches[1].clone()
    ops.rope(a[:, :d], a[:, d:2 * d], pos, hq=H, hk=H, head_dim=D, theta=10000.0)
    ops.kv_append(a[:, d:2 * d], a[:, 2 * d:], ka, va, start, B=B, Lnew=Lnew)
    b2 = qkv.clone()
    kb, vb = caches[0].clone(), caches[1].clone()
    ops.rope_kv_append(b2[:, :d], b2[:, d:2 * d], b2[:, 2 * d:], pos, kb, vb, start, hq=H, head_dim=D, theta=10000.0,
                       B=B, Lnew=Lnew)
    torch.cuda.synchronize()
    assert torch.equal(a[:, :d], b2[:, :d])
    assert torch.equal(ka, kb) and torch.equal(va, vb)


@pytest.mark.gpu
@pytest.mark.parametrize("M,F,K", [(1, 11008, 4096), (3, 264, 1000), (8, 11008, 4096), (16, 776, 520)])
def test_decode_linear_swiglu_output_bitwise(M, F, K):
    """cullavo_decode_linear transform 3 (the gate|up product with the SwiGLU in its epilogue, the
    decode step's default) is bitwise swiglu_fwd(gate|up product) of the unfused path."""
    import torch
    from cullavo_amd import ops
    g = torch.Generator().manual_seed(M + F)
    x = torch.randn(M, K, generator=g).bfloat16().cuda()
    w = (torch.randn(2 * F, K, generator=g) * K ** -0.5).bfloat16().cuda()
    ref = ops.swiglu_fwd(ops.gemm_ex(0, 0, M, 2 * F, K, x, K, w, K, torch.empty(M, 2 * F, dtype=torch.bfloat16,
                                                                                  device="cuda"), 2 * F))
    out = ops.decode_linear(x, w, transform=3)
    torch.cuda.synchronize()
    assert out.shape == (M, F)
    assert torch.equal(out, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("starts", [(3, 0, 17), (63, 64, 127), (1100, 5, 640)])
def test_attn_decode_rope_bitwise(starts):
    """cullavo_attn_decode_rope (RoPE + cache append + split-KV attention in one pass, the decode
    step's default) gives bitwise the output and cache rows of rope_kv_append + attn_decode with
    kv_len = start + 1: new rows at chunk edges (63 / 64 / 127), left padding (kv_start), a
    max_len past every length (empty chunks), q left unrotated."""
    import torch
    from cullavo_amd import ops
    B, H, D = 3, 4, 128
    d = H * D
    Lmax = max(starts) + 70
    g = torch.Generator().manual_seed(sum(starts))
    qkv = torch.randn(B, 3 * d, generator=g).bfloat16().cuda()
    pos = torch.tensor([s + 2 for s in starts], dtype=torch.int64).cuda()
    start = torch.tensor(starts, dtype=torch.int32).cuda()
    kv_start = torch.tensor([0, min(starts[1], 2), 1], dtype=torch.int32).cuda()
    caches = [torch.randn(B, Lmax, d, generator=g).bfloat16().cuda() for _ in range(2)]
    a = qkv.clone()
    ka, va = caches[0].clone(), caches[1].clone()
    ops.rope_kv_append(a[:, :d], a[:, d:2 * d], a[:, 2 * d:], pos, ka, va, start, hq=H, head_dim=D, theta=10000.0,
                       B=B, Lnew=1)
    oa = ops.attn_decode(a[:, :d], ka, va, start + 1, B=B, H=H, D=D, max_len=Lmax, scale=D ** -0.5, kv_start=kv_start)
    b2 = qkv.clone()
    kb, vb = caches[0].clone(), caches[1].clone()
    ob = ops.attn_decode_rope(b2[:, :d], b2[:, d:2 * d], b2[:, 2 * d:], pos, kb, vb, start, B=B, H=H, D=D,
                              max_len=Lmax, scale=D ** -0.5, theta=10000.0, kv_start=kv_start)
    torch.cuda.synchronize()
    assert torch.equal(b2, qkv)  # q, k, v read only
    assert torch.equal(ka, kb) and torch.equal(va, vb)
    assert torch.equal(oa, ob)


@pytest.mark.gpu
def test_decode_default_fusions_bitwise(monkeypatch):
    """The default decode fusions (SwiGLU in the gate|up product's epilogue, RoPE + append inside
    decode attention) give bitwise the logits of the separate kernels, eager and graph-replayed."""
    from cullavo_amd import generation
    cfg = O.config_small_gpu()
    m = _model(6)
    ids, mask, pix, _ = O.make_inputs(cfg, 2, 20, 3, 31)
    ids, mask, pix = ids.cuda(), mask.cuda(), pix.cuda()
    toks = torch.randint(2, cfg.image_token_index, (4, 2), generator=torch.Generator().manual_seed(9)).cuda()
    runs = []
    for fuse in (False, True):
        monkeypatch.setattr(generation, "FUSE_DECODE_GU", fuse)
        monkeypatch.setattr(generation, "FUSE_DECODE_ROPE", fuse)
        cache = m(input_ids=ids, pixel_values=pix, attention_mask=mask, use_cache=True).past_key_values
        runs.append([m(input_ids=t[:, None], past_key_values=cache, use_cache=True).logits.clone() for t in toks])
        kw = dict(input_ids=ids, pixel_values=pix, attention_mask=mask, max_new_tokens=5)
        runs.append([m.generate(**kw)])
    for i, (a, b) in enumerate(zip(runs[0], runs[2])):
        assert torch.equal(a, b), i
    assert torch.equal(runs[1][0], runs[3][0])
