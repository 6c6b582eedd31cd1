"""End-to-end parity of CuLLaVOModel (bf16 on the gfx950 kernels) against the bf16-faithful
oracle (oracle/cullavo_oracle.py on the reference's bf16 rounding points, autograd for the
gradients) and the reference's own fp32 forward/backward (golden fixtures from
tests/golden/make_golden.py).

Gates (SURVEY.md §7 "Parity tolerance", bf16 production mode):
* vs the bf16-faithful oracle on the same weights/inputs: logits rel-L2 <= 1e-2 on attended
  positions, |dloss| <= 1e-2, every trainable parameter's gradient rel-L2 <= 2e-2;
* vs the reference's fp32 golden (cross-precision: the bf16-faithful oracle itself sits at
  logits 1.06e-2 from it, tools/bf16_noise_floor.py): logits <= 2e-2, |dloss| <= 1e-2,
  gradient norms within 3e-2.
The f32 parity mode is gated at the north star's 1e-3 in tests/test_parity_modes.py.
"""
import os

import numpy as np
import pytest
import torch

from oracle import cullavo_oracle as O

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def rel_l2(a, b):
    a = a.detach().float().cpu() if torch.is_tensor(a) else torch.as_tensor(np.asarray(a, dtype=np.float32))
    b = b.detach().float().cpu() if torch.is_tensor(b) else torch.as_tensor(np.asarray(b, dtype=np.float32))
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def build(trainable="full", seed=2):
    from cullavo_amd.arch_cullavo import CuLLaVOModel
    from cullavo_amd.config import tiny_gpu
    m = CuLLaVOModel(tiny_gpu(), device="cuda", trainable=trainable, init="none")
    m.load_state_dict(O.make_weights(O.config_small_gpu(), seed))
    return m


def inputs(seed=2, batch=2, text_len=40, image_col=4, pad_tail=None):
    ids, mask, pix, labels = O.make_inputs(O.config_small_gpu(), batch, text_len, image_col, seed, pad_tail=pad_tail)
    return ids.cuda(), mask.cuda(), pix.cuda(), labels.cuda()


def oracle_bf16(seed, ids, mask, pix, labels):
    """bf16-faithful oracle forward + backward: (loss, logits, aux, {key: grad})"""
    cfg = O.config_small_gpu()
    Wb = {k: v.requires_grad_(True) for k, v in O.to_bf16(O.make_weights(cfg, seed)).items()}
    cpu = [t.cpu() if t is not None else None for t in (ids, mask, pix, labels)]
    loss, logits, aux = O.forward(Wb, cfg, cpu[0], cpu[2], cpu[1], cpu[3])
    loss.backward()
    return loss, logits, aux, {k: v.grad for k, v in Wb.items()}


def check_grads(m, ref_grads, tol=2e-2, arenas=None):
    """every trainable parameter's gradient vs the oracle's (rel-L2); returns the worst error"""
    worst, n = 0.0, 0
    for name, ar in m.arenas.items():
        if not ar.trainable or (arenas is not None and name not in arenas):
            continue
        for k, p in ar.params.items():
            ref = ref_grads.get(k)
            if ref is None or float(ref.float().norm()) == 0.0:
                assert p.grad is None or float(p.grad.float().abs().max()) == 0.0, k
                continue
            err = rel_l2(p.grad, ref)
            worst = max(worst, err)
            assert err <= tol, (k, err)
            n += 1
    assert n > 0
    return worst


def test_forward_backward_matches_bf16_oracle():
    m = build()
    ids, mask, pix, labels = inputs()
    out = m(input_ids=ids, pixel_values=pix, attention_mask=mask, labels=labels)
    loss_ref, logits_ref, aux, grads = oracle_bf16(2, ids, mask, pix, labels)
    valid = aux["attention_mask"].bool()
    err = rel_l2(out.logits.float().cpu()[valid], logits_ref.float()[valid])
    assert err <= 1e-2, err
    assert abs(out.loss.item() - loss_ref.item()) <= 1e-2, (out.loss.item(), loss_ref.item())
    out.loss.backward()
    worst = check_grads(m, grads)
    print(f"bf16 vs bf16-faithful oracle: logits {err:.2e}, dloss {abs(out.loss.item() - loss_ref.item()):.2e}, "
          f"worst grad {worst:.2e}")


def test_forward_backward_matches_reference_golden():
    """cross-precision: bf16 production path vs the reference's own fp32 forward/backward"""
    g = np.load(os.path.join(GOLD, "small_gpu.npz"))
    m = build()
    ids, mask, pix, labels = inputs()
    out = m(input_ids=ids, pixel_values=pix, attention_mask=mask, labels=labels)
    assert tuple(out.logits.shape) == tuple(g["logits_shape"])
    assert abs(out.loss.item() - float(g["loss"][0])) <= 1e-2, (out.loss.item(), float(g["loss"][0]))
    rows = torch.as_tensor(g["logits_rows"])
    sample = out.logits.detach()[:, rows].float().cpu().numpy()
    assert rel_l2(sample, g["logits_sample"]) <= 2e-2
    out.loss.backward()
    params = {}
    for ar in m.arenas.values():
        params.update(ar.params)
    checked = 0
    for key in g.files:
        if key.startswith("gradnorm/"):
            k = key[len("gradnorm/"):]
            ref = float(g[key][0])
            p = params[k]
            if not p.requires_grad:
                continue  # vision tower frozen in the "full" policy
            ours = p.grad.float().norm().item()
            assert abs(ours - ref) <= 3e-2 * ref + 1e-6, (k, ours, ref)
            checked += 1
    # element-level: the reference's own sampled fp32 gradients (fixed-stride samples of the large
    # tensors) against this bf16 path, so a bug shared by the kernels and the bf16-faithful
    # oracle cannot hide. Cross-precision tolerance: bf16 activations and weights through the
    # whole backward chain put the sampled elements ~1e-2 away (rel-L2); gate 5e-2.
    worst, n_el = 0.0, 0
    for key in g.files:
        if key.startswith("grad/"):
            k = key[len("grad/"):]
            if not params[k].requires_grad:
                continue
            stride = int(g["gradstride/" + k][0])
            ours = params[k].grad.reshape(-1)[::stride].float().cpu()
            err = rel_l2(ours, g[key])
            assert err <= 5e-2, (k, err)
            worst, n_el = max(worst, err), n_el + 1
    assert checked > 10 and n_el > 0
    print(f"bf16 vs reference fp32 golden: worst sampled-gradient rel-L2 {worst:.2e} over {n_el} tensors")


def test_right_padded_batch_matches_oracle():
    ids, mask, pix, labels = (t.cuda() for t in O.make_inputs(O.config_small_gpu(), 2, 48, 3, 3, pad_tail=[0, 9]))
    loss_ref, logits_ref, aux, grads = oracle_bf16(3, ids, mask, pix, labels)
    m = build(seed=3)
    out = m(input_ids=ids, pixel_values=pix, attention_mask=mask, labels=labels)
    valid = aux["attention_mask"].bool()
    ours = out.logits.detach().float().cpu()[valid]
    assert rel_l2(ours, logits_ref.detach().float()[valid]) <= 1e-2
    assert abs(out.loss.item() - loss_ref.item()) <= 1e-2
    out.loss.backward()
    check_grads(m, grads)


def test_return_dict_false_and_select_strategy_error():
    m = build()
    ids, mask, pix, labels = inputs()
    tup = m(input_ids=ids, pixel_values=pix, attention_mask=mask, labels=labels, return_dict=False)
    assert tup[0].dim() == 0 and tup[1].dim() == 3
    with pytest.raises(ValueError, match="Unexpected select feature strategy"):
        m(input_ids=ids, pixel_values=pix, attention_mask=mask, vision_feature_select_strategy="bogus")
    with pytest.raises(ValueError, match="number of image tokens"):
        m(input_ids=ids, pixel_values=pix[:1], attention_mask=mask, labels=labels)


def test_reference_trainable_policy_grads():
    """frozen base: only projector / embed_tokens / lm_head receive gradients"""
    m = build(trainable="reference")
    ids, mask, pix, labels = inputs()
    out = m(input_ids=ids, pixel_values=pix, attention_mask=mask, labels=labels)
    out.loss.backward()
    _, _, _, grads = oracle_bf16(2, ids, mask, pix, labels)
    check_grads(m, grads)
    assert {n for n, a in m.arenas.items() if a.trainable} == {"projector", "head", "embed"}
    assert not m.arenas["layers"].trainable


def test_full_size_layer_shapes_run():
    """one full-width Vicuna-7B decoder layer and one CLIP-L layer (B=1) through the whole model
    at config-3 shapes (L = 1088, vocab 32064) fwd+bwd: output shapes, finite loss and non-zero
    finite gradients, and the forward (logits, loss) against the bf16-faithful oracle at this
    width; per-layer gradient parity at these widths is tests/test_full_size.py's."""
    from cullavo_amd.config import CuLLaVOConfig, CLIPVisionConfig, LlamaConfig
    from cullavo_amd.arch_cullavo import CuLLaVOModel
    cfg = CuLLaVOConfig(vision_config=CLIPVisionConfig(num_hidden_layers=2),
                        text_config=LlamaConfig(num_hidden_layers=1, vocab_size=32064))
    m = CuLLaVOModel(cfg, device="cuda", trainable="full", init="random", seed=0)
    ids = torch.randint(2, 32000, (1, 513), device="cuda")
    ids[0, 35] = 32000
    pix = torch.randn(1, 3, 336, 336, device="cuda")
    labels = torch.full((1, 1088), -100, device="cuda", dtype=torch.long)
    labels[0, 611:] = torch.randint(2, 32000, (477,), device="cuda")
    out = m(input_ids=ids, pixel_values=pix, attention_mask=torch.ones_like(ids), labels=labels)
    assert out.logits.shape == (1, 1088, 32064)
    assert torch.isfinite(out.loss)
    # forward parity at full width: the bf16-faithful oracle on the same weights and inputs
    W = {}
    for ar in m.arenas.values():
        W.update({k: v.detach().cpu() for k, v in ar.params.items()})
    ocfg = O.CuLLaVOCfg(vision=O.VisionCfg(num_hidden_layers=2), text=O.TextCfg(num_hidden_layers=1))
    with torch.no_grad():
        loss_ref, logits_ref, _ = O.forward(W, ocfg, ids.cpu(), pix.cpu(), torch.ones_like(ids).cpu(), labels.cpu())
    err = rel_l2(out.logits.detach()[0], logits_ref[0])
    assert err <= 1e-2, err
    assert abs(out.loss.item() - loss_ref.item()) <= 1e-2, (out.loss.item(), loss_ref.item())
    out.loss.backward()
    gflat = m.arenas["layers"].grad_flat
    assert torch.isfinite(gflat.float()).all()
    assert gflat.float().abs().sum() > 0


def test_kmajor_weight_copies_bitwise_and_refreshed(monkeypatch):
    """The decoder layers' dX GEMMs from K-major weight copies (side-stream or synchronous
    refresh) give gradients bitwise equal to the N-major path over two AdamW steps (the copies are
    re-made after each step) and after an in-place torch write to a layer weight."""
    import cullavo_amd.modeling as MD
    from cullavo_amd.optim import FusedAdamW
    ids, mask, pix, labels = inputs()
    grads = {}
    for mode in ("off", "sync", "side"):
        monkeypatch.setattr(MD, "KMAJOR_MODE", mode)
        m = build()
        opt = FusedAdamW(list(m.arenas.values()), lr=1e-3)
        seen = []
        for step in range(3):
            if step == 2:
                with torch.no_grad():
                    m.arenas["layers"].params["language_model.model.layers.0.mlp.down_proj.weight"].mul_(0.5)
            opt.zero_grad()
            out = m(input_ids=ids, pixel_values=pix, attention_mask=mask, labels=labels)
            out.loss.backward()
            torch.cuda.synchronize()
            seen.append(m.arenas["layers"].grad_flat.clone())
            opt.step()
        grads[mode] = seen
    for mode in ("sync", "side"):
        for s, (a, b) in enumerate(zip(grads["off"], grads[mode])):
            assert torch.equal(a, b), f"mode {mode} step {s}"


def test_fused_swiglu_bwd_bitwise(monkeypatch):
    """The decoder layers' SwiGLU backward fused into the down-projection dX GEMM epilogue
    (functions.FUSED_SWIGLU_BWD, the default) gives gradients bitwise equal to the separate
    swiglu_bwd kernel (full fine-tune; with a LoRA adapter on down_proj the unfused path runs)."""
    import cullavo_amd.functions as FN
    ids, mask, pix, labels = inputs()
    for trainable in ("full",):
        grads = {}
        for fused in (True, False):
            monkeypatch.setattr(FN, "FUSED_SWIGLU_BWD", fused)
            m = build(trainable=trainable)
            out = m(input_ids=ids, pixel_values=pix, attention_mask=mask, labels=labels)
            out.loss.backward()
            torch.cuda.synchronize()
            grads[fused] = {k: a.grad_flat.clone() for k, a in m.arenas.items()
                            if getattr(a, "grad_flat", None) is not None}
        assert grads[True].keys() == grads[False].keys()
        for k in grads[True]:
            assert torch.equal(grads[True][k], grads[False][k]), f"{trainable} arena {k}"


def test_dw_side_stream_bitwise(monkeypatch):
    """Weight-gradient GEMMs on the side stream (functions.DW_STREAM "side") give gradients and
    AdamW updates bitwise equal to the single-stream path, read on the compute stream right
    after backward() with no device sync (the end-of-backward join orders them), including an
    accumulating second micro-batch (beta = 1 writes)."""
    import cullavo_amd.functions as FN
    from cullavo_amd.optim import FusedAdamW
    ids, mask, pix, labels = inputs()
    ids2, mask2, pix2, labels2 = inputs(seed=5)
    res = {}
    for mode in ("off", "side", "swg"):  # swg: only the down-projection dW, beside the SwiGLU dX GEMM
        monkeypatch.setattr(FN, "DW_STREAM", "off" if mode == "swg" else mode)
        monkeypatch.setattr(FN, "SWG_OVERLAP", mode == "swg")
        m = build()
        opt = FusedAdamW(list(m.arenas.values()), lr=1e-3)
        seen = []
        for step in range(2):
            opt.zero_grad()
            for (a, b, c, d) in ((ids, mask, pix, labels), (ids2, mask2, pix2, labels2)):
                out = m(input_ids=a, pixel_values=c, attention_mask=b, labels=d)
                out.loss.backward()
                seen.append(torch.cat([ar.grad_flat.clone() for ar in m.arenas.values() if ar.trainable]))
            opt.step()
        seen.append(torch.cat([ar.flat.clone() for ar in m.arenas.values()]))
        res[mode] = seen
    for other in ("side", "swg"):
        for i, (a, b) in enumerate(zip(res["off"], res[other])):
            assert torch.equal(a, b), (other, i)


def test_adamw_overlap_bitwise():
    """FusedAdamW(overlap=True): the update runs on a side stream per decoder layer and the next
    forward waits per layer; parameters, moments and losses over three steps are bitwise equal to
    the in-stream update (synchronize() before reading parameters outside a forward)."""
    from cullavo_amd.optim import FusedAdamW
    ids, mask, pix, labels = inputs()
    res = {}
    for overlap in (False, True):
        m = build()
        opt = FusedAdamW(list(m.arenas.values()), lr=1e-3, overlap=overlap)
        losses = []
        for _ in range(3):
            opt.zero_grad()
            out = m(input_ids=ids, pixel_values=pix, attention_mask=mask, labels=labels)
            out.loss.backward()
            opt.clip_grad_norm_(1.0)
            opt.step()
            losses.append(out.loss.detach().clone())
        opt.synchronize()
        res[overlap] = (torch.stack(losses), torch.cat([a.flat.float() for a in m.arenas.values()]),
                        torch.cat([torch.cat([mm.float(), vv.float()]) for mm, vv in opt.flat_state]))
    for a, b in zip(res[False], res[True]):
        assert torch.equal(a, b)


def test_adamw_skips_parameters_without_gradient():
    """A text-only batch never reaches the projector: like torch.optim.AdamW on a parameter
    whose .grad is None, FusedAdamW leaves it (and its step count) untouched, while the
    decoder layers move; the next image batch steps the projector at its own step 1."""
    from cullavo_amd.optim import FusedAdamW
    m = build()
    opt = FusedAdamW(list(m.arenas.values()), lr=1e-3)
    ids, mask, pix, labels = inputs()
    t_ids = ids.clone()
    t_ids[t_ids == 1000] = 7
    proj0 = m.arenas["projector"].flat.clone()
    lay0 = m.arenas["layers"].flat.clone()
    out = m(input_ids=t_ids, attention_mask=mask, labels=labels[:, -t_ids.shape[1]:])
    out.loss.backward()
    for a in m.arenas.values():
        a.finalize_grads()
    opt.step()
    opt.zero_grad()
    torch.cuda.synchronize()
    assert torch.equal(m.arenas["projector"].flat, proj0)
    assert not torch.equal(m.arenas["layers"].flat, lay0)
    pi = [a.name for a in opt.arenas].index("projector")
    assert set(opt.key_steps[pi].values()) == {0}
    out = m(input_ids=ids, pixel_values=pix, attention_mask=mask, labels=labels)
    out.loss.backward()
    for a in m.arenas.values():
        a.finalize_grads()
    opt.step()
    torch.cuda.synchronize()
    assert not torch.equal(m.arenas["projector"].flat, proj0)
    assert set(opt.key_steps[pi].values()) == {1}
    li = [a.name for a in opt.arenas].index("layers")
    assert set(opt.key_steps[li].values()) == {2}


def test_from_pretrained_forward_matches_oracle(tmp_path):
    """llava-hf checkpoint directory (config.json + two safetensors shards in the nested >= 4.45
    key layout, weights as the reference's bf16 cast) -> CuLLaVOModel.from_pretrained streams it
    into HBM -> the forward equals the bf16-faithful oracle on the same tensors (reference
    cullavo/load_cullavo.py:86 from_pretrained, then arch_cullavo.py:546-677)."""
    import json
    from safetensors.torch import save_file

    from cullavo_amd.arch_cullavo import CuLLaVOModel
    cfg = O.config_small_gpu()
    W = O.to_bf16(O.make_weights(cfg, 4))
    v, t = cfg.vision, cfg.text
    hf = {"model_type": "llava", "image_token_index": cfg.image_token_index, "pad_token_id": cfg.pad_token_id,
          "vision_feature_layer": -2, "vision_feature_select_strategy": "default", "projector_hidden_act": "gelu",
          "vision_config": {"image_size": v.image_size, "patch_size": v.patch_size, "hidden_size": v.hidden_size,
                            "num_hidden_layers": v.num_hidden_layers, "num_attention_heads": v.num_attention_heads,
                            "intermediate_size": v.intermediate_size, "hidden_act": "quick_gelu"},
          "text_config": {"hidden_size": t.hidden_size, "num_hidden_layers": t.num_hidden_layers,
                          "num_attention_heads": t.num_attention_heads, "intermediate_size": t.intermediate_size,
                          "vocab_size": t.vocab_size, "rms_norm_eps": t.rms_norm_eps, "rope_theta": t.rope_theta}}
    (tmp_path / "config.json").write_text(json.dumps(hf))

    def new_layout(k):  # transformers >= 4.45 nested LlavaModel names
        if k.startswith(("vision_tower.", "multi_modal_projector.")):
            return "model." + k
        if k.startswith("language_model.model."):
            return "model.language_model." + k[len("language_model.model."):]
        return k[len("language_model."):]  # lm_head
    keys = sorted(W)
    for i, part in enumerate((keys[:len(keys) // 2], keys[len(keys) // 2:])):
        save_file({new_layout(k): W[k].contiguous() for k in part}, str(tmp_path / f"model-0000{i + 1}-of-00002.safetensors"))
    m = CuLLaVOModel.from_pretrained(str(tmp_path), device="cuda", trainable="none")
    for k, p in m.state_dict().items():
        assert torch.equal(p.cpu(), W[k]), k
    ids, mask, pix, labels = O.make_inputs(cfg, 2, 40, 4, 4)
    loss_ref, logits_ref, aux = O.forward(W, cfg, ids, pix, mask, labels)
    with torch.no_grad():
        out = m(input_ids=ids.cuda(), pixel_values=pix.cuda(), attention_mask=mask.cuda(), labels=labels.cuda())
    assert rel_l2(out.logits.float().cpu(), logits_ref.float()) <= 1e-2
    assert abs(out.loss.item() - loss_ref.item()) <= 1e-2
