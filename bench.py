"""CuLLaVO train-step throughput on MI355X (BASELINE.json metric):
"train-step samples/sec (336px img + 512-tok prompt, 7B LM) at 1/2/4/8 MI355X".

A step = one full training step of CuLLaVOModel (llava-1.5-7b: CLIP ViT-L/14-336 + Vicuna-7B)
on one synthetic batch resident in HBM: vision forward (frozen), projector, merge, 32 decoder
layers, lm_head + shifted masked CE, the complete backward, bucketed RCCL gradient all-reduce
(N>1), global-norm clip and fused AdamW. Per-GPU batch 8 (config 3; config 4 at N=8 = global
64), weak scaling. Random-init weights (no checkpoints offline), synthetic data.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

`--gpus N > 1` without a launcher env (no WORLD_SIZE) starts the N ranks itself, before this process
touches the GPU: a child `python -m torch.distributed.run --nnodes=1 --nproc-per-node N
--master-addr 127.0.0.1` of this same script (the reference launches its own ranks the same way,
/root/reference/run:59-71 `accelerate launch --num_processes`); rank 0's JSON line is forwarded
and the child's exit code returned. A formed world that differs from --gpus is an error (exit 3).

At N = 1 the default run also times the other BASELINE workloads, each in a child process started
before this process touches the GPU (so their memory never overlaps): config 2 (CLIP ViT-L/14-336
encoder, bs 64), config 5 (ViT-L + Llama-2-13B, L = 1600, bs 4) and the reference's own recipe on
config 3 (LoRA r=64 + projector / lm_head / embed, frozen base). They are reported under
"workloads", each with its own roofline object; the headline (metric / value) stays config 3.

Prints ONE compact JSON line on rank 0, the last line of stdout (<= 4 KiB, so a driver that keeps
the tail of stdout always holds it whole): the headline, its roofline, the decoder-layer roofline,
cpu_baseline, a one-line summary per sub-workload and (N > 1) the exchange. The full record (every
GEMM family and shape with its library ceiling, each sub-workload's own full record) goes to the
sidecar file --detail-out (default gpurun_out/bench_detail.json), named in the line's "detail".
See README / DESIGN.md §Measurement for every field.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md; no sparsity)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=8, help="samples per GPU")
    ap.add_argument("--config", default="llava-1.5-7b")
    ap.add_argument("--trainable", default="full", choices=["full", "reference", "lora"])
    ap.add_argument("--text-len", type=int, default=513)
    ap.add_argument("--bucket-mb", type=int, default=256)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--high-prio", action="store_true",
                    help="run the training step on a high-priority HIP stream (the optimizer's side stream "
                         "stays at the default priority; A/B experiment)")
    ap.add_argument("--overlap", action="store_true",
                    help="run the optimizer update on a side stream under the next forward (A/B; off by default)")
    ap.add_argument("--no-overlap", action="store_true",
                    help="optimizer update in-stream (the default; kept for A/B scripts)")
    ap.add_argument("--workload", default="step", choices=["step", "vit", "decode"],
                    help="step: the training step (default; configs 3/4/5 by --config/--batch/--text-len); "
                         "vit: BASELINE config 2, the CLIP ViT-L/14-336 encoder forward at bs=--batch (64); "
                         "decode: 7B KV-cache decode (the step-2-pre generate path) at batch --batch")
    ap.add_argument("--sub-workloads", default=",".join(SUB_WORKLOADS),
                    help="N=1 headline runs only: the other workloads timed in child processes ('' = none)")
    ap.add_argument("--no-sub", action="store_true", help="time this workload only")
    ap.add_argument("--detail-out", default=os.path.join(REPO, "gpurun_out", "bench_detail.json"),
                    help="sidecar file for the full record ('' = none); the stdout line stays compact")
    ap.add_argument("--launch-probe", action="store_true",
                    help="launcher self-test: form the world, all-reduce one tensor on the host, print one "
                         "JSON line on rank 0 (no GPU work; tests/test_bench_launch.py)")
    return ap.parse_args(argv)


# the other BASELINE workloads a default N = 1 run reports beside the config-3 headline
SUB_WORKLOADS = {
    "config2-vit": ["--workload", "vit", "--batch", "64"],
    "config5-full": ["--config", "llava-1.5-13b", "--batch", "4", "--text-len", "1025"],
    "config3-lora": ["--trainable", "lora"],
    "decode-b1": ["--workload", "decode", "--batch", "1"],
    "decode-b8": ["--workload", "decode", "--batch", "8"],
}


def workload_key(args) -> str:
    """the key PMC records are filed under (profiles/roofline_traffic.json)"""
    if args.workload == "vit":
        return "config2-vit"
    if args.workload == "decode":
        return f"decode-b{args.batch}"
    return f"{'config5' if '13b' in args.config else 'config3'}-{args.trainable}"


def run_sub_workloads(args, names):
    """Each workload in its own child process (sequentially, before this process initialises the
    GPU), its one JSON line parsed and condensed; a failing child is reported, not fatal."""
    import subprocess
    import tempfile
    out = {}
    for name in names:
        fd, side = tempfile.mkstemp(prefix=f"bench_{name}_", suffix=".json")
        os.close(fd)
        cmd = [sys.executable, os.path.abspath(__file__), "--no-sub", "--no-cpu-baseline", "--detail-out", side,
               "--steps", str(min(args.steps, 10)), "--warmup", str(min(args.warmup, 3)), *SUB_WORKLOADS[name]]
        t0 = time.perf_counter()
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
            lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            if r.returncode != 0 or not lines:
                out[name] = {"error": f"rc {r.returncode}: {(r.stderr or r.stdout)[-400:]}"}
                continue
            try:
                rec = json.load(open(side))  # the child's full record
            except (OSError, ValueError):
                rec = json.loads(lines[-1])
        except subprocess.TimeoutExpired:
            out[name] = {"error": "timed out after 600 s"}
            continue
        finally:
            if os.path.exists(side):
                os.remove(side)
        rec.pop("detail", None)
        rec["wall_s"] = round(time.perf_counter() - t0, 1)
        out[name] = rec
    return out


# ---- the compact headline line ----------------------------------------------------------------
LINE_LIMIT = 4096  # bytes: the final stdout line must fit a driver's tail whole
HEAD_KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
             "vs_baseline", "dtype", "data", "config", "model_tflops_per_gpu", "mfu", "loss", "gflop_per_image",
             "prefill_ms")
ROOF_KEYS = ("kernel", "bound", "achieved", "peak", "unit", "frac", "traffic", "algorithmic_bytes", "mfma_busy",
             "avg_ms", "launches_timed", "library_ceiling")


def _short(s, n):
    s = str(s)
    return s if len(s) <= n else s[:n - 3] + "..."


def workload_summary(rec: dict) -> dict:
    """one sub-workload in a few fields: its value, step time and the frac of its roofline kernel"""
    if "error" in rec:
        return {"error": _short(rec["error"], 160)}
    roof = rec.get("roofline") or {}
    out = {"value": rec.get("value"), "unit": rec.get("unit"), "ms_per_step": rec.get("ms_per_step"),
           "roofline_frac": roof.get("frac"), "bound": roof.get("bound"), "kernel": _short(roof.get("kernel", ""), 48)}
    if "mfu" in rec:
        out["mfu"] = rec["mfu"]
    if "step_roofline" in rec:
        out["step_roofline_frac"] = rec["step_roofline"].get("frac")
    return out


def compact_line(full: dict) -> dict:
    """The final stdout line built from the full record: headline fields, the roofline without its
    per-family tables, layer_roofline, cpu_baseline, exchange, one summary per sub-workload."""
    line = {k: full[k] for k in HEAD_KEYS if k in full}
    if isinstance(line.get("config"), dict) and "workload" in line["config"]:
        line["config"] = dict(line["config"], workload=_short(line["config"]["workload"], 220))
    roof = full.get("roofline") or {}
    line["roofline"] = {k: roof[k] for k in ROOF_KEYS if k in roof}
    if "kernel" in line["roofline"]:
        line["roofline"]["kernel"] = _short(line["roofline"]["kernel"], 260)
    for k in ("layer_roofline", "step_roofline", "exchange"):
        if k in full:
            line[k] = full[k]
    if "traced_pass" in full:  # the instrumented pass the roofline came from (value is untraced)
        line["traced_pass"] = {k: full["traced_pass"][k] for k in ("steps", "ms_per_step") if k in full["traced_pass"]}
    if "cpu_baseline" in full:
        cb = dict(full["cpu_baseline"])
        cb["sample"] = _short(cb.get("sample", ""), 420)
        line["cpu_baseline"] = cb
    if "workloads" in full:
        line["workloads"] = {n: workload_summary(r) for n, r in full["workloads"].items()}
    if "detail" in full:
        line["detail"] = full["detail"]
    s = json.dumps(line)
    if len(s.encode()) > LINE_LIMIT:  # never let the headline outgrow the tail: drop the optional parts
        for k in ("workloads", "step_roofline", "data"):
            line.pop(k, None)
            if len(json.dumps(line).encode()) <= LINE_LIMIT:
                break
    return line


def emit(full: dict, args) -> None:
    """Full record to the sidecar (if any), then the compact line as the last line of stdout."""
    path = getattr(args, "detail_out", "")
    if path:
        try:
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
            with open(path, "w") as f:
                json.dump(full, f, indent=1)
            full = dict(full, detail=os.path.relpath(os.path.abspath(path), REPO))
        except OSError as e:
            print(f"bench.py: could not write {path}: {e}", file=sys.stderr)
    print(json.dumps(compact_line(full)), flush=True)




def vit_main(args):
    """BASELINE config 2: CLIP ViT-L/14-336 encoder, bs 64 per GPU, forward of the 23 layers
    hidden_states[-2] needs (what the CuLLaVO step runs; reference cullavo/arch_cullavo.py:586-597),
    bf16, random-init weights, synthetic pixels resident in HBM. value = images/s (all ranks)."""
    import torch
    import torch.distributed as dist

    from cullavo_amd import ops
    from cullavo_amd.arena import ParamArena
    from cullavo_amd.config import CLIPVisionConfig, CuLLaVOConfig
    from cullavo_amd.modeling import CLIPVisionTransformer, clip_specs, init_random_
    from cullavo_amd.perf import flops_per_sample, needed_vision_layers
    from cullavo_amd.trainer import init_distributed, local_device_index

    init_distributed()
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    torch.cuda.set_device(local_device_index())
    vc = CLIPVisionConfig()
    cfg = CuLLaVOConfig(vision_config=vc)
    ar = ParamArena("vision", clip_specs(vc, "vision_tower.vision_model."), device="cuda")
    init_random_({"vision": ar}, seed=0)
    vt = CLIPVisionTransformer(vc, ar.params, "vision_tower.vision_model.", ar)
    n_layers = needed_vision_layers(cfg)
    g = torch.Generator(device="cuda").manual_seed(1234 + rank)
    pix = torch.randn(args.batch, 3, vc.image_size, vc.image_size, device="cuda", generator=g)
    fl_img = flops_per_sample(cfg, 513)["vit"]
    with torch.no_grad():
        for _ in range(args.warmup):
            vt.hidden_state(pix, n_layers)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            vt.hidden_state(pix, n_layers)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        # a separate traced pass (HIP events around every GEMM launch) for the roofline
        traced_steps = max(1, min(args.steps, 3))
        ops.trace_gemm("all")
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(traced_steps):
            vt.hidden_state(pix, n_layers)
        torch.cuda.synchronize()
        traced_elapsed = time.perf_counter() - t1
    launches = ops.trace_launches()
    fams = gemm_families(launches)
    if world > 1:
        t = torch.tensor([elapsed], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    imgs = world * args.batch * args.steps
    tf = fl_img * args.batch / (elapsed / args.steps) / 1e12
    top = fams[0]
    if rank == 0:
        traffic, mfma_busy = measured_traffic(top["kernel"], workload_key(args))
        line = {
            "metric": "CLIP ViT-L/14-336 encoder images/sec (forward, hidden_states[-2])",
            "value": round(imgs / elapsed, 2), "unit": "images/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic (seeded pixels in HBM, random-init weights)",
            "config": {"workload": f"config 2: CLIP ViT-L/14-336 encoder, bs={args.batch}/GPU, 336 px, "
                                   f"{n_layers} layers (hidden_states[-2]) + patch embed, bf16, forward",
                       "model": "clip-vit-large-patch14-336", "global_batch": world * args.batch, "seq_len": 577,
                       "parallelism": f"dp{world}"},
            "model_tflops_per_gpu": round(tf, 2), "gflop_per_image": round(fl_img / 1e9, 1),
            "roofline": {"kernel": f"{top['kernel']}: {top['role']}, {len(top['shapes'])} shapes "
                                   f"{['x'.join(map(str, sh)) for sh in top['shapes']]} (M x N x K), "
                                   f"{top['launches'] // traced_steps} launches/step, "
                                   f"{100 * top['ms'] / (traced_elapsed * 1e3):.1f} % of the traced encoder time",
                         "bound": "mfma", "achieved": round(top["achieved_tflops"], 2), "peak": PEAK_BF16_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(top["achieved_tflops"] / PEAK_BF16_TFLOPS, 4),
                         "traffic": traffic, "mfma_busy": mfma_busy,
                         "algorithmic_bytes": round(top["bytes"] / top["launches"]),
                         "avg_ms": round(top["ms"] / top["launches"], 4),
                         "encoder_frac": round(tf / PEAK_BF16_TFLOPS, 4),
                         "library_ceiling": None},
            "gemm_kernels": [{"kernel": f["kernel"], "role": f["role"],
                              "share": round(f["ms"] / (traced_elapsed * 1e3), 4),
                              "achieved_tflops": round(f["achieved_tflops"], 1),
                              "library_ceiling": gemm_ceiling(f) if world == 1 else None} for f in fams[:4]],
            "gemm_shapes": gemm_shapes(launches, traced_steps),
            "traced_pass": {"steps": traced_steps, "ms_per_step": round(traced_elapsed / traced_steps * 1e3, 3)},
        }
        line["roofline"]["library_ceiling"] = line["gemm_kernels"][0]["library_ceiling"]
        emit(line, args)
    if world > 1:
        dist.destroy_process_group()


def decode_main(args):
    """KV-cache decode of the 7B LM (the step-2-pre generate() loop,
    reference cullavo/arch_cullavo.py:365 and the cached branch :605-636): prefill of the config-3
    prompt (336 px image + 513 text tokens -> 1088 merged rows) at batch --batch, then timed decode
    steps replayed from the captured HIP graph (generation.DecodeGraph). value = generated tokens/s
    over all sequences. Roofline: HBM, the weight-streaming GEMV (gemv_k) -- the bytes one launch
    must read (W, X, C) over its mean launch time, measured with HIP events on an eager step -- and
    the whole step's weight stream (13.2 GB of LM + head weights per token step / step time)."""
    import torch

    from cullavo_amd import ops
    from cullavo_amd.arch_cullavo import CuLLaVOModel
    from cullavo_amd.config import llava_1_5_7b
    from cullavo_amd.data import synthetic_batch
    from cullavo_amd.generation import DecodeGraph

    torch.cuda.set_device(0)
    cfg = llava_1_5_7b()
    m = CuLLaVOModel(cfg, device="cuda", trainable="none", init="random", seed=0)
    m.eval()
    B = args.batch
    sb = synthetic_batch(cfg, B, args.text_len, 35, seed=1234, device="cuda")
    t = cfg.text_config
    wbytes = 2 * (t.num_hidden_layers * (4 * t.hidden_size ** 2 + 3 * t.hidden_size * t.intermediate_size)
                  + t.vocab_size * t.hidden_size)
    n_tok = max(32, 8 * args.steps)
    L0 = args.text_len + cfg.vision_config.num_patches - 1
    gen = torch.Generator(device="cuda").manual_seed(7)
    with torch.no_grad():
        def prefill():
            out = m._forward_cached(sb["input_ids"], sb["pixel_values"], sb["attention_mask"], None, None, None,
                                    cfg.vision_feature_layer, cfg.vision_feature_select_strategy, None, True,
                                    max_len=L0 + n_tok + 8 * args.warmup + 8)
            return out.past_key_values, out.logits[:, -1]
        cache, logits = prefill()  # warm (allocations, first launches)
        # eager decode steps with every GEMM launch bracketed by events: the GEMV's own rate
        ops.trace_gemm("all")
        tok = torch.randint(2, 32000, (B,), device="cuda", generator=gen)
        for _ in range(4):
            logits = m(input_ids=tok[:, None], past_key_values=cache, use_cache=True).logits[:, -1]
        torch.cuda.synchronize()
        launches = ops.trace_launches()
        ops.trace_gemm(None)
        gv = [(k, ms) for k, ms in launches if k[0] <= 16 and k[3] == 0 and k[4] == 0]
        g_bytes = sum(2.0 * (k[0] * k[2] + k[1] * k[2] + k[0] * k[1]) for k, _ in gv)
        g_ms = sum(ms for _, ms in gv)
        # timed: a fresh prefill, then n_tok graph replays
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        cache, logits = prefill()
        torch.cuda.synchronize()
        prefill_ms = (time.perf_counter() - t0) * 1e3
        graph = DecodeGraph(m, cache)
        for _ in range(8 * args.warmup):
            logits = graph.step(logits.argmax(-1))[:, -1]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n_tok):
            logits = graph.step(logits.argmax(-1))[:, -1]
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
    step_s = elapsed / n_tok
    n_launch = len(gv)
    if not n_launch or g_ms <= 0:
        raise RuntimeError("decode bench: no GEMV launch was traced in the eager decode steps")
    achieved = g_bytes / (g_ms * 1e-3) / 1e9
    line = {
        "metric": f"7B KV-cache decode tokens/sec (batch {B}, {L0}-row prompt)", "value": round(B * n_tok / elapsed, 2),
        "unit": "tokens/s", "n_gpus": 1, "steps": n_tok, "warmup": 8 * args.warmup,
        "ms_per_step": round(step_s * 1e3, 4), "higher_is_better": True, "scaling": "replicas only",
        "vs_baseline": None, "dtype": "bf16", "data": "synthetic (seeded prompt + pixels, random-init weights)",
        "config": {"workload": f"decode: ViT-L/14-336 + Vicuna-7B, prompt 336 px + {args.text_len} tokens "
                               f"(L0={L0}), batch {B}, greedy, one HIP-graph replay per token",
                   "model": "llava-1.5-7b", "global_batch": B, "seq_len": L0, "parallelism": "dp1"},
        "prefill_ms": round(prefill_ms, 2), "weight_bytes": wbytes,
        "roofline": {"kernel": f"{gemm_kernel_name(B, 4096, 4096)[0]} / {gemm_kernel_name(B, 4096, 11008)[0]}: decode "
                             f"Linears Y = X W^T at M = {B}, {n_launch // 4} launches per step "
                               f"(eager step, HIP events per launch)",
                     "bound": "hbm", "achieved": round(achieved, 1), "peak": 8000.0, "unit": "GB/s",
                     "frac": round(achieved / 8000.0, 4), "traffic": measured_traffic("gemv_k<", f"decode-b{B}")[0],
                     "traffic_unit": "bytes/launch averaged over every GEMV dispatch of one profiled decode run "
                                     "(rocprofv3 FETCH_SIZE x2 + WRITE_SIZE; profiles/roofline_traffic.json)",
                     "algorithmic_bytes": round(g_bytes / max(n_launch, 1)),
                     "avg_ms": round(g_ms / max(n_launch, 1), 5)},
        "step_roofline": {"what": "LM + head weight bytes per token step / replayed step time (every kernel of the "
                                  "step, attention and norms included)",
                          "achieved": round(wbytes / step_s / 1e9, 1), "peak": 8000.0, "unit": "GB/s",
                          "frac": round(wbytes / step_s / 8e12, 4)},
    }
    emit(line, args)


def cpu_baseline(cfg, text_len: int, budget_s: float):
    """The oracle (CPU fp32 restatement of the reference path) timed on this host's cores:
    one Vicuna-7B decoder layer fwd+bwd, one CLIP-L/14 layer fwd, the lm_head fwd+bwd at B=1,
    L=text_len+575; extrapolated to a full sample (x32 LM layers, x23 ViT layers)."""
    import torch
    from oracle import cullavo_oracle as O

    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    torch.set_num_threads(threads)
    ocfg = O.config_7b()
    t, v = ocfg.text, ocfg.vision
    L = text_len + v.num_patches - 1
    g = torch.Generator().manual_seed(0)
    d, f = t.hidden_size, t.intermediate_size
    lp = "language_model.model.layers.0."
    W = {lp + f"self_attn.{n}_proj.weight": torch.randn(d, d, generator=g) * d ** -0.5 for n in "qkvo"}
    W[lp + "mlp.gate_proj.weight"] = torch.randn(f, d, generator=g) * d ** -0.5
    W[lp + "mlp.up_proj.weight"] = torch.randn(f, d, generator=g) * d ** -0.5
    W[lp + "mlp.down_proj.weight"] = torch.randn(d, f, generator=g) * f ** -0.5
    W[lp + "input_layernorm.weight"] = torch.ones(d)
    W[lp + "post_attention_layernorm.weight"] = torch.ones(d)
    for k in W:
        W[k].requires_grad_(True)
    h = torch.randn(1, L, d, generator=g, requires_grad=True)
    pos = torch.arange(L)[None]
    cos, sin = O.rope_cos_sin(pos, t.head_dim, t.rope_theta)
    allowed = O.causal_allowed(torch.ones(1, L, dtype=torch.long))

    def lm_layer():
        out = O.llama_layer(h, W, lp, t, cos, sin, allowed)
        out.sum().backward()

    vp = "vision_tower.vision_model.encoder.layers.0."
    dv = v.hidden_size
    VW = {}
    for n in ("q_proj", "k_proj", "v_proj", "out_proj"):
        VW[vp + f"self_attn.{n}.weight"] = torch.randn(dv, dv, generator=g) * dv ** -0.5
        VW[vp + f"self_attn.{n}.bias"] = torch.zeros(dv)
    VW[vp + "mlp.fc1.weight"] = torch.randn(v.intermediate_size, dv, generator=g) * dv ** -0.5
    VW[vp + "mlp.fc1.bias"] = torch.zeros(v.intermediate_size)
    VW[vp + "mlp.fc2.weight"] = torch.randn(dv, v.intermediate_size, generator=g) * v.intermediate_size ** -0.5
    VW[vp + "mlp.fc2.bias"] = torch.zeros(dv)
    for n in ("layer_norm1", "layer_norm2"):
        VW[vp + n + ".weight"] = torch.ones(dv)
        VW[vp + n + ".bias"] = torch.zeros(dv)
    vh = torch.randn(1, v.num_patches + 1, dv, generator=g)

    def vit_layer():
        with torch.no_grad():
            O.clip_layer(vh, VW, vp, v)

    Wh = (torch.randn(t.vocab_size, d, generator=g) * d ** -0.5).requires_grad_(True)
    x = torch.randn(1, L, d, generator=g, requires_grad=True)
    tgt = torch.randint(0, t.vocab_size, (L,), generator=g)

    def head():
        logits = torch.nn.functional.linear(x, Wh)
        torch.nn.functional.cross_entropy(logits.view(-1, t.vocab_size), tgt).backward()

    def timed(fn, reps):
        fn()  # warm
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        return (time.perf_counter() - t0) / reps

    t_start = time.perf_counter()
    t_lm = timed(lm_layer, 1)
    reps = max(1, int((budget_s * 0.6) / max(t_lm, 1e-3)))
    if reps > 1:
        t_lm = timed(lm_layer, min(reps, 5))
    t_vit = timed(vit_layer, 2)
    t_head = timed(head, 1)
    per_sample = t.num_hidden_layers * t_lm + O.needed_vision_layers(ocfg, -2) * t_vit + t_head
    return {"value": 1.0 / per_sample, "unit": "samples/s", "cores": threads, "kind": "port",
            "sample": (f"oracle fp32 on {threads} host threads: 1 Vicuna-7B decoder layer fwd+bwd "
                       f"({t_lm:.2f}s) + 1 CLIP-L/14 layer fwd ({t_vit:.3f}s) + lm_head fwd+bwd ({t_head:.2f}s) at "
                       f"B=1, L={L}, extrapolated x{t.num_hidden_layers} LM / x{O.needed_vision_layers(ocfg, -2)} "
                       f"ViT layers; {time.perf_counter() - t_start:.1f}s of CPU work")}


def layer_roofline(spans: dict, fl: dict, args, tc):
    """The north star's "fused causal-attention + MLP step": one decoder layer (RMSNorm, q|k|v,
    RoPE, causal flash attention, o_proj + residual, RMSNorm, gate|up, SwiGLU, down + residual;
    reference cullavo/arch_cullavo.py:638-647 -> transformers LlamaDecoderLayer, FA2 per
    load_cullavo.py:72) forward + backward, timed by HIP events on the compute stream around every
    LlamaLayerFn forward and backward of the timed steps. Algorithmic FLOPs per layer and sample:
    GEMM fwd 2·L·(4d² + 3dF) (x3 with dX + dW when the weights train, x2 when frozen) + causal
    attention 2·L²·d (x3.5: forward + the FA2 backward's 2.5)."""
    fwd, bwd = spans.get("fwd", []), spans.get("bwd", [])
    if not fwd or not bwd:
        return None
    n_f, n_b = len(fwd), len(bwd)
    ms_f, ms_b = sum(fwd) / n_f, sum(bwd) / n_b
    gemm_mult = 3.0 if args.trainable == "full" else 2.0
    per_sample = gemm_mult * fl["lm_gemm_layer"] + 3.5 * fl["lm_attn_layer"]
    if args.trainable == "lora":  # the layer's own adapters (r = 64 on q, k, v, o, gate, up, down): fwd x3
        from cullavo_amd.perf import _lora_fwd
        d, f = tc.hidden_size, tc.intermediate_size
        per_sample += 3 * _lora_fwd(args.text_len + 575, 64, [(d, d)] * 4 + [(f, d)] * 2 + [(d, f)])
    flops = per_sample * args.batch
    tf = flops / ((ms_f + ms_b) * 1e-3) / 1e12
    return {"what": "one decoder layer fwd+bwd (attention + MLP + norms/RoPE/SwiGLU), HIP events per layer",
            "fwd_ms": round(ms_f, 4), "bwd_ms": round(ms_b, 4), "layers_timed": min(n_f, n_b),
            "gflop_per_layer": round(flops / 1e9, 1), "achieved": round(tf, 1), "peak": PEAK_BF16_TFLOPS,
            "unit": "TFLOP/s", "frac": round(tf / PEAK_BF16_TFLOPS, 4)}


def gemm_kernel_name(M, N, K, al=0, bl=0, lora=False):
    """rocprof name (template arguments as rocprofv3 prints them) + workgroup count of the
    kernel cullavo_gemm picks for a bf16-output problem (cullavo_gemm_plan); lora: the
    instantiation with the fused LoRA up-projection (gemm256_k<..., LORA = true>).
    gemm256_k<AL, BL, CT, BM, BN, LDR, LORA, SWG, EPI>: EPI 1 / 2 the direct (register) epilogue of
    plain / bias-residual products, 0 the LDS-staged one. The problem key carries no epilogue, so a
    forward / dX family whose products differ in it is named with EPI "*" (either of 1, 2; the PMC
    tools match "*" as a wildcard); the SwiGLU-backward dX (SWG = true) is a family of its own only
    by rocprof name. "<MODE>": every epilogue-mode instantiation of the persistent kernel."""
    import ctypes
    from cullavo_amd import _lib
    g = ctypes.c_int64(0)
    tile = _lib.lib().cullavo_gemm_plan(M, N, K, al, bl, ctypes.byref(g))
    ep = os.environ.get("CULLAVO_GEMM_EPILOGUE")
    ep = 1 if ep is None else int(ep)
    direct = bool(ep & 1) and not ep & 128
    lf = "true" if lora else "false"

    def g256(bm):
        if lora or not direct or (bm == 192):
            e = "0"
        elif (al, bl) == (1, 1):
            e = "1"  # weight gradients: always plain
        else:
            e = "*"
        return f"gemm256_k<{al}, {bl}, 1, {bm}, 256, 1, {lf}, false, {e}>"
    names = {0: f"gemm_k<{al}, {bl}, 1, 0>", 2: g256(256), 3: g256(192),
             9: f"gemm256_k<{al}, {bl}, 1, 256, 256, 1, false, false, 0> split-K + splitk_reduce_k<1>",
             10: g256(288), 14: "gemv_k<1, 0, 1, 0, 4>" if K >= 8192 else ("gemv_k<1, 0, 1, 0, 4, 16>" if N > 16384 else "gemv_k<1, 0, 1, 0, 8>")}
    def persistent(t):
        # the persistent forward kernels (gemm.hip launch256p / launch288pd), one instantiation per
        # epilogue mode (0 plain, 1 bias/residual, 2 activation); one block per CU
        if t in (2, 10) and (al, bl) == (0, 0) and not lora and ep & 1 and not ep & 32 and (
                t == 2 or (direct and (ep & 256 or K < 2048 or N <= 2048))):
            return f"gemm256pd_k<*, {256 if t == 2 else 288}>" if direct else "gemm256p_k<MODE>"
        return None
    if tile >= 100:  # the M-tail split: the head rows' kernel (+ a thin split-K product for the rest)
        base = persistent(tile - 100) or names.get(tile - 100, f"tile{tile - 100}<{al}, {bl}>")
        return base + " M-split", int(g.value)
    if persistent(tile):
        return persistent(tile), min(int(g.value), 256)  # 256 CUs on MI355X
    return names.get(tile, f"tile{tile}<{al}, {bl}>"), int(g.value)


GEMM_ROLE = {(0, 0): "forward Y = X W^T", (0, 1): "input gradient dX = dY W", (1, 1): "weight gradient dW = dY^T X",
             (1, 0): "transposed-A"}


def gemm_families(launches):
    """Group traced GEMM launches by kernel instantiation: launches, FLOPs, ms, algorithmic HBM
    bytes (A + B read once, C written; + C read when accumulating is not traced: beta = 0 in the
    step) -> achieved TFLOP/s per kernel, sorted by GPU time."""
    fam = {}
    for key, ms in launches:
        M, N, K, al, bl = key[:5]
        lora = len(key) > 5
        name, _ = gemm_kernel_name(M, N, K, al, bl, lora)
        role = GEMM_ROLE[(al, bl)] + (" + fused LoRA up-projection" if lora else "")
        f = fam.setdefault(name, {"kernel": name, "role": role, "layouts": (al, bl), "launches": 0, "ms": 0.0,
                                  "flops": 0.0, "bytes": 0.0, "shapes": set()})
        f["launches"] += 1
        f["ms"] += ms
        f["flops"] += 2.0 * M * N * K
        f["bytes"] += 2.0 * (M * K + N * K + M * N)
        f["shapes"].add((M, N, K))
    out = sorted(fam.values(), key=lambda f: -f["ms"])
    for f in out:
        f["achieved_tflops"] = f["flops"] / (f["ms"] * 1e-3) / 1e12
        f["shapes"] = sorted(f["shapes"])
    return out


def gemm_shapes(launches, steps, top=12):
    """per-shape GEMM time of the timed steps (the largest first): where each family's time goes"""
    sh = {}
    for key, ms in launches:
        r = sh.setdefault(tuple(key), [0, 0.0])
        r[0] += 1
        r[1] += ms
    out = []
    for key, (n, ms) in sorted(sh.items(), key=lambda kv: -kv[1][1])[:top]:
        M, N, K, al, bl = key[:5]
        name, grid = gemm_kernel_name(M, N, K, al, bl, len(key) > 5)
        out.append({"shape": f"{M}x{N}x{K}", "layouts": [al, bl], "kernel": name, "grid": grid,
                    "launches_per_step": round(n / steps, 2), "ms_per_step": round(ms / steps, 3),
                    "tflops": round(2.0 * M * N * K * n / (ms * 1e-3) / 1e12, 1)})
    return out


def measured_traffic(kname, workload):
    """HBM bytes per launch of the roofline kernel (average over its launches in one profiled
    step) and its MFMA busy fraction, from the committed PMC passes of THIS workload (records
    keyed by workload and kernel; None when no pass was taken on that pair)."""
    path = os.path.join(REPO, "profiles", "roofline_traffic.json")
    try:
        recs = json.load(open(path))
    except (OSError, ValueError):
        return None, None
    for rec in recs.get("records", []):
        if rec.get("kernel") == kname and rec.get("workload") == workload:
            return rec.get("bytes_per_launch"), rec.get("mfma_busy_frac")
    return None, None


def gemm_ceiling(fam, iters=10):
    """hipBLASLt (torch.matmul, same layouts) against this kernel on the family's largest shape,
    same process, random bf16 operands: the measured library ceiling BASELINE.md §2 asks for"""
    import torch

    from cullavo_amd import ops
    (M, N, K) = max(fam["shapes"], key=lambda s: s[0] * s[1] * s[2])
    al, bl = fam["layouts"]
    g = torch.Generator(device="cuda").manual_seed(0)
    A = torch.randn((K, M) if al else (M, K), device="cuda", generator=g).bfloat16()
    B = torch.randn((K, N) if bl else (N, K), device="cuda", generator=g).bfloat16()
    C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    Am = A.t() if al else A
    Bm = B if bl else B.t()  # [K, N]

    def ours():  # gemm_ex with split-K allowed: the plan the step's Linears run (cullavo_gemm_plan)
        ops.gemm_ex(al, bl, M, N, K, A, A.stride(0), B, B.stride(0), C, N)

    def lib():
        torch.matmul(Am, Bm, out=C)

    res = {}
    for name, fn in (("ours", ours), ("hipblaslt", lib), ("ours2", ours), ("hipblaslt2", lib)):
        fn()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        e.synchronize()
        res[name] = 2.0 * M * N * K / (s.elapsed_time(e) / iters * 1e-3) / 1e12
    del A, B, C
    return {"shape": f"{M}x{N}x{K}", "layouts": [al, bl],
            "this_kernel_tflops": round(max(res["ours"], res["ours2"]), 1),
            "hipblaslt_tflops": round(max(res["hipblaslt"], res["hipblaslt2"]), 1)}


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_cmd(n: int, argv: list[str], port: int) -> list[str]:
    """the child command that forms an N-rank world on this node (one process per GPU)"""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def self_launch(n: int, argv: list[str]) -> int:
    """Start N ranks of this script under torch.distributed.run (this process never touches the
    GPU), forward rank 0's JSON line to stdout and everything else to stderr; the launcher's exit
    code is returned (non-zero when any rank failed)."""
    import subprocess
    cmd = launch_cmd(n, argv, free_port())
    print(f"bench.py: --gpus {n} without a launcher env; starting {n} ranks: {' '.join(cmd)}", file=sys.stderr,
          flush=True)
    env = dict(os.environ)
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, env=env, text=True)
    json_lines = 0
    for line in p.stdout:  # rank 0 prints the one JSON line; anything else goes to stderr
        if line.startswith("{"):
            json_lines += 1
            sys.stdout.write(line)
            sys.stdout.flush()
        else:
            sys.stderr.write(line)
    rc = p.wait()
    if rc == 0 and json_lines != 1:
        print(f"bench.py: expected one JSON line from rank 0, got {json_lines}", file=sys.stderr)
        return 4
    return rc


def launch_probe(args, world: int) -> None:
    """--launch-probe: the N>1 launch path without a GPU (world formation, rank env, max-over-ranks
    reduction, one line on rank 0)."""
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo")
    rank = dist.get_rank()
    if os.environ.get("CULLAVO_PROBE_FAIL_RANK") == str(rank):  # tests: a rank that dies
        sys.exit(1)
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({"metric": "launch-probe", "n_gpus": dist.get_world_size(), "gpus_arg": args.gpus,
                          "max_over_ranks": t.item(), "local_ranks": world}), flush=True)
    dist.destroy_process_group()


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse(argv)
    subs = None
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(self_launch(args.gpus, argv))  # before anything touches the GPU
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher formed WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(3)
    if args.launch_probe:
        return launch_probe(args, world)
    names = [n for n in args.sub_workloads.split(",") if n]
    if world == 1 and not args.no_sub and args.workload == "step" and names:
        subs = run_sub_workloads(args, names)  # before this process touches the GPU
    if args.workload == "vit":
        if args.batch == 8:
            args.batch = 64  # BASELINE config 2
        return vit_main(args)
    if args.workload == "decode":
        return decode_main(args)
    import torch
    import torch.distributed as dist

    from cullavo_amd import ops
    from cullavo_amd.trainer import CuLLaVO_Trainer

    opt = {"MODEL": {"CONFIG": args.config}, "LLM": {"TRAINABLE": args.trainable},
           "DATA": {"BATCH_SIZE_PER_GPU": args.batch, "TEXT_LEN": args.text_len, "IMAGE_COL": 35,
                    "STEPS": args.warmup + args.steps},
           "BUCKET_MB": args.bucket_mb, "OPTIMIZER": {"OVERLAP": args.overlap and not args.no_overlap}}
    tr = CuLLaVO_Trainer(opt)
    rank = tr.accel.process_index
    tr.init_train()
    cm = tr.model.cullavo_model
    batch = next(iter(tr.train_dataloaders))  # resident in HBM before timing

    prio_stream = None
    if args.high_prio:
        prio_stream = torch.cuda.Stream(priority=-1)
        prio_stream.wait_stream(torch.cuda.current_stream())

    def step():
        if prio_stream is not None:
            with torch.cuda.stream(prio_stream), tr.accel.accumulate(tr.model):
                info, _, _ = tr.train_step(batch)
            return info["loss_llm"]
        with tr.accel.accumulate(tr.model):
            info, _, _ = tr.train_step(batch)
        return info["loss_llm"]

    for _ in range(args.warmup):
        loss = step()
    torch.cuda.synchronize()

    # the headline: K steps timed with no instrumentation (no per-launch or per-layer events)
    cfg = cm.config
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0

    # then a separate traced pass for the roofline: every GEMM launch bracketed by HIP events on the
    # stream it runs on (the roofline object reports the kernel with the largest share of GPU time),
    # HIP events around every decoder layer's forward and backward, the exchange's exposure events
    traced_steps = max(1, min(args.steps, 3))
    ops.trace_gemm("all")
    from cullavo_amd import functions as F
    F.trace_layers(True)
    reducer = tr.accel.reducer
    if reducer is not None:
        reducer.measure = True
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(traced_steps):
        loss = step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    traced_elapsed = time.perf_counter() - t1
    launches = ops.trace_launches()  # (stops the tracing)
    spans = F.layer_spans()
    fams = gemm_families(launches)
    exchange = None
    if world > 1:
        t = torch.tensor([elapsed, traced_elapsed], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, traced_elapsed = t[0].item(), t[1].item()
        st = reducer.exposure_stats() if reducer is not None else None
        # the exposed-exchange figure is the slowest rank's too
        e = torch.tensor([st["exposed_ms"] if st else -1.0, st["host_rendezvous_ms"] if st else -1.0],
                         device="cuda")
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        exchange = {"backend": dist.get_backend(), "rccl_world_size": dist.get_world_size()
                    if dist.get_backend() == "nccl" else None, "world_size": dist.get_world_size(),
                    "allreduce_bytes_per_step": reducer.bytes_per_step if reducer is not None else 0,
                    "buckets": len(reducer.buckets) if reducer is not None else 0,
                    "exposed_exchange_ms": round(e[0].item(), 3),
                    "host_rendezvous_ms": round(e[1].item(), 3),
                    "exposed_def": "max over ranks of the mean over timed steps: compute stream's backward end "
                                   "-> all buckets reduced (clip + AdamW may start), HIP events"}
    loss_v = float(loss)

    from cullavo_amd.perf import flops_per_sample

    fl = flops_per_sample(cfg, args.text_len, args.trainable)
    samples = world * args.batch * args.steps
    value = samples / elapsed
    step_tflops = fl["train"] * world * args.batch / (elapsed / args.steps) / 1e12
    top = fams[0]
    kname = top["kernel"]
    traffic, mfma_busy = measured_traffic(kname, workload_key(args))
    achieved = top["achieved_tflops"]
    n_launch = top["launches"]
    if rank == 0:
        line = {
            "metric": "train-step samples/sec (336px img + 512-tok prompt, 7B LM)" if "13b" not in args.config
                      else "train-step samples/sec (336px img + 1024-tok prompt, 13B LM)",
            "value": round(value, 4),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (seeded ids/pixels/labels in HBM, random-init weights)",
            "config": {"workload": f"{'config 5: ViT-L/14-336 + Llama-2-13B' if '13b' in args.config else 'config 3: ViT-L/14-336 + Vicuna-7B'}, "
                                   f"seq 576+{args.text_len - 1} (L={args.text_len + 575}), "
                                   f"bs={args.batch}/GPU, bf16, {args.trainable} fine-tune "
                                   f"({'LoRA r=64 on the LM + ViT layers 12-22' if args.trainable == 'lora' else 'vision frozen'}), AdamW",
                       "model": args.config, "global_batch": world * args.batch,
                       "seq_len": args.text_len + cfg.vision_config.num_patches - 1,
                       "parallelism": f"dp{world}", "trainable": args.trainable},
            "model_tflops_per_gpu": round(step_tflops / world, 2),
            "mfu": round(step_tflops / world / PEAK_BF16_TFLOPS, 4),
            "loss": round(loss_v, 5),
            "roofline": {
                "kernel": f"{kname}: {top['role']}, {len(top['shapes'])} shapes "
                          f"{['x'.join(map(str, sh)) for sh in top['shapes']]} (M x N x K), "
                          f"{n_launch // traced_steps} launches/step, {100 * top['ms'] / (traced_elapsed * 1e3):.1f} % of "
                          f"the traced steps",
                "bound": "mfma",
                "achieved": round(achieved, 2),
                "peak": PEAK_BF16_TFLOPS,
                "unit": "TFLOP/s",
                "frac": round(achieved / PEAK_BF16_TFLOPS, 4),
                "traffic": traffic,
                "traffic_unit": "bytes/launch averaged over the kernel's launches in one step of this workload (HBM, "
                                "rocprofv3 FETCH_SIZE x2 + WRITE_SIZE; profiles/roofline_traffic.json)" if traffic else None,
                "algorithmic_bytes": round(top["bytes"] / n_launch),
                "mfma_busy": mfma_busy,
                "avg_ms": round(top["ms"] / n_launch, 4),
                "launches_timed": n_launch,
                "flops_per_launch": top["flops"] / n_launch,
            },
            "gemm_kernels": [{"kernel": f["kernel"], "role": f["role"],
                              "share_of_step": round(f["ms"] / (traced_elapsed * 1e3), 4),
                              "achieved_tflops": round(f["achieved_tflops"], 1),
                              "frac": round(f["achieved_tflops"] / PEAK_BF16_TFLOPS, 4)} for f in fams[:6]],
            "gemm_shapes": gemm_shapes(launches, traced_steps),
            "traced_pass": {"steps": traced_steps, "ms_per_step": round(traced_elapsed / traced_steps * 1e3, 3),
                            "what": "roofline, gemm_kernels, gemm_shapes and layer_roofline come from this separate "
                                    "pass with HIP events around every GEMM launch and decoder layer; value and "
                                    "ms_per_step from the untraced timed loop"},
        }
        if world == 1:
            # every family's largest shape in isolation against hipBLASLt, same process: the
            # library ceiling per family, and the isolated rate beside the in-step one (in the
            # step, launches can share the GPU with the optimizer's side-stream update)
            for f, entry in zip(fams[:6], line["gemm_kernels"]):
                entry["library_ceiling"] = gemm_ceiling(f)
            line["roofline"]["library_ceiling"] = line["gemm_kernels"][0]["library_ceiling"]
        lr = layer_roofline(spans, fl, args, cfg.text_config)
        if lr is not None:
            line["layer_roofline"] = lr
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(cfg, args.text_len, args.cpu_seconds)
        if subs is not None:
            line["workloads"] = subs
        if exchange is not None:
            line["exchange"] = exchange
        emit(line, args)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
