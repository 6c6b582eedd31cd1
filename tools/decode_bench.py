"""KV-cache generation throughput on the 7B config: prefill of the
config-3 prompt (336 px image + 512 text tokens -> 1088 merged rows) and greedy decode steps.
Prints one JSON line: prefill ms, decode ms/token, tokens/s (all sequences), and the weight
stream rate (bf16 LM + head bytes read per decode step / step time) against HBM's ~8 TB/s.

  python tools/decode_bench.py [--batch 1] [--new 64] [--text-len 513]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--new", type=int, default=64)
    ap.add_argument("--text-len", type=int, default=513)
    a = ap.parse_args()
    from cullavo_amd.arch_cullavo import CuLLaVOModel
    from cullavo_amd.config import llava_1_5_7b
    from cullavo_amd.data import synthetic_batch
    cfg = llava_1_5_7b()
    m = CuLLaVOModel(cfg, device="cuda", trainable="none", init="random", seed=0)
    m.eval()
    sb = synthetic_batch(cfg, a.batch, a.text_len, 35, seed=1234, device="cuda")
    ids, mask, pix = sb["input_ids"], sb["attention_mask"], sb["pixel_values"]
    t = cfg.text_config
    wbytes = 2 * (t.num_hidden_layers * (4 * t.hidden_size ** 2 + 3 * t.hidden_size * t.intermediate_size)
                  + t.vocab_size * t.hidden_size)
    with torch.no_grad():
        m.generate(input_ids=ids, pixel_values=pix, attention_mask=mask, max_new_tokens=4)  # warm-up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = m(input_ids=ids, pixel_values=pix, attention_mask=mask, use_cache=True)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        cache = out.past_key_values
        tok = out.logits[:, -1].argmax(-1)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        for _ in range(a.new):
            out = m(input_ids=tok[:, None], past_key_values=cache, use_cache=True)
            tok = out.logits[:, -1].argmax(-1)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
    step = (t3 - t2) / a.new
    print(json.dumps({"metric": "7B KV-cache decode", "batch": a.batch, "prompt_rows": cache.get_seq_length() - a.new,
                      "prefill_ms": round((t1 - t0) * 1e3, 2), "decode_ms_per_step": round(step * 1e3, 3),
                      "tokens_per_s": round(a.batch / step, 2), "weight_stream_TBps": round(wbytes / step / 1e12, 3),
                      "hbm_peak_TBps": 8.0}))


if __name__ == "__main__":
    main()
