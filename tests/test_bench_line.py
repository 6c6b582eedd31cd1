"""bench.py's final stdout line must stay compact (VERDICT r04 "Missing #1": the ~20.7 KB line of
round 4 overflowed the driver's 8 KB tail and left the round unmeasured). The full record goes to
the sidecar file; the line keeps the headline, roofline, layer_roofline, cpu_baseline, exchange and
one summary per sub-workload. CPU only: canned records, no GPU."""
import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

CANNED = os.path.join(REPO, "profiles", "r04", "final", "bench_closing.json")


def _full():
    """round 4's closing full record (the line that overflowed), plus a layer_roofline"""
    with open(CANNED) as f:
        rec = json.loads([ln for ln in f.read().splitlines() if ln.startswith("{")][-1])
    rec["layer_roofline"] = {"what": "x" * 80, "fwd_ms": 3.2, "bwd_ms": 6.6, "layers_timed": 320,
                             "gflop_per_layer": 10842.0, "achieved": 1106.0, "peak": 2500.0, "unit": "TFLOP/s",
                             "frac": 0.4424}
    return rec


REQUIRED = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "dtype", "config", "mfu",
            "roofline", "cpu_baseline", "layer_roofline")


def test_canned_round4_record_is_over_the_limit_and_the_line_is_not():
    full = _full()
    assert len(json.dumps(full)) > 16000  # the record that broke round 4's measurement
    line = bench.compact_line(full)
    s = json.dumps(line)
    assert len(s.encode()) <= bench.LINE_LIMIT, len(s)
    for k in REQUIRED:
        assert k in line, k
    roof = line["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "algorithmic_bytes", "mfma_busy",
              "library_ceiling"):
        assert k in roof, k
    assert roof["frac"] == full["roofline"]["frac"] and line["value"] == full["value"]
    assert set(line["workloads"]) == set(full["workloads"])
    for w in line["workloads"].values():
        assert "value" in w and "roofline_frac" in w
    assert "gemm_shapes" not in s and "gemm_kernels" not in s


def test_worst_case_line_with_exchange_and_failed_workloads_fits():
    full = _full()
    full["exchange"] = {"backend": "nccl", "rccl_world_size": 8, "world_size": 8,
                        "allreduce_bytes_per_step": 13520000000, "buckets": 46, "exposed_exchange_ms": 12.345,
                        "host_rendezvous_ms": 0.5, "exposed_def": "y" * 200}
    full["workloads"] = {n: {"error": "Traceback " + "z" * 2000} for n in bench.SUB_WORKLOADS}
    full["cpu_baseline"]["sample"] = "s" * 3000
    full["config"]["workload"] = "w" * 1000
    line = bench.compact_line(full)
    assert len(json.dumps(line).encode()) <= bench.LINE_LIMIT
    assert "exchange" in line and "cpu_baseline" in line and "roofline" in line


def test_emit_writes_sidecar_and_prints_one_compact_last_line(tmp_path, capsys):
    full = _full()

    class A:
        detail_out = str(tmp_path / "detail.json")

    bench.emit(full, A())
    out = capsys.readouterr().out.strip().splitlines()
    assert len(out) == 1 and out[0].startswith("{")
    line = json.loads(out[0])
    assert len(out[0].encode()) <= bench.LINE_LIMIT
    side = json.load(open(A.detail_out))
    assert side["gemm_shapes"] == full["gemm_shapes"] and side["workloads"] == full["workloads"]
    assert line["detail"].endswith("detail.json")


def test_layer_roofline_flops():
    from cullavo_amd.config import llava_1_5_7b
    from cullavo_amd.perf import flops_per_sample

    cfg = llava_1_5_7b()
    fl = flops_per_sample(cfg, 513, "full")
    args = type("A", (), {"trainable": "full", "batch": 8, "text_len": 513})()
    spans = {"fwd": [3.0] * 64, "bwd": [6.0] * 64}
    lr = bench.layer_roofline(spans, fl, args, cfg.text_config)
    # 3 x 440.4 GFLOP (GEMMs fwd + dX + dW) + 3.5 x 9.71 (causal attention) per sample, x 8 samples
    assert lr["gflop_per_layer"] == pytest.approx(8 * (3 * 440.37 + 3.5 * 9.70), rel=2e-3)
    assert lr["achieved"] == pytest.approx(lr["gflop_per_layer"] / 9.0, rel=1e-3)
    assert lr["frac"] == pytest.approx(lr["achieved"] / 2500.0, rel=1e-3)
    assert bench.layer_roofline({"fwd": [], "bwd": []}, fl, args, cfg.text_config) is None
