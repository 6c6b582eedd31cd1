"""bench.py's N > 1 launch path on the CPU (VERDICT r03 "Missing #1"): `python bench.py --gpus N`
without a launcher env must start its own N ranks (torch.distributed.run, 127.0.0.1), forward
rank 0's single JSON line and fail non-zero when the formed world differs from --gpus.
The reference launches its ranks itself too (/root/reference/run:59-71)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")
LAUNCH_ENV = ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
              "GROUP_RANK", "ROLE_RANK", "TORCHELASTIC_RUN_ID")


def _env(**extra):
    env = {k: v for k, v in os.environ.items() if k not in LAUNCH_ENV}
    env.update(extra)
    return env


@pytest.mark.parametrize("n", [2, 4])
def test_self_launch_forms_world_and_forwards_one_line(n):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--launch-probe"], capture_output=True,
                       text=True, timeout=240, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == n and rec["gpus_arg"] == n
    assert rec["max_over_ranks"] == float(n)  # every rank took part in the reduction
    assert "starting" in r.stderr and "torch.distributed.run" in r.stderr


def test_world_mismatch_is_an_error():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-probe"], capture_output=True, text=True,
                       timeout=120, env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"))
    assert r.returncode == 3, (r.returncode, r.stderr)
    assert "WORLD_SIZE=1" in r.stderr


def test_launch_cmd_shape():
    sys.path.insert(0, REPO)
    import bench
    cmd = bench.launch_cmd(8, ["--gpus", "8", "--steps", "5"], 29999)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--master-addr=127.0.0.1" in cmd and "--nnodes=1" in cmd
    assert cmd[-3:] == ["--gpus", "8", "--steps", "5"][-3:] and bench.__file__.rstrip("c") in cmd


def test_failing_rank_propagates_exit_code():
    """a rank that dies makes the launcher (and bench.py) exit non-zero, with no JSON forwarded"""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-probe"], capture_output=True, text=True,
                       timeout=240, env=_env(CULLAVO_PROBE_FAIL_RANK="1"))
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
