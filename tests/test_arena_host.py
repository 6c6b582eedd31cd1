"""Host-side arena bookkeeping (CPU): the staleness key that decides when the K-major weight
copies of the decoder dX GEMMs are re-made, and the sumsq workspace contract."""
import torch

from cullavo_amd import ops
from cullavo_amd.arena import ParamArena


def _arena():
    return ParamArena("t", [("a.weight", (8, 16)), ("b.weight", (16, 8))], device="cpu", trainable=False)


def test_state_changes_on_torch_inplace_writes_through_views():
    ar = _arena()
    s0 = ar._state()
    with torch.no_grad():
        ar.params["a.weight"].copy_(torch.ones(8, 16))
    s1 = ar._state()
    assert s1 != s0
    ar.view("b.weight", (16, 8)).mul_(2.0)
    assert ar._state() != s1


def test_state_changes_on_kernel_writes_reported_by_note_written():
    ar = _arena()
    s0 = ar._state()
    ar.note_written()  # what FusedAdamW.step and the RCCL broadcast call after raw-pointer writes
    assert ar._state() != s0


def test_sumsq_workspace_size_matches_header():
    src = open(ops.__file__.replace("ops.py", "../include/cullavo_capi.h")).read()
    assert f"#define CULLAVO_SUMSQ_PARTIALS {ops.SUMSQ_PARTIALS}" in src
