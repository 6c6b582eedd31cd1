"""The C-ABI library loads on a CPU-only host and exports every symbol include/*.h declares;
host-side argument validation errors come back through cullavo_last_error() (no GPU call)."""
import ctypes
import os
import re

import pytest

import cullavo_amd
from cullavo_amd import _lib


def test_header_parses_and_library_exports_every_symbol():
    decls = _lib.declarations()
    assert len(decls) >= 30
    lib = _lib.lib()
    for name in decls:
        assert hasattr(lib, name), name
    assert _lib.abi_version() >= 2 and lib.cullavo_abi_version() == _lib.abi_version()


def test_nm_exports_match_header():
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (cullavo_\w+)", out))
    assert set(_lib.declarations()) <= exported


def test_validation_errors_surface_without_gpu():
    # K not a multiple of 8 is rejected on the host before any launch
    with pytest.raises(ValueError, match="multiple of 8"):
        _lib.call("gemm", 0, 0, 16, 16, 12, None, 12, None, 12, None, 16, 1, 1.0, None, 0, None, None, 0, 0.0, None)
    with pytest.raises(ValueError, match="head_dim"):
        _lib.call("rope", None, 128, None, 128, None, 4, 1, 1, 12, 10000.0, 0, 1, None)
    with pytest.raises(Exception, match="head_dim must be 16, 32, 64 or 128"):
        _lib.call("attn_fwd", None, 96, None, 96, None, 96, None, 96, None, 1, 1, 4, 4, 96, 1.0, 1, None, 1, None)


def test_workspace_queries():
    lib = _lib.lib()
    assert lib.cullavo_norm_bwd_workspace(8704, 4096) == 2 * 1024 * 4096 * 4
    assert lib.cullavo_colsum_workspace(100, 4096) == 32 * 4096 * 4


def test_product_path_refuses_cpu_tensors():
    import torch
    from cullavo_amd import ops
    with pytest.raises(RuntimeError, match="GPU only"):
        ops.rmsnorm_fwd(torch.zeros(4, 8), torch.ones(8), 1e-5)
