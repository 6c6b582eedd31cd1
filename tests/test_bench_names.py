"""bench.gemm_kernel_name (the rocprof name the bench files a GEMM family under, from the library's
plan) and tools/pmc_family.py's name pattern agree with the instantiations the library launches, so
a PMC record taken on the GPU box is found again by the bench line. Host-only: cullavo_gemm_plan is
host code (no GPU needed)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import bench  # noqa: E402
import pmc_family  # noqa: E402

T = 8704


@pytest.mark.parametrize("shape,name", [
    ((T, 22016, 4096, 0, 0), "gemm256_k<0, 0, 1, 288, 256, 1, false, false, *>"),       # gate|up forward
    ((T, 4096, 22016, 0, 1), "gemm256_k<0, 1, 1, 288, 256, 1, false, false, *>"),       # gate|up dX
    ((22016, 4096, T, 1, 1), "gemm256_k<1, 1, 1, 256, 256, 1, false, false, 1> M-split"),  # round split
    ((12288, 4096, T, 1, 1), "gemm256_k<1, 1, 1, 256, 256, 1, false, false, 1>"),       # q|k|v dW
    ((36928, 4096, 1024, 0, 0), "gemm256pd_k<*, 288> M-split"),                          # ViT fc1
    ((36928, 3072, 1024, 0, 0), "gemm256pd_k<*, 256>"),                                  # ViT q|k|v
    ((36928, 1024, 4096, 0, 0), "gemm256pd_k<*, 288> M-split"),                          # ViT fc2
])
def test_gemm_kernel_names_of_the_step_shapes(shape, name, monkeypatch):
    monkeypatch.delenv("CULLAVO_GEMM_EPILOGUE", raising=False)
    M, N, K, al, bl = shape
    got, grid = bench.gemm_kernel_name(M, N, K, al, bl)
    assert got == name
    assert grid > 0


@pytest.mark.parametrize("family,rocprof,match", [
    ("gemm256_k<0, 0, 1, 288, 256, 1, false, false, *>",
     "void (anonymous namespace)::gemm256_k<0, 0, 1, 288, 256, 1, false, false, 2>(cvgemm::GemmArgs)", True),
    ("gemm256_k<0, 0, 1, 288, 256, 1, false, false, *>",
     "void (anonymous namespace)::gemm256_k<0, 1, 1, 288, 256, 1, false, false, 1>(cvgemm::GemmArgs)", False),
    ("gemm256pd_k<*, 288> M-split", "void (anonymous namespace)::gemm256pd_k<2, 288>(cvgemm::GemmArgs)", True),
    ("gemm256pd_k<*, 288> M-split", "void (anonymous namespace)::gemm256pd_k<2, 256>(cvgemm::GemmArgs)", False),
    ("gemm256p_k<MODE>", "void (anonymous namespace)::gemm256p_k<1>(cvgemm::GemmArgs)", True),
])
def test_pmc_family_pattern(family, rocprof, match):
    assert bool(pmc_family.name_pattern(family).search(rocprof)) == match
