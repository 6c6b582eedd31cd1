"""ctypes binding of libcullavo_hip.so.

The argument types are generated from ``include/cullavo_capi.h`` itself, so the Python side
cannot drift from the C-ABI: every ``int cullavo_*(...)`` / ``size_t cullavo_*(...)``
declaration in the header becomes a bound function with matching ctypes argtypes.
There is no CPU fallback: a missing or unloadable library raises.
"""
from __future__ import annotations

import ctypes
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libcullavo_hip.so")
# A/B of two builds of the library in one process tree (tools): CULLAVO_LIB_AB names another build of
# the same ABI; unset, the in-tree library is the only one ever loaded. The override is announced on
# stderr (a stray variable must not silently change the kernels a run uses), and lib() still checks the
# build's ABI against the header
if os.environ.get("CULLAVO_LIB_AB"):
    LIB_PATH = os.environ["CULLAVO_LIB_AB"]
    import sys as _sys
    print(f"cullavo_amd: CULLAVO_LIB_AB is set, loading {LIB_PATH} instead of the in-tree library",
          file=_sys.stderr, flush=True)
HEADER = os.path.join(os.path.dirname(_HERE), "include", "cullavo_capi.h")

_CTYPE = {
    "int": ctypes.c_int,
    "int64_t": ctypes.c_int64,
    "float": ctypes.c_float,
    "double": ctypes.c_double,
    "size_t": ctypes.c_size_t,
    "uint64_t": ctypes.c_uint64,
}

DT_F32 = 0
DT_BF16 = 1
ACT_NONE = 0
ACT_GELU = 1
ACT_QUICK_GELU = 2
ACT_SWIGLU_BWD = 3  # down-proj dX GEMM epilogue writing dgate | dup (CULLAVO_ACT_SWIGLU_BWD)

_lib = None
_decls: dict[str, tuple[str, list[tuple[str, str]]]] | None = None


def parse_header(path: str = HEADER) -> dict[str, tuple[str, list[tuple[str, str]]]]:
    """Return {name: (return type, [(c type, arg name), ...])} for every cullavo_* function."""
    txt = open(path).read()
    txt = re.sub(r"/\*.*?\*/", " ", txt, flags=re.S)
    out = {}
    for m in re.finditer(r"(int|size_t|const char\s*\*)\s+(cullavo_\w+)\s*\(([^)]*)\)\s*;", txt):
        ret, name, args = m.group(1), m.group(2), m.group(3).strip()
        params = []
        if args and args != "void":
            for a in args.split(","):
                a = " ".join(a.split())
                am = re.match(r"(.*?)(\w+)$", a)
                ctype, pname = am.group(1).strip(), am.group(2)
                params.append((ctype, pname))
        out[name] = (" ".join(ret.split()), params)
    return out


def _argtype(ctype: str):
    if "*" in ctype:
        return ctypes.c_void_p
    base = ctype.replace("const", "").strip()
    return _CTYPE[base]


def declarations():
    global _decls
    if _decls is None:
        _decls = parse_header()
    return _decls


def abi_version(path: str = HEADER) -> int:
    """CULLAVO_ABI_VERSION of the header the binding is generated from."""
    return int(re.search(r"#define CULLAVO_ABI_VERSION (\d+)", open(path).read()).group(1))


def lib():
    """Load and bind the HIP library (raises if it is absent: there is no CPU fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} is missing: build the HIP extension first "
                "(python -c 'import __graft_entry__ as g; g.build()')"
            )
        L = ctypes.CDLL(LIB_PATH)
        L.cullavo_abi_version.restype = ctypes.c_int
        if L.cullavo_abi_version() != abi_version():
            raise RuntimeError(f"{LIB_PATH} was built for ABI {L.cullavo_abi_version()} but "
                               f"{HEADER} declares ABI {abi_version()}: rebuild the library")
        for name, (ret, params) in declarations().items():
            fn = getattr(L, name)
            fn.argtypes = [_argtype(t) for t, _ in params]
            fn.restype = {"int": ctypes.c_int, "size_t": ctypes.c_size_t}.get(ret, ctypes.c_char_p)
        _lib = L
        # tuning switches for A/B runs (tools, bench): kernel-choice overrides from the env
        if os.environ.get("CULLAVO_ATTN_BWD_MODE"):
            L.cullavo_attn_set_bwd_tiles(int(os.environ["CULLAVO_ATTN_BWD_MODE"]))
        if os.environ.get("CULLAVO_ATTN_BWD_STAGE"):  # backward staging A/B (cullavo_attn_set_bwd_stage)
            L.cullavo_attn_set_bwd_stage(int(os.environ["CULLAVO_ATTN_BWD_STAGE"]))
        if os.environ.get("CULLAVO_GEMM_TILE"):
            L.cullavo_gemm_set_tile(int(os.environ["CULLAVO_GEMM_TILE"]))
        if os.environ.get("CULLAVO_SPLITK_TARGET"):  # split-K plan A/B (cullavo_gemm_set_splitk_target)
            L.cullavo_gemm_set_splitk_target(int(os.environ["CULLAVO_SPLITK_TARGET"]))
        if os.environ.get("CULLAVO_GEMM_MSPLIT"):  # M-tail split A/B (cullavo_gemm_set_msplit)
            L.cullavo_gemm_set_msplit(int(os.environ["CULLAVO_GEMM_MSPLIT"]))
        if os.environ.get("CULLAVO_GEMM_GROUP"):  # tile-order A/B (cullavo_gemm_set_group)
            L.cullavo_gemm_set_group(int(os.environ["CULLAVO_GEMM_GROUP"]))
        if os.environ.get("CULLAVO_GEMM_EPILOGUE"):  # epilogue A/B: bit 0 LDS-staged, bit 1 nt stores
            L.cullavo_gemm_set_epilogue(int(os.environ["CULLAVO_GEMM_EPILOGUE"]))
        if os.environ.get("CULLAVO_GEMM_DMA"):  # DMA-offset A/B (cullavo_gemm_set_dma)
            L.cullavo_gemm_set_dma(int(os.environ["CULLAVO_GEMM_DMA"]))
        if os.environ.get("CULLAVO_GEMV_NT"):  # decode weight-load policy A/B (cullavo_gemv_set_nt)
            L.cullavo_gemv_set_nt(int(os.environ["CULLAVO_GEMV_NT"]))
        if os.environ.get("CULLAVO_RATE288") is not None:  # 288-row tile A/B (0 = out of the plan)
            L.cullavo_gemm_set_tile_rate(10, float(os.environ["CULLAVO_RATE288"]), None)
        if os.environ.get("CULLAVO_ATTN_RESCALE"):  # deferred-rescale A/B (cullavo_attn_set_rescale)
            L.cullavo_attn_set_rescale(float(os.environ["CULLAVO_ATTN_RESCALE"]), None)
    return _lib


class CullavoError(RuntimeError):
    pass


def call(name: str, *args) -> int:
    """Invoke cullavo_<name>; raise CullavoError with cullavo_last_error() on failure."""
    L = lib()
    rc = getattr(L, "cullavo_" + name)(*args)
    if rc != 0:
        msg = L.cullavo_last_error().decode(errors="replace")
        if rc == 1:
            raise ValueError(f"cullavo_{name}: {msg}")
        raise CullavoError(f"cullavo_{name} failed (code {rc}): {msg}")
    return rc
