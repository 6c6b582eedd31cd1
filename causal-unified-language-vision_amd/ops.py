"""Torch-facing wrappers of the C-ABI kernels (one function per cullavo_* entry point).

PyTorch owns every tensor (caching allocator); these wrappers only validate shapes, allocate
outputs/workspaces with torch and pass raw device pointers plus the current HIP stream across
the boundary (SURVEY.md §8(b) "Ownership", "Threading / streams"). Nothing here computes on
the CPU: every function requires CUDA(HIP) tensors and fails loudly otherwise.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from ._lib import ACT_GELU, ACT_NONE, ACT_QUICK_GELU, ACT_SWIGLU_BWD, DT_BF16, DT_F32, call, lib

__all__ = [
    "ACT_NONE", "ACT_GELU", "ACT_QUICK_GELU", "ACT_SWIGLU_BWD", "gemm", "gemm_ex", "linear", "linear_dx", "linear_dx_t", "transpose2d", "linear_dw",
    "rmsnorm_fwd", "rmsnorm_bwd", "layernorm_fwd", "layernorm_bwd", "swiglu_fwd", "swiglu_bwd",
    "act_bwd", "colsum", "rope", "attn_fwd", "attn_bwd", "embedding_fwd", "embedding_bwd",
    "im2col_patches", "vision_embed_ln", "merge_plan", "row_gather2", "shift_targets", "ce_fwd",
    "ce_reduce", "ce_bwd", "adamw", "sumsq", "clip_coef", "scale_inplace", "kv_append", "attn_decode",
    "clip_image_preprocess", "visimage_geometry", "draw_boxes",
]

_DT = {torch.bfloat16: DT_BF16, torch.float32: DT_F32}


def _dt(t: torch.Tensor) -> int:
    try:
        return _DT[t.dtype]
    except KeyError:
        raise TypeError(f"unsupported dtype {t.dtype} (bf16 / f32 only)") from None


def _dev(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("cullavo kernels run on the GPU only: got a CPU tensor (no CPU fallback)")


def _ptr(t):
    return None if t is None else t.data_ptr()


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _ld(t: torch.Tensor) -> int:
    """leading dimension (row stride, elements) of a 2-D row-major view"""
    if t.dim() != 2 or t.stride(1) != 1:
        raise ValueError("expected a 2-D view with unit column stride")
    return t.stride(0)


# ---- GEMM ------------------------------------------------------------------------------------
_TRACE = {"key": None, "events": []}


def trace_gemm(key):
    """Time GEMM launches with HIP events recorded on the stream each kernel is launched on
    (bench.py's roofline): key = (M, N, K, a_layout, b_layout) traces that problem, key = "all"
    every bf16 GEMM launch; None stops tracing."""
    _TRACE["key"] = key
    _TRACE["events"] = []


def _traced(key):
    k = _TRACE["key"]
    return k is not None and (k == "all" or k == key)


def trace_result():
    """(average ms per traced launch, number of launches); synchronises the events."""
    evs = _TRACE["events"]
    if not evs:
        return 0.0, 0
    evs[-1][1].synchronize()
    ms = [a.elapsed_time(b) for a, b, _ in evs]
    _TRACE["key"] = None
    return sum(ms) / len(ms), len(ms)


def trace_launches():
    """[(problem key, ms)] of every traced launch; synchronises the events and stops tracing."""
    evs = _TRACE["events"]
    _TRACE["key"] = None
    if not evs:
        return []
    evs[-1][1].synchronize()
    return [(k, a.elapsed_time(b)) for a, b, k in evs]


def _split256(M, N, K, a_layout, b_layout) -> bool:
    """the library splits this problem over K given a workspace from the caller: cullavo_gemm_plan
    tile 9 (a small 256x256 grid with a long K on the 8-wave kernel) or 100 + t (the M-tail split,
    whose thin second product runs split-K). Asked per call, not cached: the plan depends on the
    library's forced tile and tile rates (cullavo_gemm_set_tile / _set_tile_rate), which callers
    may change at any time (one ~1 us host call per GEMM)."""
    t = lib().cullavo_gemm_plan(M, N, K, a_layout, b_layout, None)
    return t == 9 or t >= 100


def gemm(a_layout: int, b_layout: int, M: int, N: int, K: int, A, lda, B, ldb, C, ldc, *,
         alpha: float = 1.0, bias=None, act: int = ACT_NONE, preact=None, residual=None, ldr: int = 0,
         beta: float = 0.0):
    _dev(A, B, C, bias, preact, residual)
    if A.dtype == torch.float32:  # f32 parity mode: every operand f32 (cullavo_gemm_ex f32_operands)
        return gemm_ex(a_layout, b_layout, M, N, K, A, lda, B, ldb, C, ldc, alpha=alpha, bias=bias, act=act,
                       preact=preact, residual=residual, ldr=ldr, beta=beta, split_k=False)
    if _split256(M, N, K, a_layout, b_layout):  # small grid, long K: split-K with a torch workspace
        return gemm_ex(a_layout, b_layout, M, N, K, A, lda, B, ldb, C, ldc, alpha=alpha, bias=bias, act=act,
                       preact=preact, residual=residual, ldr=ldr, beta=beta)
    traced = _traced((M, N, K, a_layout, b_layout))
    if traced:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(torch.cuda.current_stream())
    call("gemm", a_layout, b_layout, M, N, K, _ptr(A), lda, _ptr(B), ldb, _ptr(C), ldc, _dt(C), float(alpha),
         _ptr(bias), act, _ptr(preact), _ptr(residual), ldr, float(beta), _stream())
    if traced:
        e1.record(torch.cuda.current_stream())
        key = (M, N, K, a_layout, b_layout)
        _TRACE["events"].append((e0, e1, key))
    return C


class GemmDesc(ctypes.Structure):
    """Mirror of cullavo_gemm_desc (include/cullavo_capi.h); tests check the size against the
    library's cullavo_gemm_desc_size()."""
    _fields_ = [("a_layout", ctypes.c_int), ("b_layout", ctypes.c_int), ("M", ctypes.c_int64),
                ("N", ctypes.c_int64), ("K", ctypes.c_int64), ("A", ctypes.c_void_p), ("lda", ctypes.c_int64),
                ("B", ctypes.c_void_p), ("ldb", ctypes.c_int64), ("C", ctypes.c_void_p), ("ldc", ctypes.c_int64),
                ("c_dtype", ctypes.c_int), ("alpha", ctypes.c_float), ("bias", ctypes.c_void_p),
                ("act", ctypes.c_int), ("preact", ctypes.c_void_p), ("residual", ctypes.c_void_p),
                ("ldr", ctypes.c_int64), ("beta", ctypes.c_float), ("addend", ctypes.c_void_p),
                ("ld_addend", ctypes.c_int64), ("drop_operand", ctypes.c_int), ("drop_p", ctypes.c_float),
                ("drop_seed", ctypes.c_uint64), ("workspace", ctypes.c_void_p), ("workspace_bytes", ctypes.c_int64),
                ("f32_operands", ctypes.c_int), ("lora_u", ctypes.c_void_p), ("ld_lora_u", ctypes.c_int64),
                ("lora_b", ctypes.c_void_p), ("lora_out", ctypes.c_int64), ("lora_r", ctypes.c_int),
                ("lora_scale", ctypes.c_float)]


DROP_NONE, DROP_A, DROP_B, DROP_OUT = 0, 1, 2, 3
SMALL_M = 256  # Linear calls with at most this many rows (KV-cache decode) may run split-K
# the LoRA up-projection fused into the base GEMM (cullavo_gemm_desc.lora_*): on by default; the
# unfused path (t materialised by its own GEMMs, added as `addend`) stays for A/B and ineligible shapes
LORA_FUSE = os.environ.get("CULLAVO_LORA_FUSE", "1") != "0"


def gemm_ex(a_layout: int, b_layout: int, M: int, N: int, K: int, A, lda, B, ldb, C, ldc, *,
            alpha: float = 1.0, bias=None, act: int = ACT_NONE, preact=None, residual=None, ldr: int = 0,
            beta: float = 0.0, addend=None, ld_addend: int = 0, drop_operand: int = DROP_NONE,
            drop_p: float = 0.0, drop_seed: int = 0, split_k: bool = True, lora=None):
    """cullavo_gemm_ex: gemm() plus the LoRA addend, dropout masks and split-K (see the header).
    The split-K workspace comes from torch's caching allocator (kernels never allocate).
    lora = (u, b_stack, module_width, scale): the fused LoRA up-projection (ABI 3 desc fields)."""
    _dev(A, B, C, bias, preact, residual, addend)
    f32 = A.dtype == torch.float32
    for t in (B, C, bias, preact, residual, addend):
        if f32 and t is not None and t.dtype != torch.float32:
            raise TypeError("gemm: f32 operands need every operand and the output in f32")
    d = GemmDesc(a_layout, b_layout, M, N, K, _ptr(A), lda, _ptr(B), ldb, _ptr(C), ldc, _dt(C), float(alpha),
                 _ptr(bias), act, _ptr(preact), _ptr(residual), ldr, float(beta), _ptr(addend), ld_addend,
                 drop_operand, float(drop_p), int(drop_seed) & 0xFFFFFFFFFFFFFFFF, None, 0, int(f32))
    if lora is not None:
        u, bst, width, scale = lora
        _dev(u, bst)
        d.lora_u, d.ld_lora_u, d.lora_b, d.lora_out = _ptr(u), _ld(u), _ptr(bst), int(width)
        d.lora_r, d.lora_scale = int(bst.shape[1]), float(scale)
        split_k = False
    ws = None
    # decode rows (M <= 16, forward layouts): the library streams W through its GEMV kernel
    # (cullavo_gemm_plan tile 14) and takes no split-K workspace
    gemv = M <= 16 and not f32 and lib().cullavo_gemm_plan(M, N, K, a_layout, b_layout, None) == 14
    if split_k and not f32 and not gemv:
        nbytes = lib().cullavo_gemm_workspace(ctypes.addressof(d))
        if nbytes:
            ws = torch.empty(nbytes, dtype=torch.uint8, device=C.device)
            d.workspace, d.workspace_bytes = ws.data_ptr(), nbytes
    # traced: the unsplit launches and the 8-wave split-K (bench.py names its family by cullavo_gemm_plan)
    traced = (not f32 and (ws is None or _split256(M, N, K, a_layout, b_layout)) and not (drop_operand and drop_p > 0)
              and _traced((M, N, K, a_layout, b_layout)))
    if traced:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(torch.cuda.current_stream())
    call("gemm_ex", ctypes.addressof(d), _stream())
    if traced:
        e1.record(torch.cuda.current_stream())
        # the key names the kernel's problem; a 6th element marks the LoRA-fused instantiation
        key = (M, N, K, a_layout, b_layout) if lora is None else (M, N, K, a_layout, b_layout, "lora")
        _TRACE["events"].append((e0, e1, key))
    return C


def linear(x, w, bias=None, *, act: int = ACT_NONE, residual=None, want_preact: bool = False, out=None,
           addend=None):
    """y = act(x @ w.T + bias [+ addend]) (+ residual); x [M,K] (row stride may exceed K), w [N,K].
    addend [M,N] is the LoRA term, added after the bias with peft's roundings; it may also be a
    lora.LoraTerm (the adapters' u, not yet multiplied by lora_B), which the base GEMM fuses when
    the library can (lora_fusable) and which is materialised otherwise."""
    M, K = x.shape
    N = w.shape[0]
    if w.shape[1] != K:
        raise ValueError(f"linear: x {tuple(x.shape)} vs w {tuple(w.shape)}")
    y = out if out is not None else torch.empty((M, N), dtype=x.dtype, device=x.device)
    pre = torch.empty((M, N), dtype=x.dtype, device=x.device) if want_preact else None
    ldr = _ld(residual) if residual is not None else 0
    if addend is not None and hasattr(addend, "fused_args"):
        fa = addend.fused_args(M, N) if LORA_FUSE and x.dtype == torch.bfloat16 else None
        if fa is not None:
            gemm_ex(0, 0, M, N, K, x, _ld(x), w, _ld(w), y, _ld(y), bias=bias, act=act, preact=pre,
                    residual=residual, ldr=ldr, lora=fa)
            return (y, pre) if want_preact else y
        addend = addend.materialize()
    if addend is None and M > SMALL_M:
        gemm(0, 0, M, N, K, x, _ld(x), w, _ld(w), y, _ld(y), bias=bias, act=act, preact=pre,
             residual=residual, ldr=ldr)
    elif addend is None:  # decode-sized rows: let the library split K over the idle CUs
        gemm_ex(0, 0, M, N, K, x, _ld(x), w, _ld(w), y, _ld(y), bias=bias, act=act, preact=pre,
                residual=residual, ldr=ldr)
    else:
        if addend.shape != (M, N):
            raise ValueError(f"linear: addend {tuple(addend.shape)} != {(M, N)}")
        gemm_ex(0, 0, M, N, K, x, _ld(x), w, _ld(w), y, _ld(y), bias=bias, act=act, preact=pre,
                residual=residual, ldr=ldr, addend=addend, ld_addend=_ld(addend))
    return (y, pre) if want_preact else y


def _swiglu_dx(a_layout_b, M, K, N, dy, w, gu):
    """dgu [M, 2K] = swiglu_bwd(dy @ w, gu) with the SwiGLU backward in the GEMM epilogue."""
    if gu.shape != (M, 2 * K) or gu.dtype != torch.bfloat16 or dy.dtype != torch.bfloat16:
        raise ValueError(f"swiglu dx: gu {tuple(gu.shape)} {gu.dtype} vs {(M, 2 * K)} bf16")
    dgu = torch.empty((M, 2 * K), dtype=dy.dtype, device=dy.device)
    gemm(0, a_layout_b, M, K, N, dy, _ld(dy), w, _ld(w), dgu, _ld(dgu), act=ACT_SWIGLU_BWD, residual=gu,
         ldr=_ld(gu))
    return dgu


def linear_dx(dy, w, *, residual=None, out=None, swiglu_gu=None):
    """dx = dy @ w (+ residual); dy [M,N], w [N,K] -> [M,K]. With swiglu_gu = gu [M, 2K] (the
    SwiGLU's gate | up) it returns swiglu_bwd(dx, gu) [M, 2K] instead, fused into the GEMM."""
    M, N = dy.shape
    K = w.shape[1]
    if swiglu_gu is not None:
        return _swiglu_dx(1, M, K, N, dy, w, swiglu_gu)
    dx = out if out is not None else torch.empty((M, K), dtype=dy.dtype, device=dy.device)
    gemm(0, 1, M, K, N, dy, _ld(dy), w, _ld(w), dx, _ld(dx), residual=residual,
         ldr=_ld(residual) if residual is not None else 0)
    return dx


def linear_dx_t(dy, wt, *, residual=None, out=None, swiglu_gu=None):
    """dx = dy @ wt.T (+ residual); dy [M,N], wt [K,N] (the K-major copy of w [N,K], ParamArena
    .transposed): both operands reduction-contiguous, bitwise equal to linear_dx(dy, w)."""
    M, N = dy.shape
    K = wt.shape[0]
    if wt.shape[1] != N:
        raise ValueError(f"linear_dx_t: dy {tuple(dy.shape)} vs wt {tuple(wt.shape)}")
    if swiglu_gu is not None:
        return _swiglu_dx(0, M, K, N, dy, wt, swiglu_gu)
    dx = out if out is not None else torch.empty((M, K), dtype=dy.dtype, device=dy.device)
    gemm(0, 0, M, K, N, dy, _ld(dy), wt, _ld(wt), dx, _ld(dx), residual=residual,
         ldr=_ld(residual) if residual is not None else 0)
    return dx


def transpose2d(src, dst):
    """dst[c, r] = src[r, c] for 16-bit matrices (cullavo_transpose16); returns dst."""
    _dev(src, dst)
    if src.dtype not in (torch.bfloat16, torch.float16) or dst.dtype != src.dtype:
        raise ValueError("transpose2d: bf16/fp16 tensors of one dtype")
    rows, cols = src.shape
    if dst.shape != (cols, rows) or src.stride(1) != 1 or dst.stride(1) != 1:
        raise ValueError(f"transpose2d: src {tuple(src.shape)} -> dst {tuple(dst.shape)} (row-major)")
    call("transpose16", _ptr(src), src.stride(0), _ptr(dst), dst.stride(0), rows, cols, _stream())
    return dst


def linear_dw(dy, x, out, *, beta: float = 0.0):
    """out[N,K] = dy^T x (+ beta*out); dy [M,N], x [M,K]"""
    M, N = dy.shape
    K = x.shape[1]
    if out.shape != (N, K):
        raise ValueError(f"linear_dw: out {tuple(out.shape)} != {(N, K)}")
    gemm(1, 1, N, K, M, dy, _ld(dy), x, _ld(x), out, _ld(out), beta=beta)
    return out


# ---- norms -----------------------------------------------------------------------------------
def rmsnorm_fwd(x, w, eps: float):
    _dev(x, w)
    rows, cols = x.shape
    y = torch.empty_like(x)
    rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
    call("rmsnorm_fwd", _ptr(x), _ptr(w), _ptr(y), _ptr(rstd), rows, cols, float(eps), _dt(x), _stream())
    return y, rstd


def _norm_ws(rows, cols, device):
    n = lib().cullavo_norm_bwd_workspace(rows, cols) // 4
    return torch.empty(n, dtype=torch.float32, device=device)


def rmsnorm_bwd(dy, x, w, rstd, *, dres=None, dw=None, beta: float = 0.0):
    _dev(dy, x, w, rstd, dres, dw)
    rows, cols = x.shape
    dx = torch.empty_like(x)
    ws = _norm_ws(rows, cols, x.device) if dw is not None else None
    call("rmsnorm_bwd", _ptr(dy), _ptr(x), _ptr(w), _ptr(rstd), _ptr(dx), _ptr(dres), _ptr(dw),
         _dt(dw) if dw is not None else DT_BF16, float(beta), _ptr(ws), rows, cols, _dt(x), _stream())
    return dx


def layernorm_fwd(x, w, b, eps: float):
    _dev(x, w, b)
    rows, cols = x.shape
    y = torch.empty_like(x)
    mean = torch.empty(rows, dtype=torch.float32, device=x.device)
    rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
    call("layernorm_fwd", _ptr(x), _ptr(w), _ptr(b), _ptr(y), _ptr(mean), _ptr(rstd), rows, cols, float(eps),
         _dt(x), _stream())
    return y, mean, rstd


def layernorm_bwd(dy, x, w, mean, rstd, *, dres=None, dw=None, db=None, beta: float = 0.0):
    _dev(dy, x, w, mean, rstd, dres, dw, db)
    rows, cols = x.shape
    dx = torch.empty_like(x)
    ws = _norm_ws(rows, cols, x.device) if dw is not None else None
    call("layernorm_bwd", _ptr(dy), _ptr(x), _ptr(w), _ptr(mean), _ptr(rstd), _ptr(dx), _ptr(dres), _ptr(dw),
         _ptr(db), _dt(dw) if dw is not None else DT_BF16, float(beta), _ptr(ws), rows, cols, _dt(x), _stream())
    return dx


# ---- element-wise ----------------------------------------------------------------------------
def swiglu_fwd(gu):
    _dev(gu)
    rows, F2 = gu.shape
    out = torch.empty((rows, F2 // 2), dtype=gu.dtype, device=gu.device)
    call("swiglu_fwd", _ptr(gu), rows, F2 // 2, _ptr(out), _dt(gu), _stream())
    return out


def lora_dx(du, a_stack, dx, *, n_mod: int, drop_p: float, seeds):
    """dx += the LoRA group's input gradient through its dropout, one launch (cullavo_lora_dx):
    for m in order, dx = bf16(dx + mask_m / (1-p) * du[:, 64m:64m+64] @ a_stack[64m:64m+64]),
    bitwise the per-module gemm_ex(0, 1, ..., drop_operand=DROP_OUT, beta=1) calls."""
    _dev(du, a_stack, dx)
    M, N = dx.shape
    s = [int(x) for x in seeds] + [0] * (3 - len(seeds))
    call("lora_dx", int(n_mod), M, N, _ptr(du), _ld(du), _ptr(a_stack), _ld(a_stack), _ptr(dx), _ld(dx),
         float(drop_p), s[0], s[1], s[2], _stream())
    return dx


def decode_linear(x, w, *, transform: int = 0, norm_w=None, eps: float = 0.0, residual=None):
    """Decode rows (M <= 16) through cullavo_decode_linear: y = T(x) @ w.T (+ residual) with T the
    fused input transform (0 none, 1 RMSNorm with norm_w / eps, 2 SwiGLU of x = gate|up [M, 2K]);
    transform 3: y = SwiGLU(x @ w.T) for the fused gate|up weight w [2N, K] (y [M, N]); 4: 1 and 3."""
    _dev(x, w, norm_w, residual)
    M = x.shape[0]
    N, K = w.shape
    if transform in (3, 4):
        N //= 2
    y = torch.empty((M, N), dtype=x.dtype, device=x.device)
    call("decode_linear", int(transform), M, N, K, _ptr(x), _ld(x), _ptr(norm_w), float(eps), _ptr(w), _ld(w),
         _ptr(y), _ld(y), _ptr(residual), _ld(residual) if residual is not None else 0, _stream())
    return y


def swiglu_bwd(dout, gu):
    _dev(dout, gu)
    rows, F2 = gu.shape
    dgu = torch.empty_like(gu)
    call("swiglu_bwd", _ptr(dout), _ptr(gu), rows, F2 // 2, _ptr(dgu), _dt(gu), _stream())
    return dgu


def act_bwd(act: int, dy, preact):
    _dev(dy, preact)
    dx = torch.empty_like(dy)
    call("act_bwd", act, _ptr(dy), _ptr(preact), _ptr(dx), dy.numel(), _dt(dy), _stream())
    return dx


def colsum(x, out, *, beta: float = 0.0):
    _dev(x, out)
    rows, cols = x.shape
    ws = torch.empty(lib().cullavo_colsum_workspace(rows, cols) // 4, dtype=torch.float32, device=x.device)
    call("colsum", _ptr(x), rows, cols, _ptr(out), _dt(out), float(beta), _ptr(ws), _dt(x), _stream())
    return out


def rope(q, k, position_ids, *, hq: int, hk: int, head_dim: int, theta: float, inverse: bool = False):
    """in-place rotary embedding of q [T, >=hq*D] and k [T, >=hk*D] (views with row strides)"""
    _dev(q, k, position_ids)
    T = q.shape[0]
    call("rope", _ptr(q), _ld(q), _ptr(k), _ld(k) if k is not None else 0, _ptr(position_ids), T, hq, hk,
         head_dim, float(theta), int(inverse), _dt(q), _stream())


# ---- attention -------------------------------------------------------------------------------
def attn_fwd(q, k, v, *, B: int, H: int, Lq: int, Lk: int, D: int, scale: float, causal: bool,
             kv_start=None, out=None):
    """q/k/v: [B*L, >=H*D] row-strided views. Returns (o [B*Lq, H*D], lse [B,H,Lq] f32)."""
    _dev(q, k, v, kv_start)
    o = out if out is not None else torch.empty((B * Lq, H * D), dtype=q.dtype, device=q.device)
    lse = torch.empty((B, H, Lq), dtype=torch.float32, device=q.device)
    call("attn_fwd", _ptr(q), _ld(q), _ptr(k), _ld(k), _ptr(v), _ld(v), _ptr(o), _ld(o), _ptr(lse), B, H, Lq, Lk,
         D, float(scale), int(causal), _ptr(kv_start), _dt(q), _stream())
    return o, lse


def rope_kv_append(q, k, v, position_ids, k_cache, v_cache, start, *, hq: int, head_dim: int, theta: float,
                   B: int, Lnew: int):
    """cullavo_rope_kv_append: rope(q, k) in place on q, the rotated k and v appended to the caches
    (k itself is left unrotated); bitwise rope() + kv_append()."""
    _dev(q, k, v, position_ids, k_cache, v_cache, start)
    hd = k_cache.shape[-1]
    call("rope_kv_append", _ptr(q), _ld(q), _ptr(k), _ld(k), _ptr(v), _ld(v), _ptr(position_ids), B * Lnew, hq,
         hd // head_dim, head_dim, float(theta), _ptr(k_cache), _ptr(v_cache), k_cache.stride(1), k_cache.stride(0),
         _ptr(start), Lnew, _dt(q), _stream())


def kv_append(k, v, k_cache, v_cache, start, *, B: int, Lnew: int):
    """k, v: [B*Lnew, >=hd] row-strided views; caches [B, Lmax, hd]; start int32 [B]."""
    _dev(k, v, k_cache, v_cache, start)
    hd = k_cache.shape[-1]
    call("kv_append", _ptr(k), _ld(k), _ptr(v), _ld(v), _ptr(k_cache), _ptr(v_cache), k_cache.stride(1),
         k_cache.stride(0), _ptr(start), B, Lnew, hd, _stream())


def attn_decode_rope(q, k, v, position_ids, k_cache, v_cache, start, *, B: int, H: int, D: int, max_len: int,
                     scale: float, theta: float, kv_start=None, out=None):
    """cullavo_attn_decode_rope: rope_kv_append (Lnew = 1) + attn_decode over keys
    [kv_start, start + 1) in one pass; q, k, v the unrotated projection rows [B, >=H*D] (q is left
    unrotated), the rotated key and the value written to cache row start[b]."""
    _dev(q, k, v, position_ids, k_cache, v_cache, start, kv_start)
    o = out if out is not None else torch.empty((B, H * D), dtype=q.dtype, device=q.device)
    nbytes = lib().cullavo_attn_decode_workspace(B, H, max_len, D)
    ws = torch.empty(nbytes // 4, dtype=torch.float32, device=q.device)
    call("attn_decode_rope", _ptr(q), _ld(q), _ptr(k), _ld(k), _ptr(v), _ld(v), _ptr(position_ids), float(theta),
         _ptr(k_cache), _ptr(v_cache), k_cache.stride(1), k_cache.stride(0), _ptr(start), _ptr(kv_start), _ptr(o),
         _ld(o), B, H, max_len, D, float(scale), _ptr(ws), _stream())
    return o


def attn_decode(q, k_cache, v_cache, kv_len, *, B: int, H: int, D: int, max_len: int, scale: float,
                kv_start=None, out=None):
    """One query row per batch (q [B, >=H*D]) against cache keys kv_start[b] <= j < kv_len[b]."""
    _dev(q, k_cache, v_cache, kv_len, kv_start)
    o = out if out is not None else torch.empty((B, H * D), dtype=q.dtype, device=q.device)
    nbytes = lib().cullavo_attn_decode_workspace(B, H, max_len, D)
    ws = torch.empty(nbytes // 4, dtype=torch.float32, device=q.device)
    call("attn_decode", _ptr(q), _ld(q), _ptr(k_cache), _ptr(v_cache), k_cache.stride(1), k_cache.stride(0),
         _ptr(kv_len), _ptr(kv_start), _ptr(o), _ld(o), B, H, max_len, D, float(scale), _ptr(ws), _stream())
    return o


def attn_bwd(q, k, v, o, do, lse, *, B: int, H: int, Lq: int, Lk: int, D: int, scale: float, causal: bool,
             kv_start=None, dq=None, dk=None, dv=None):
    _dev(q, k, v, o, do, lse, kv_start)
    dq = dq if dq is not None else torch.empty((B * Lq, H * D), dtype=q.dtype, device=q.device)
    dk = dk if dk is not None else torch.empty((B * Lk, H * D), dtype=q.dtype, device=q.device)
    dv = dv if dv is not None else torch.empty((B * Lk, H * D), dtype=q.dtype, device=q.device)
    delta = torch.empty((B, H, Lq), dtype=torch.float32, device=q.device)
    nbytes = lib().cullavo_attn_bwd_workspace(B, H, Lq, Lk, D, _dt(q))
    ws = torch.empty(nbytes, dtype=torch.uint8, device=q.device) if nbytes else None
    call("attn_bwd_ws", _ptr(q), _ld(q), _ptr(k), _ld(k), _ptr(v), _ld(v), _ptr(o), _ld(o), _ptr(do), _ld(do),
         _ptr(lse), _ptr(delta), _ptr(dq), _ld(dq), _ptr(dk), _ld(dk), _ptr(dv), _ld(dv), B, H, Lq, Lk, D,
         float(scale), int(causal), _ptr(kv_start), _dt(q), _ptr(ws), nbytes, _stream())
    return dq, dk, dv


# ---- embeddings / merge ----------------------------------------------------------------------
def embedding_fwd(ids, table):
    _dev(ids, table)
    ids = ids.reshape(-1)
    vocab, dim = table.shape
    out = torch.empty((ids.numel(), dim), dtype=table.dtype, device=table.device)
    call("embedding_fwd", _ptr(ids), ids.numel(), _ptr(table), vocab, dim, _ptr(out), _dt(table), _stream())
    return out


def embedding_bwd(ids, dout, dtable, *, beta: float = 0.0):
    _dev(ids, dout, dtable)
    ids = ids.reshape(-1)
    vocab, dim = dtable.shape
    call("embedding_bwd", _ptr(ids), ids.numel(), _ptr(dout), vocab, dim, _ptr(dtable), _dt(dtable), float(beta),
         _dt(dout), _stream())
    return dtable


def im2col_patches(pixels, patch: int, kpad: int, dtype=torch.bfloat16):
    _dev(pixels)
    B, C, H, W = pixels.shape
    P = (H // patch) * (W // patch)
    out = torch.empty((B * (1 + P), kpad), dtype=dtype, device=pixels.device)
    pixels = pixels.contiguous()
    call("im2col_patches", _ptr(pixels), _dt(pixels), B, C, H, W, patch, _ptr(out), kpad, _dt(out), _stream())
    return out


def vision_embed_ln(x, cls, pos, w, b, *, B: int, T: int, eps: float):
    _dev(x, cls, pos, w, b)
    y = torch.empty_like(x)
    call("vision_embed_ln", _ptr(x), _ptr(cls), _ptr(pos), _ptr(w), _ptr(b), _ptr(y), B, T, x.shape[1],
         float(eps), _dt(x), _stream())
    return y


def merge_plan(ids, mask, *, L: int, image_token: int, n_patches: int, left_padding: bool):
    _dev(ids, mask)
    B, S = ids.shape
    dev = ids.device
    text_dst = torch.empty((B, S), dtype=torch.int64, device=dev)
    src = torch.empty((B, L), dtype=torch.int64, device=dev)
    mmask = torch.empty((B, L), dtype=torch.int64, device=dev)
    pos = torch.empty((B, L), dtype=torch.int64, device=dev)
    ids = ids.contiguous()
    mask = mask.contiguous().to(torch.int64) if mask is not None else None
    call("merge_plan", _ptr(ids), _ptr(mask), B, S, L, int(image_token), int(n_patches), int(left_padding),
         _ptr(text_dst), _ptr(src), _ptr(mmask), _ptr(pos), _stream())
    return text_dst, src, mmask, pos


def row_gather2(src, a, b):
    _dev(src, a, b)
    dim = a.shape[-1]
    a2 = a.reshape(-1, dim)
    b2 = b.reshape(-1, dim) if b is not None else a2
    out = torch.empty((src.numel(), dim), dtype=a.dtype, device=a.device)
    call("row_gather2", _ptr(src), src.numel(), _ptr(a2), a2.shape[0], _ptr(b2), dim, _ptr(out), _dt(a), _stream())
    return out


# ---- loss ------------------------------------------------------------------------------------
def shift_targets(labels, mask, ignore_index: int = -100):
    _dev(labels, mask)
    B, L = labels.shape
    if mask is not None and tuple(mask.shape) != (B, L):
        raise ValueError(f"shift_targets: labels {tuple(labels.shape)} and attention mask {tuple(mask.shape)} differ")
    tgt = torch.empty((B * L,), dtype=torch.int64, device=labels.device)
    labels = labels.contiguous().to(torch.int64)
    mask = mask.contiguous().to(torch.int64) if mask is not None else None
    call("shift_targets", _ptr(labels), _ptr(mask), B, L, int(ignore_index), _ptr(tgt), _stream())
    return tgt


def ce_fwd(logits, targets, ignore_index: int = -100):
    _dev(logits, targets)
    rows, V = logits.shape
    if targets.numel() != rows:
        raise ValueError(f"ce_fwd: {targets.numel()} targets for {rows} logit rows")
    row_loss = torch.empty(rows, dtype=torch.float32, device=logits.device)
    row_lse = torch.empty(rows, dtype=torch.float32, device=logits.device)
    call("ce_fwd", _ptr(logits), _ld(logits), _ptr(targets), rows, V, int(ignore_index), _ptr(row_loss),
         _ptr(row_lse), _dt(logits), _stream())
    return row_loss, row_lse


def ce_reduce(row_loss, targets, ignore_index: int = -100):
    out = torch.empty(3, dtype=torch.float32, device=row_loss.device)
    call("ce_reduce", _ptr(row_loss), _ptr(targets), row_loss.numel(), int(ignore_index), _ptr(out), _stream())
    return out


def ce_bwd(logits, targets, row_lse, loss_out, grad_loss=None, ignore_index: int = -100, out=None):
    _dev(logits, targets, row_lse, loss_out, grad_loss)
    rows, V = logits.shape
    d = out if out is not None else torch.empty_like(logits)
    call("ce_bwd", _ptr(logits), _ld(logits), _ptr(targets), _ptr(row_lse), _ptr(loss_out), _ptr(grad_loss), rows,
         V, int(ignore_index), _ptr(d), _ld(d), _dt(logits), _stream())
    return d


# ---- optimiser -------------------------------------------------------------------------------
def adamw(param, grad, exp_avg, exp_avg_sq, *, lr: float, beta1: float, beta2: float, eps: float,
          weight_decay: float, step: int, grad_scale=None):
    _dev(param, grad, exp_avg, exp_avg_sq, grad_scale)
    call("adamw", _ptr(param), _ptr(grad), _ptr(exp_avg), _ptr(exp_avg_sq), param.numel(), float(lr),
         float(beta1), float(beta2), float(eps), float(weight_decay), int(step), _ptr(grad_scale), _dt(param),
         _dt(exp_avg), _stream())


SUMSQ_PARTIALS = 1024  # CULLAVO_SUMSQ_PARTIALS
_SUMSQ_WS: dict = {}


def sumsq(x, out):
    """out[0] += sum(x^2), deterministic (fixed-order block partials in a cached f32 workspace;
    calls are stream-ordered, so one workspace per device serves them all)"""
    _dev(x, out)
    if not x.is_contiguous():
        raise ValueError("sumsq: x must be contiguous")
    ws = _SUMSQ_WS.get(x.device)
    if ws is None:
        ws = _SUMSQ_WS[x.device] = torch.empty(SUMSQ_PARTIALS, dtype=torch.float32, device=x.device)
    call("sumsq", _ptr(x), x.numel(), _ptr(out), _ptr(ws), _dt(x), _stream())


def clip_coef(sumsq_buf, max_norm: float, coef, norm_out=None):
    call("clip_coef", _ptr(sumsq_buf), float(max_norm), _ptr(coef), _ptr(norm_out), _stream())


def scale_inplace(x, scale):
    call("scale_inplace", _ptr(x), x.numel(), _ptr(scale), _dt(x), _stream())


# ---- image preprocessing (data step) -----------------------------------------------------------
def clip_image_preprocess(images, Hr, Wr, h_bounds, h_kk, h_ksize, v_bounds, v_kk, v_ksize, top, left, crop_h,
                          crop_w, rescale, mean, std, tmp, out):
    """uint8 [B, C, H, W] (any strides) -> out [B, C, crop_h, crop_w]: PIL-bicubic resize to
    (Hr, Wr) with the given Pillow coefficient tables, crop at (top, left), rescale, normalise"""
    _dev(images, h_bounds, h_kk, v_bounds, v_kk, tmp, out)
    B, C, H, W = images.shape
    if not out.is_contiguous() or tuple(out.shape) != (B, C, crop_h, crop_w):
        raise ValueError("out must be a contiguous [B, C, crop_h, crop_w] tensor")
    if tmp.numel() < B * C * H * crop_w:
        raise ValueError("tmp too small")
    sb, sc, sy, sx = images.stride()
    call("clip_image_preprocess", _ptr(images), B, C, H, W, sb, sc, sy, sx, Hr, Wr, _ptr(h_bounds), _ptr(h_kk),
         int(h_ksize), _ptr(v_bounds), _ptr(v_kk), int(v_ksize), top, left, crop_h, crop_w, float(rescale),
         *[float(m) for m in mean], *[float(s) for s in std], _ptr(tmp), _ptr(out), _dt(out), _stream())
    return out


_VISIMAGE = {}


def visimage_geometry(H: int, W: int, device):
    """(rows, cols) device int32 maps and transData (sx, tx, sy, ty) of a VisImage of H x W"""
    key = (H, W, str(device))
    if key not in _VISIMAGE:
        rows = np.zeros(H, np.int32)
        cols = np.zeros(W, np.int32)
        td = np.zeros(4, np.float64)
        rc = lib().cullavo_visimage_geometry(H, W, rows.ctypes.data, cols.ctypes.data, td.ctypes.data)
        if rc != 0:
            raise RuntimeError(f"cullavo_visimage_geometry({H}, {W}) failed: {lib().cullavo_last_error().decode()}")
        _VISIMAGE[key] = (torch.from_numpy(rows).to(device), torch.from_numpy(cols).to(device),
                          tuple(float(v) for v in td))
    return _VISIMAGE[key]


def draw_order(boxes: np.ndarray) -> np.ndarray:
    """overlay_instances' order: np.argsort(-areas) on the float32 boxes (largest first)"""
    b = np.asarray(boxes, np.float32).reshape(-1, 4)
    return np.argsort(-np.prod(b[:, 2:] - b[:, :2], axis=1))


def draw_boxes(images, boxes, colors, font_size: float = 16.0, alpha: float = 0.5, check: bool = True):
    """Visualizer(img).overlay_instances(boxes, assigned_colors).get_image() for a batch.

    images: uint8 [B, 3, H, W] on the GPU (any strides); boxes: per image an [n_i, 4] array of
    (x0, y0, x1, y1) pixels (float32, as the reference passes them); colors: per image n_i RGB
    triples. Returns a new uint8 [B, 3, H, W] tensor. check=True reads the kernel's overflow
    flag back (one small device-to-host copy) and raises if a box exceeded its capacity."""
    _dev(images)
    if images.dtype != torch.uint8 or images.dim() != 4 or images.shape[1] != 3:
        raise ValueError("images must be a uint8 [B, 3, H, W] tensor")
    B, _, H, W = images.shape
    if len(boxes) != B or len(colors) != B:
        raise ValueError("one box list and one colour list per image")
    dev = images.device
    rows, cols, td = visimage_geometry(H, W, dev)
    nmax = max([len(b) for b in boxes] + [0])
    bx = np.zeros((B, max(nmax, 1), 4), np.float32)
    cl = np.zeros((B, max(nmax, 1), 3), np.uint8)
    nb = np.zeros(B, np.int32)
    for i, (b, c) in enumerate(zip(boxes, colors)):
        b = np.asarray(b, np.float32).reshape(-1, 4)
        if not np.isfinite(b).all():
            raise ValueError(f"image {i}: box coordinates must be finite")
        if len(c) != len(b):
            raise ValueError(f"image {i}: {len(b)} boxes but {len(c)} colours")
        order = draw_order(b)
        bx[i, :len(b)] = b[order]
        cl[i, :len(b)] = np.asarray(c, np.uint8).reshape(-1, 3)[order]
        nb[i] = len(b)
    bx_d = torch.from_numpy(bx).to(dev)
    cl_d = torch.from_numpy(cl).to(dev)
    nb_d = torch.from_numpy(nb).to(dev)
    ws = torch.empty(int(lib().cullavo_draw_boxes_workspace(B, max(nmax, 1))), dtype=torch.uint8, device=dev)
    out = torch.empty((B, 3, H, W), dtype=torch.uint8, device=dev)
    width_px = max(font_size / 4.0, 1.0) * 100.0 / 72.0
    a8 = int(alpha * 255 + 0.5)
    sb, sc, sy, sx = images.stride()
    call("draw_boxes", _ptr(images), B, 3, H, W, sb, sc, sy, sx, _ptr(rows), _ptr(cols), _ptr(bx_d), _ptr(nb_d),
         _ptr(cl_d), nmax, *td, float(width_px), a8, _ptr(ws), _ptr(out), _stream())
    if check and int(ws[:4].view(torch.int32).item()) != 0:
        raise RuntimeError("draw_boxes: a box outline or its cells exceeded the kernel's capacity")
    return out
