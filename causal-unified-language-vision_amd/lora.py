"""LoRA adapters on the CuLLaVO path.

What the reference trains (cullavo/load_cullavo.py:94-112, :128-138): peft LoRA with r=64,
lora_alpha=16, lora_dropout=0.05, bias='none' on every Linear of the language model except
lm_head (find_all_linear_names, :8-20) and on every Linear of the vision tower except out_proj
in encoder layers 12-22 (layers_to_transform, :101); plus projector, lm_head and embed_tokens.
The base weights are frozen (the reference keeps them in NF4; here they stay bf16 in HBM).

peft's LoraLayer on an nn.Linear (peft, un-vendored and absent here, restated from its
published algorithm; oracle/cullavo_oracle.py:lora_linear is the CPU restatement):

    result = base_layer(x) + lora_B(lora_A(dropout(x))) * scaling,   scaling = lora_alpha / r
    lora_A.weight [r, in] ~ kaiming_uniform(a=sqrt(5)) = U(+-1/sqrt(in)),  lora_B.weight [out, r] = 0

MI355X mapping. The Linears that share one input form a group (q|k|v, gate|up, or a single
Linear); per group and step:
  forward   u = dropout_m(x) A_m^T        per module (mask applied while the operand is staged;
                                           one stacked GEMM when no dropout is active)
            t = scaling * u_m B_m^T       into the column block of module m
            y = x W^T (+ bias) + t        the base GEMM with t as its epilogue addend, with
                                           peft's roundings: round(round(x W^T + b) + t)
  backward  du = scaling * dy_m B_m       (the gradient of lora_A's output)
            dB_m = scaling * dy_m^T u_m,  dA_m = du_m^T dropout_m(x)
            dx += mask_m * du_m A_m / (1-p)   (mask applied in the GEMM epilogue, accumulating)
The dropout mask is a counter-based hash of (seed, token, feature) (csrc/common.h), so the
forward and both backward uses regenerate it instead of storing it.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field

import torch

from . import ops
from .ops import DROP_A, DROP_B, DROP_OUT

# CULLAVO_LORA_DX_FUSE=0: the per-module dx products instead of cullavo_lora_dx (A/B switch)
LORA_DX_FUSE = os.environ.get("CULLAVO_LORA_DX_FUSE", "1") != "0"

LM_TARGETS = ("q_proj", "k_proj", "v_proj", "o_proj", "gate_proj", "up_proj", "down_proj")
VISION_TARGETS = ("q_proj", "k_proj", "v_proj", "fc1", "fc2")


@dataclass
class LoraSettings:
    r: int = 64
    lora_alpha: float = 16.0
    lora_dropout: float = 0.05
    adapter: str = "step1"
    vision_layers: tuple = field(default_factory=lambda: tuple(range(12, 23)))
    lm: bool = True
    vision: bool = True

    @property
    def scaling(self) -> float:
        return self.lora_alpha / self.r


def lm_groups(cfg):
    """[(group, [(module suffix, out, in), ...])] of one decoder layer (inputs shared per group)."""
    d, f = cfg.hidden_size, cfg.intermediate_size
    return [("qkv", [(f"self_attn.{n}_proj", d, d) for n in "qkv"]),
            ("o", [("self_attn.o_proj", d, d)]),
            ("gu", [("mlp.gate_proj", f, d), ("mlp.up_proj", f, d)]),
            ("down", [("mlp.down_proj", d, f)])]


def vision_groups(cfg):
    d, f = cfg.hidden_size, cfg.intermediate_size
    return [("qkv", [(f"self_attn.{n}_proj", d, d) for n in "qkv"]),
            ("fc1", [("mlp.fc1", f, d)]),
            ("fc2", [("mlp.fc2", d, f)])]


def a_key(prefix, suffix, s: LoraSettings):
    return f"{prefix}{suffix}.lora_A.{s.adapter}.weight"


def b_key(prefix, suffix, s: LoraSettings):
    return f"{prefix}{suffix}.lora_B.{s.adapter}.weight"


def lora_specs(cuda_cfg, s: LoraSettings):
    """Arena layout: per group all lora_A of the group adjacent ([n*r, in] stack), then all
    lora_B adjacent. Keys follow peft's `<module>.lora_A.<adapter>.weight`."""
    specs = []

    def add(prefix, groups):
        for _, mods in groups:
            specs.extend((a_key(prefix, suf, s), (s.r, inn)) for suf, _, inn in mods)
            specs.extend((b_key(prefix, suf, s), (out, s.r)) for suf, out, _ in mods)

    if s.vision:
        v = cuda_cfg.vision_config
        for i in s.vision_layers:
            if i < v.num_hidden_layers:
                add(f"vision_tower.vision_model.encoder.layers.{i}.", vision_groups(v))
    if s.lm:
        t = cuda_cfg.text_config
        for i in range(t.num_hidden_layers):
            add(f"language_model.model.layers.{i}.", lm_groups(t))
    return specs


def init_lora_(arena, seed: int = 0):
    """peft's default init: lora_A ~ kaiming_uniform(a=sqrt(5)) = U(-1/sqrt(in), 1/sqrt(in)),
    lora_B = 0 (so the adapted model starts equal to the base model)."""
    g = torch.Generator(device=arena.device)
    g.manual_seed(seed)
    with torch.no_grad():
        for key, p in arena.params.items():
            if ".lora_A." in key:
                bound = 1.0 / math.sqrt(p.shape[1])
                p.uniform_(-bound, bound, generator=g)
            else:
                p.zero_()


_M64 = (1 << 64) - 1


def module_seed(step_seed: int, uid: int, m: int) -> int:
    """Per-module, per-step dropout seed (each peft LoRA module has its own nn.Dropout)."""
    x = (step_seed * 0x9E3779B97F4A7C15 + (uid * 8 + m + 1) * 0xBF58476D1CE4E5B9) & _M64
    x ^= x >> 31
    return (x * 0x94D049BB133111EB) & _M64


class LoraTerm:
    """The adapters' share t = scaling * u_m B_m^T of a group's Linear outputs, not yet computed.
    ops.linear fuses it into the base GEMM (cullavo_gemm_desc.lora_*: one 64-deep MFMA K-tile
    after the main loop, t added with peft's roundings and never written to HBM) when the library
    supports the shape, and calls materialize() (the separate r = 64 GEMMs) otherwise."""

    def __init__(self, group, u):
        self.group, self.u = group, u

    def fused_args(self, M: int, N: int):
        g = self.group
        w = g.outs[0]
        if (g.r != 64 or M <= 16 or N != g.out_total or any(o != w for o in g.outs) or w % 256
                or self.u.dtype != torch.bfloat16 or ops._ld(self.u) % 8):
            return None
        return self.u, g.b_stack(), w, g.scaling

    def materialize(self):
        return self.group.up_project(self.u)


class LoraGroup:
    """The LoRA adapters of the Linears that share one input (see the module docstring)."""

    def __init__(self, arena, prefix: str, mods, s: LoraSettings, uid: int):
        self.arena, self.s, self.uid = arena, s, uid
        self.r, self.n = s.r, len(mods)
        self.in_f = mods[0][2]
        self.outs = [o for _, o, _ in mods]
        self.offs = [sum(self.outs[:i]) for i in range(self.n)]
        self.out_total = sum(self.outs)
        self.suffixes = [suf for suf, _, _ in mods]
        self.a_keys = [a_key(prefix, suf, s) for suf in self.suffixes]
        self.b_keys = [b_key(prefix, suf, s) for suf in self.suffixes]
        arena.check_adjacent(self.a_keys)
        arena.check_adjacent(self.b_keys)

    @property
    def scaling(self):
        return self.s.scaling

    def A(self, m):
        return self.arena.params[self.a_keys[m]]

    def B(self, m):
        return self.arena.params[self.b_keys[m]]

    def a_stack(self):
        return self.arena.view(self.a_keys[0], (self.n * self.r, self.in_f))

    def params(self):
        return [self.arena.params[k] for k in self.a_keys + self.b_keys]

    def dropping(self, train: bool) -> bool:
        return train and self.s.lora_dropout > 0.0

    def forward(self, x, train: bool, step_seed: int):
        """(t [M, out_total] = scaling * lora_B(lora_A(dropout(x))) per module block, u [M, n*r])"""
        M, r, R = x.shape[0], self.r, self.n * self.r
        ldx = ops._ld(x)
        u = torch.empty((M, R), dtype=x.dtype, device=x.device)
        if self.dropping(train):
            for m in range(self.n):
                ops.gemm_ex(0, 0, M, r, self.in_f, x, ldx, self.A(m), self.in_f, u[:, m * r:], R,
                            drop_operand=DROP_A, drop_p=self.s.lora_dropout,
                            drop_seed=module_seed(step_seed, self.uid, m))
        else:
            ops.gemm_ex(0, 0, M, R, self.in_f, x, ldx, self.a_stack(), self.in_f, u, R)
        return LoraTerm(self, u), u

    def up_project(self, u):
        """t [M, out_total] = scaling * u_m B_m^T per module block (the unfused addend)"""
        M, r, R = u.shape[0], self.r, self.n * self.r
        t = torch.empty((M, self.out_total), dtype=u.dtype, device=u.device)
        for m in range(self.n):
            ops.gemm_ex(0, 0, M, self.outs[m], r, u[:, m * r:], R, self.B(m), r, t[:, self.offs[m]:], self.out_total,
                        alpha=self.scaling)
        return t

    def b_stack(self):
        return self.arena.view(self.b_keys[0], (self.out_total, self.r))

    def backward(self, dy, x, u, dx, train: bool, step_seed: int):
        """Writes dA / dB into the arena's gradient slots and accumulates the adapters' share of
        dx into dx (dy: [M, out_total] gradient of the group's Linear outputs)."""
        ar = self.arena
        M, r, R = x.shape[0], self.r, self.n * self.r
        ldx, ldy = ops._ld(x), ops._ld(dy)
        du = torch.empty((M, R), dtype=dy.dtype, device=dy.device)
        for m in range(self.n):
            ops.gemm_ex(0, 1, M, r, self.outs[m], dy[:, self.offs[m]:], ldy, self.B(m), r, du[:, m * r:], R,
                        alpha=self.scaling)
            g, beta = ar.grad_slot(self.b_keys[m])
            ops.gemm_ex(1, 1, self.outs[m], r, M, dy[:, self.offs[m]:], ldy, u[:, m * r:], R, g, r,
                        alpha=self.scaling, beta=beta)
        if self.dropping(train):
            p = self.s.lora_dropout
            seeds = [module_seed(step_seed, self.uid, m) for m in range(self.n)]
            # the group's dx contributions in one pass over dx (cullavo_lora_dx, bitwise the
            # per-module products below)
            fused_dx = (LORA_DX_FUSE and dx is not None and dx.dtype == torch.bfloat16 and r == 64
                        and self.n <= 3)
            for m in range(self.n):
                g, beta = ar.grad_slot(self.a_keys[m])
                ops.gemm_ex(1, 1, r, self.in_f, M, du[:, m * r:], R, x, ldx, g, self.in_f, beta=beta,
                            drop_operand=DROP_B, drop_p=p, drop_seed=seeds[m])
                if dx is not None and not fused_dx:
                    ops.gemm_ex(0, 1, M, self.in_f, r, du[:, m * r:], R, self.A(m), self.in_f, dx, ops._ld(dx),
                                beta=1.0, drop_operand=DROP_OUT, drop_p=p, drop_seed=seeds[m])
            if fused_dx:
                ops.lora_dx(du, self.a_stack(), dx, n_mod=self.n, drop_p=p, seeds=seeds)
        else:
            g, beta = ar.grad_slot(self.a_keys[0], (R, self.in_f))
            ar.mark_written(self.a_keys[1:])
            ops.gemm_ex(1, 1, R, self.in_f, M, du, R, x, ldx, g, self.in_f, beta=beta)
            if dx is not None:
                ops.gemm_ex(0, 1, M, self.in_f, R, du, R, self.a_stack(), self.in_f, dx, ops._ld(dx), beta=1.0)
        ar.commit(self.a_keys + self.b_keys)


class NoLora:
    """Stand-in for layers without adapters (keeps the layer Functions branch-free)."""

    def forward(self, x, train, step_seed):
        return None, None

    def backward(self, dy, x, u, dx, train, step_seed):
        return None

    def params(self):
        return []


NO_LORA = NoLora()
