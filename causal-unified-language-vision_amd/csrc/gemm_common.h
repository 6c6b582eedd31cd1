// Shared device helpers of the bf16 MFMA GEMM kernels (gemm.hip, gemm_pp.hip): the kernel
// argument block, LDS image layouts, fragment reads, LDS-DMA staging and the epilogues.
#pragma once
#include "common.h"

namespace cvgemm {


constexpr int BM = 128, BN = 128, BK = 64;
constexpr int kTileBytes = 128 * 64 * 2;  // 16 KiB per operand tile

typedef __attribute__((ext_vector_type(8))) __bf16 frag8;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

struct GemmArgs {
  const u16* A;
  const u16* B;
  void* C;
  const u16* bias;
  u16* preact;
  const u16* residual;
  int64_t M, N, K, lda, ldb, ldc, ldr;
  float alpha, beta;
  int act;
  int tiles_m, tiles_n;
  const u16* addend;  // LoRA term added after bias: v = round(round(alpha*AB + bias) + addend)
  int64_t ld_add;
  int drop_mode;      // 0 none, 1 A operand, 2 B operand (register-staged kernel), 3 output
  uint32_t drop_thr;
  float drop_scale;
  uint64_t drop_seed;
  float* part;        // split-K: f32 partials [gridDim.y][M][N] (register-staged kernel only)
  int kt_per;         // K-tiles per split
  int epi_lds;        // 8-wave kernels: LDS-staged 16-B epilogue (all pointers 16-B aligned)
  int nt_store;       // C written with non-temporal stores (streamed past the caches)
  int sk_dp;          // 8-wave kernels: tiles in the grid (the XCD remap's block count)
  int group_m;        // 8-wave tile order: > 0 groups of group_m M-tiles sweep N; < 0 groups of
                      // -group_m N-tiles sweep M
  int dma_pre;        // 8-wave 256-row kernels: per-lane DMA offsets precomputed, K advance in soffset
  // fused LoRA up-projection (gemm256_k<..., LORA = true>): t = round(lora_scale * u_m B_m^T) for
  // the module m = n / lora_out of each output column, added to round(alpha*acc + bias)
  const u16* lora_u;  // [M, n_mod * 64] (row stride ld_lu): lora_A outputs of the group's modules
  int64_t ld_lu;
  const u16* lora_b;  // [N, 64] row-major: the group's lora_B weights stacked in column order
  int64_t lora_out;   // output columns per module (a multiple of 256)
  float lora_scale;
};

template <typename V>
DEV void st_c(const GemmArgs& p, V* dst, const V& v) {
  if (p.nt_store) __builtin_nontemporal_store(v, dst);
  else *dst = v;
}

// ---- LDS images -----------------------------------------------------------------------------
// layout 0 image: [128 rows][64 k], 16 B chunk c of row r at chunk slot c ^ ((r >> 1) & 7)
DEV int img0_off(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }
// layout 1 image: [64 k][128 rows], 32 B unit u of k-row k at unit slot u ^ swz(k)
DEV int swz1(int k) { return (k & 7) ^ (((k >> 3) & 1) << 2); }
// position of 16-column unit u in k-row k of a ROWS-wide layout-1 image (an involution): the
// XOR swizzle within the first 16 units; the 288-wide image's last two units stay in place (its
// 576-B k-rows already shift by 16 banks per row)
template <int ROWS>
DEV int upos(int u, int k) { return (ROWS == 288 && u >= 16) ? u : (u ^ swz1(k)); }
DEV int img1_off(int k, int unit) { return k * 256 + ((unit ^ swz1(k)) << 5); }

// global -> registers for one 128 x 64 operand tile (4 x 16 B per thread)
template <int LAYOUT>
DEV void load_tile(const u16* __restrict__ X, int64_t ld, int64_t idx0, int64_t idx_max, int64_t k0,
                   int64_t K, u16x8 (&r)[4]) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = t + 256 * i;
    if (LAYOUT == 0) {
      const int row = q >> 3, c = q & 7;
      const int64_t gi = idx0 + row, gk = k0 + c * 8;
      r[i] = (gi < idx_max && gk < K) ? *reinterpret_cast<const u16x8*>(X + gi * ld + gk) : u16x8(0);
    } else {
      const int k = q >> 4, ch = q & 15;
      const int64_t gk = k0 + k, gi = idx0 + ch * 8;
      r[i] = (gk < K && gi < idx_max) ? *reinterpret_cast<const u16x8*>(X + gk * ld + gi) : u16x8(0);
    }
  }
}

template <int LAYOUT>
DEV void store_tile(char* lds, const u16x8 (&r)[4]) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = t + 256 * i;
    int off;
    if (LAYOUT == 0) {
      off = img0_off(q >> 3, q & 7);
    } else {
      const int k = q >> 4, ch = q & 15;
      off = img1_off(k, ch >> 1) + ((ch & 1) << 4);
    }
    *reinterpret_cast<u16x8*>(lds + off) = r[i];
  }
}

// LoRA dropout on a staged operand tile (the operand is the activation x[token][feature]):
// layout 0 element (row gi, col gk) is (token gi, feature gk); layout 1 (k-row gk, col gi) is
// (token gk, feature gi).
template <int LAYOUT>
DEV void drop_tile(const GemmArgs& p, int64_t idx0, int64_t k0, u16x8 (&r)[4]) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = t + 256 * i;
    int64_t tok, f0;
    if (LAYOUT == 0) { tok = idx0 + (q >> 3); f0 = k0 + (q & 7) * 8; }
    else { tok = k0 + (q >> 4); f0 = idx0 + (q & 15) * 8; }
    float ms[8];
    drop_scales<8>(p.drop_seed, p.drop_thr, p.drop_scale, tok, f0, ms);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = bf2f(r[i][j]);
      r[i][j] = ms[j] != 0.f ? f2bf(v * ms[j]) : (u16)0;
    }
  }
}

// fragment X[idx = rbase + (lane&15)][k = ks*32 + 8*(lane>>4) + j], j = 0..7
template <int LAYOUT>
DEV frag8 read_frag(const char* lds, int rbase, int ks, int lane) {
  if (LAYOUT == 0) {
    const int row = rbase + (lane & 15);
    const int c = ks * 4 + (lane >> 4);
    u16x8 v = *reinterpret_cast<const u16x8*>(lds + img0_off(row, c));
    return __builtin_bit_cast(frag8, v);
  } else {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int unit = rbase >> 4;
    s16x4 lo, hi;
    {
      const int k = ks * 32 + 8 * g + q;
      lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + img1_off(k, unit) + 8 * p));
    }
    {
      const int k = ks * 32 + 8 * g + 4 + q;
      hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + img1_off(k, unit) + 8 * p));
    }
    typedef __attribute__((ext_vector_type(8))) short s16x8;
    s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(frag8, v);
  }
}

DEV float act_apply(int act, float x) {
  if (act == CULLAVO_ACT_GELU) return 0.5f * x * (1.f + erff(x * 0.70710678118654752f));  // one op: one rounding
  if (act == CULLAVO_ACT_QUICK_GELU) {
    // CLIP quick_gelu x * sigmoid(1.702 x) (tf:activations.py:117-123) as the reference's bf16
    // tensors evaluate it: the product 1.702 x and the sigmoid each round to bf16, the final
    // product rounds in the store
    // exp and reciprocal by the hardware approximations (v_exp_f32, v_rcp_f32: ~1 ulp in f32),
    // which the bf16 rounding of the sigmoid absorbs except within ~1 ulp of a bf16 tie; the
    // IEEE division sequence made this epilogue a third of the ViT fc1 GEMM
    // (tools/vit_gemm_bench.py)
    const float t = round_bf(1.702f * x);
    const float e = __builtin_amdgcn_exp2f(t * -1.4426950408889634f);
    const float sg = round_bf(__builtin_amdgcn_rcpf(1.f + e));
    return sg * x;
  }
  return x;
}

// quick_gelu of act_apply on 8 values, two at a time: the products and the sum as packed f32
// (v_pk_mul_f32 / v_pk_add_f32) and both bf16 roundings as one v_cvt_pk_bf16_f32 per pair; the
// same operations in the same order as act_apply, so bit-identical (the epilogue of the ViT fc1
// GEMM, where the activation was ~30 % of the GEMM's time, tools/vit_gemm_bench.py)
typedef float f32x2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
DEV f32x2v round_bf2(f32x2v x) {
  const unsigned u = __builtin_bit_cast(unsigned, __builtin_convertvector(x, bf16x2v));
  return f32x2v{__uint_as_float(u << 16), __uint_as_float(u & 0xFFFF0000u)};
}
DEV void quick_gelu8(float (&v)[8]) {
#pragma unroll
  for (int j = 0; j < 8; j += 2) {
    const f32x2v x = {v[j], v[j + 1]};
    const f32x2v t = round_bf2(1.702f * x);
    const f32x2v a = t * -1.4426950408889634f;
    const f32x2v d = 1.f + f32x2v{__builtin_amdgcn_exp2f(a.x), __builtin_amdgcn_exp2f(a.y)};
    const f32x2v sg = round_bf2(f32x2v{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)});
    const f32x2v y = sg * x;
    v[j] = y.x;
    v[j + 1] = y.y;
  }
}

// bijective XCD-aware remap (cdna_hip_programming.md §5 "XCD swizzle must be bijective")
DEV int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

// CULLAVO_ACT_SWIGLU_BWD epilogue for NV consecutive columns: the product is dh = d(silu(g) * u)
// of the SwiGLU, rounded to bf16 as the unfused path stores it; with g = gu[m][n], u = gu[m][F + n]
// (gu = p.residual, F = p.N) it writes dg to C[m][n] and du to C[m][F + n], in the arithmetic of
// swiglu_bwd_k (elementwise.hip) so the fused and unfused paths are bitwise equal.
// the SwiGLU backward's sigmoid: v_rcp_f32 (1 ulp) instead of the IEEE division sequence (~10 VALU
// ops; the SwiGLU-backward dX 1001-1016 -> 1013-1032 TF/s, profiles/r06/gemm/swiglu_rcp_ab.txt);
// elementwise.hip swiglu_bwd_k uses the same expression, so the fused and unfused paths stay bitwise
DEV float sigmoid_rcp(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }

// the arithmetic of one lane's NV columns: dg -> oa, du -> ob (shared by every SwiGLU-backward path)
template <int NV, typename UV>
DEV void swiglu_bwd_math(const float* acc, float alpha, const UV& gv, const UV& uv, UV& oa, UV& ob) {
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const float dv = round_bf(acc[j] * alpha);
    const float g = bf2f(gv[j]), u = bf2f(uv[j]);
    const float sg = sigmoid_rcp(g);
    const float silu = g * sg;
    ob[j] = f2bf(dv * round_bf(silu));
    oa[j] = f2bf(dv * u * sg * (1.f + g * (1.f - sg)));
  }
}

template <int NV>
DEV void swiglu_bwd_store(const GemmArgs& p, const float* acc, int64_t m, int64_t n) {
  typedef __attribute__((ext_vector_type(NV))) unsigned short uv_t;
  const u16* gr = p.residual + m * p.ldr;
  const uv_t gv = *reinterpret_cast<const uv_t*>(gr + n);
  const uv_t uv = *reinterpret_cast<const uv_t*>(gr + p.N + n);
  uv_t oa, ob;
  swiglu_bwd_math<NV>(acc, p.alpha, gv, uv, oa, ob);
  u16* cp = (u16*)p.C + m * p.ldc + n;
  *reinterpret_cast<uv_t*>(cp) = oa;
  *reinterpret_cast<uv_t*>(cp + p.N) = ob;
}

// epilogue for one lane's C[m][n .. n+3] (bias -> preact -> act -> residual -> beta -> store)
template <int CT>
DEV void store4(const GemmArgs& p, const f32x4& acc, int64_t m, int64_t n) {
  if (m >= p.M || n >= p.N) return;
  if (CT == CULLAVO_DT_BF16 && p.act == CULLAVO_ACT_SWIGLU_BWD) {
    const float a[4] = {acc[0], acc[1], acc[2], acc[3]};
    swiglu_bwd_store<4>(p, a, m, n);
    return;
  }
  float v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = acc[j] * p.alpha;
  if (p.drop_mode == 3) {
    float ms[4];
    drop_scales<4>(p.drop_seed, p.drop_thr, p.drop_scale, m, n, ms);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = ms[j] != 0.f ? v[j] * ms[j] : 0.f;
  }
  if (p.bias) {
    const u16x4 bv = *reinterpret_cast<const u16x4*>(p.bias + n);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] += bf2f(bv[j]);
  }
  if (p.addend) {
    const u16x4 av = *reinterpret_cast<const u16x4*>(p.addend + m * p.ld_add + n);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = round_bf(v[j]) + bf2f(av[j]);
  }
  if (p.act != CULLAVO_ACT_NONE || p.preact) {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = round_bf(v[j]);
    if (p.preact) {
      u16x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = f2bf(v[j]);
      *reinterpret_cast<u16x4*>(p.preact + m * p.ldc + n) = o;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = act_apply(p.act, v[j]);
  }
  if (p.residual) {
    const u16x4 rv = *reinterpret_cast<const u16x4*>(p.residual + m * p.ldr + n);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = round_bf(v[j]) + bf2f(rv[j]);
  }
  if (CT == CULLAVO_DT_BF16) {
    u16* cp = (u16*)p.C + m * p.ldc + n;
    if (p.beta != 0.f) {
      const u16x4 old = *reinterpret_cast<const u16x4*>(cp);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] += p.beta * bf2f(old[j]);
    }
    u16x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = f2bf(v[j]);
    st_c(p, reinterpret_cast<u16x4*>(cp), o);
  } else {
    float* cp = (float*)p.C + m * p.ldc + n;
    f32x4 o;
    if (p.beta != 0.f) {
      const f32x4 old = *reinterpret_cast<const f32x4*>(cp);
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = v[j] + p.beta * old[j];
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = v[j];
    }
    st_c(p, reinterpret_cast<f32x4*>(cp), o);
  }
}

// the same epilogue for 8 consecutive columns C[m][n .. n+7] with 16-B accesses (the
// LDS-staged path below; every pointer 16-B aligned and every ld a multiple of 8, see
// lds_epi_ok)
template <int CT>
DEV void store8(const GemmArgs& p, const float (&a)[8], int64_t m, int64_t n) {
  if (m >= p.M || n >= p.N) return;  // N % 8 == 0: the whole group is in range
  if (CT == CULLAVO_DT_BF16 && p.act == CULLAVO_ACT_SWIGLU_BWD) {
    swiglu_bwd_store<8>(p, a, m, n);
    return;
  }
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = a[j] * p.alpha;
  if (p.drop_mode == 3) {
    float ms[8];
    drop_scales<8>(p.drop_seed, p.drop_thr, p.drop_scale, m, n, ms);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = ms[j] != 0.f ? v[j] * ms[j] : 0.f;
  }
  if (p.bias) {
    const u16x8 bv = *reinterpret_cast<const u16x8*>(p.bias + n);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] += bf2f(bv[j]);
  }
  if (p.addend) {
    const u16x8 av = *reinterpret_cast<const u16x8*>(p.addend + m * p.ld_add + n);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = round_bf(v[j]) + bf2f(av[j]);
  }
  if (p.act != CULLAVO_ACT_NONE || p.preact) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = round_bf(v[j]);
    if (p.preact) {
      u16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(v[j]);
      *reinterpret_cast<u16x8*>(p.preact + m * p.ldc + n) = o;
    }
    if (p.act == CULLAVO_ACT_QUICK_GELU) {
      quick_gelu8(v);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = act_apply(p.act, v[j]);
    }
  }
  if (p.residual) {
    const u16x8 rv = *reinterpret_cast<const u16x8*>(p.residual + m * p.ldr + n);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = round_bf(v[j]) + bf2f(rv[j]);
  }
  if (CT == CULLAVO_DT_BF16) {
    u16* cp = (u16*)p.C + m * p.ldc + n;
    if (p.beta != 0.f) {
      const u16x8 old = *reinterpret_cast<const u16x8*>(cp);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += p.beta * bf2f(old[j]);
    }
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(v[j]);
    st_c(p, reinterpret_cast<u16x8*>(cp), o);
  } else {
    float* cp = (float*)p.C + m * p.ldc + n;
    f32x4 o0, o1;
    if (p.beta != 0.f) {
      const f32x4 q0 = *reinterpret_cast<const f32x4*>(cp), q1 = *reinterpret_cast<const f32x4*>(cp + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) { o0[j] = v[j] + p.beta * q0[j]; o1[j] = v[4 + j] + p.beta * q1[j]; }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) { o0[j] = v[j]; o1[j] = v[4 + j]; }
    }
    st_c(p, reinterpret_cast<f32x4*>(cp), o0);
    st_c(p, reinterpret_cast<f32x4*>(cp + 4), o1);
  }
}

// LDS-staged epilogue of the 8-wave kernels (256-column tiles): per row half (wave row wm),
// the owning waves write their f32 accumulators into a [BM/2][256] image (16-B chunk c of row
// r at chunk c ^ (r & 15): conflict-free ds_write_b128), then all 512 threads run store8 on
// 8 contiguous columns each, so every global access is a full-width 16-B access and 32 lanes
// cover one 512-B output row (the per-lane 8-B stores of the MFMA layout touch 16 rows per
// instruction; measured +3-4 % on the whole GEMM, tools/lab/gemm_lab.hip).
// the LDS epilogue's path for this product (lds_epilogue's cases): 0 plain, 1 bias and / or residual,
// 2 activation, 3 SwiGLU backward, 4 the general store8
template <int CT>
DEV int lds_epi_mode(const GemmArgs& p) {
  const bool lean = CT == CULLAVO_DT_BF16 && p.act == CULLAVO_ACT_NONE && p.preact == nullptr &&
                    p.addend == nullptr && p.beta == 0.f && p.drop_mode != 3 && !p.nt_store;
  if (lean && p.bias == nullptr && p.residual == nullptr && !(p.epi_lds & 8)) return 0;
  if (lean && !(p.epi_lds & 4) && !(p.bias == nullptr && p.residual == nullptr)) return 1;
  if (CT == CULLAVO_DT_BF16 && p.act != CULLAVO_ACT_NONE && p.act != CULLAVO_ACT_SWIGLU_BWD && p.preact == nullptr &&
      p.addend == nullptr && p.residual == nullptr && p.beta == 0.f && p.drop_mode != 3 && !p.nt_store &&
      !(p.epi_lds & 16))
    return 2;
  if (CT == CULLAVO_DT_BF16 && p.act == CULLAVO_ACT_SWIGLU_BWD && !(p.epi_lds & 16)) return 3;
  return 4;
}

// one 8-column group of the LDS epilogue by mode (the arithmetic of store8 in every case)
template <int CT>
DEV void lds_store_item(const GemmArgs& p, float (&v)[8], int64_t m, int64_t n, int mode) {
  if (mode == 4) {
    store8<CT>(p, v, m, n);
    return;
  }
  if (m >= p.M || n >= p.N) return;
  if (mode == 3) {
    swiglu_bwd_store<8>(p, v, m, n);
    return;
  }
  float b[8], rs[8];
  if (mode != 0 && p.bias) {
    const u16x8 bv = *reinterpret_cast<const u16x8*>(p.bias + n);
#pragma unroll
    for (int j = 0; j < 8; ++j) b[j] = bf2f(bv[j]);
  }
  if (mode == 1 && p.residual) {
    const u16x8 rv = *reinterpret_cast<const u16x8*>(p.residual + m * p.ldr + n);
#pragma unroll
    for (int j = 0; j < 8; ++j) rs[j] = bf2f(rv[j]);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float x = v[j] * p.alpha;
    if (mode != 0 && p.bias) x += b[j];
    if (mode == 2) x = round_bf(x);
    if (mode == 1 && p.residual) x = round_bf(x) + rs[j];
    v[j] = x;
  }
  if (mode == 2) {
    if (p.act == CULLAVO_ACT_QUICK_GELU) {
      quick_gelu8(v);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = act_apply(p.act, v[j]);
    }
  }
  u16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = f2bf(v[j]);
  *reinterpret_cast<u16x8*>(reinterpret_cast<u16*>(p.C) + m * p.ldc + n) = o;
}

// item i of a half's LDS image: 8 consecutive f32 outputs of one row (thread idx = tid + 512 i:
// row idx >> 5, columns (idx & 31) * 8 ..), and their coordinates
template <int R>
DEV void lds_epi_item(const char* smem, int i, int half, int64_t m0, int64_t n0, float (&v)[8], int64_t& m,
                      int64_t& n) {
  const int idx = threadIdx.x + 512 * i;
  const int r = idx >> 5, pr = idx & 31;
  const int sw = (pr >> 3) & 1;  // odd chunk first for pairs 8-15, 24-31: conflict-free reads
  const int c0 = 2 * pr + sw, c1 = 2 * pr + 1 - sw;
  const char* rowp = smem + r * 1024;
  const f32x4 x0 = *reinterpret_cast<const f32x4*>(rowp + ((c0 ^ (r & 15)) << 4));
  const f32x4 x1 = *reinterpret_cast<const f32x4*>(rowp + ((c1 ^ (r & 15)) << 4));
  const f32x4 lo = sw ? x1 : x0, hi = sw ? x0 : x1;
#pragma unroll
  for (int j = 0; j < 4; ++j) { v[j] = lo[j]; v[4 + j] = hi[j]; }
  m = m0 + half * R + r;
  n = n0 + pr * 8;
}

// SWG: the instantiation for the SwiGLU-backward epilogue only (act 3, bf16; gemm256_k<..., SWG = true>,
// chosen by the host for that act): per row half, every item's g and u rows (16 B each) are loaded
// BEFORE the half's accumulators are staged in LDS, so the loads' latency runs under the staging and
// the barrier, and the items are unrolled (the general path below is a rolled loop whose every item
// waited for its own two dependent loads: the 8704 x 11008 x 4096 dX ran at 1021 against 1274 TF/s
// plain). Same arithmetic as swiglu_bwd_store (swiglu_bwd_math): bitwise.
template <int CT, int BM2, int TMW, int TN>
DEV void lds_epilogue_swiglu(const GemmArgs& p, f32x4 (&acc)[TMW][TN], char* smem, int64_t m0, int64_t n0, int wm,
                             int wn, int lane) {
  constexpr int R = BM2 / 2;
  constexpr int NI = R * 32 / 512;       // items per thread and half: 9 (288 rows) or 8 (256)
  constexpr int NB = NI % 3 == 0 ? 3 : 4;  // items per batch: one batch's loads in flight ahead
  u16x8 gv[NI], uv[NI];
  auto load = [&](int half, int i) {
    const int idx = threadIdx.x + 512 * i;
    const int64_t m = m0 + half * R + (idx >> 5), n = n0 + (idx & 31) * 8;
    if (m < p.M && n < p.N) {
      const u16* gr = p.residual + m * p.ldr + n;
      gv[i] = *reinterpret_cast<const u16x8*>(gr);
      uv[i] = *reinterpret_cast<const u16x8*>(gr + p.N);
    }
  };
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    // the first batch's loads fly under the staging (sched_barriers keep the compiler from hoisting
    // later batches' loads: with the other half's accumulators live, more would spill)
#pragma unroll
    for (int i = 0; i < NB; ++i) load(half, i);
    __builtin_amdgcn_sched_barrier(0);
    if (wm == half) {
#pragma unroll
      for (int tm = 0; tm < TMW; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
          const int r = tm * 16 + (lane & 15);
          const int c = wn * 16 + tn * 4 + (lane >> 4);
          *reinterpret_cast<f32x4*>(smem + r * 1024 + ((c ^ (r & 15)) << 4)) = acc[tm][tn];
        }
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < NI; b += NB) {
      __builtin_amdgcn_sched_barrier(0);
      if (b + NB < NI) {
#pragma unroll
        for (int i = b + NB; i < b + 2 * NB && i < NI; ++i) load(half, i);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = b; i < b + NB; ++i) {
        float v[8];
        int64_t m, n;
        lds_epi_item<R>(smem, i, half, m0, n0, v, m, n);
        if (m < p.M && n < p.N) {
          u16x8 oa, ob;
          swiglu_bwd_math<8>(v, p.alpha, gv[i], uv[i], oa, ob);
          u16* cp = (u16*)p.C + m * p.ldc + n;
          *reinterpret_cast<u16x8*>(cp) = oa;
          *reinterpret_cast<u16x8*>(cp + p.N) = ob;
        }
      }
    }
    __syncthreads();
  }
}

template <int CT, int BM2, int TMW, int TN>
DEV void lds_epilogue(const GemmArgs& p, f32x4 (&acc)[TMW][TN], char* smem, int64_t m0, int64_t n0, int wm,
                      int wn, int lane) {
  static_assert(TN == 4, "256-column tiles");
  constexpr int R = BM2 / 2;
  // plain bf16 outputs (no bias / addend / activation / residual / beta / output dropout / nt: the
  // q|k|v, gate|up and lm_head products, every dX without a residual and every dW): store8's
  // arithmetic reduces to o = bf16(alpha * acc), written by a lean loop. The general store8 path
  // (runtime-checked epilogue options per 8 columns) measured ~1/4 of a K = 1024 product and ~1/10
  // of a K = 4096 one (tools/lab/gemm256p_lab.hip, profiles/r05/gemm/persistent_lab.txt).
  // bias_res: the same with an optional bias and / or residual (the o_proj / down_proj forward,
  // the ViT's biased products): store8's v = alpha acc + bias, then bf16(bf16(v) + residual)
  // (epi_lds bits 2 / 3: A/B switches that send these cases to the general path)
  const bool lean = CT == CULLAVO_DT_BF16 && p.act == CULLAVO_ACT_NONE && p.preact == nullptr &&
                    p.addend == nullptr && p.beta == 0.f && p.drop_mode != 3 && !p.nt_store;
  const bool plain = lean && p.bias == nullptr && p.residual == nullptr && !(p.epi_lds & 8);
  const bool bias_res = lean && !plain && !(p.epi_lds & 4);
  // (unrolled activation / SwiGLU-backward paths here measured a slower 7B step: every 8-wave
  // kernel carried their code -- the persistent forward kernel has them per instantiation)
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    if (wm == half) {
#pragma unroll
      for (int tm = 0; tm < TMW; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
          const int r = tm * 16 + (lane & 15);
          const int c = wn * 16 + tn * 4 + (lane >> 4);
          *reinterpret_cast<f32x4*>(smem + r * 1024 + ((c ^ (r & 15)) << 4)) = acc[tm][tn];
        }
    }
    __syncthreads();
    if (plain) {  // two versions of the loop, chosen once (uniform)
#pragma unroll
      for (int i = 0; i < R * 32 / 512; ++i) {
        float v[8];
        int64_t m, n;
        lds_epi_item<R>(smem, i, half, m0, n0, v, m, n);
        if (m < p.M && n < p.N) {
          u16x8 o;
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = f2bf(v[j] * p.alpha);
          *reinterpret_cast<u16x8*>(reinterpret_cast<u16*>(p.C) + m * p.ldc + n) = o;
        }
      }
    } else if (bias_res) {
#pragma unroll
      for (int i = 0; i < R * 32 / 512; ++i) {
        float v[8];
        int64_t m, n;
        lds_epi_item<R>(smem, i, half, m0, n0, v, m, n);
        if (m < p.M && n < p.N) {
          float b[8], rs[8];
          if (p.bias) {
            const u16x8 bv = *reinterpret_cast<const u16x8*>(p.bias + n);
#pragma unroll
            for (int j = 0; j < 8; ++j) b[j] = bf2f(bv[j]);
          }
          if (p.residual) {
            const u16x8 rv = *reinterpret_cast<const u16x8*>(p.residual + m * p.ldr + n);
#pragma unroll
            for (int j = 0; j < 8; ++j) rs[j] = bf2f(rv[j]);
          }
          u16x8 o;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float x = v[j] * p.alpha;
            if (p.bias) x += b[j];
            if (p.residual) x = round_bf(x) + rs[j];
            o[j] = f2bf(x);
          }
          *reinterpret_cast<u16x8*>(reinterpret_cast<u16*>(p.C) + m * p.ldc + n) = o;
        }
      }
    } else {  // rolled: one copy of the general store8 per half keeps the kernel's code small
#pragma unroll 1
      for (int i = 0; i < R * 32 / 512; ++i) {
        float v[8];
        int64_t m, n;
        lds_epi_item<R>(smem, i, half, m0, n0, v, m, n);
        store8<CT>(p, v, m, n);
      }
    }
    __syncthreads();
  }
}

// ============================================================================================
// Direct epilogue (round 6): the tile's C straight from the accumulators, no LDS round trip
// ============================================================================================
// In the 16x16 MFMA layout a lane holds 4 consecutive columns of one row per (tm, tn). Packed to
// bf16 (two dwords per tile) and swapped with v_permlane16_swap (rows 1 / 3 of the first operand <->
// rows 0 / 2 of the second, 16-lane rows) between the tiles tn = 2 pr and 2 pr + 1, each lane holds 8
// consecutive columns: lane group g = lane >> 4 has tile 2 pr + (g & 1), columns 8 (g >> 1) .. + 7.
// So a wave stores its 16 x 64 block of one tm as two 16-B stores per lane (rows of 2 x 32 B), with
// no ds_write / ds_read / barrier. Lab (tools/lab/gemm_hc_lab.hip, profiles/r06/gemm/hc_lab.txt):
// 2-6 % faster than the LDS-staged epilogue in the persistent kernel at equal results.
// The stores are buffer stores on C's descriptor: an out-of-range row or column gets an offset past
// num_records and is dropped, so every wave always issues exactly 2 TMW store instructions (the
// persistent kernel counts them in its vmcnt). MODE: 0 plain, 1 bias and / or residual, 2 activation
// (after an optional bias) -- lds_epi_mode's cases 0-2, in store8's arithmetic (bitwise).
typedef __attribute__((ext_vector_type(4))) unsigned u32x4e;

DEV unsigned pk_bf2(float a, float b) { return (unsigned)f2bf(a) | ((unsigned)f2bf(b) << 16); }

template <int MODE, int TMW>
DEV void direct_epilogue(const GemmArgs& p, const f32x4 (&acc)[TMW][4], __amdgpu_buffer_rsrc_t rc, int64_t wm0,
                         int64_t wn0, int lane) {
  const int g = lane >> 4;
  float bv[4][4];
#pragma unroll
  for (int tn = 0; tn < 4; ++tn)
#pragma unroll
    for (int j = 0; j < 4; ++j) bv[tn][j] = 0.f;
  if (MODE != 0 && p.bias) {
#pragma unroll
    for (int tn = 0; tn < 4; ++tn) {
      const int64_t n = wn0 + tn * 16 + g * 4;
      if (n < p.N) {
        const u16x4 b4 = *reinterpret_cast<const u16x4*>(p.bias + n);
#pragma unroll
        for (int j = 0; j < 4; ++j) bv[tn][j] = bf2f(b4[j]);
      }
    }
  }
  const bool res = MODE == 1 && p.residual != nullptr;
  // this lane's chunk column (after the swap) for pair pr: wn0 + (2 pr + (g & 1)) * 16 + (g >> 1) * 8
  const int64_t nc0 = wn0 + (g & 1) * 16 + (g >> 1) * 8;
  // every residual chunk of the wave loaded before the first store (vmcnt retires in issue order,
  // so a load issued after a store would wait for that store too: per 16-row group, a store-drain
  // latency); buffer loads on the residual's own descriptor (out-of-range chunks read as zeros and
  // are not stored), one 32-bit offset each
  const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)p.residual, (short)0, res ? (int)(((p.M - 1) * p.ldr + p.N) * 2) : 0, 0x00020000);
  auto res_load = [&](int tm, u16x8 (&r)[2]) {
    const int64_t m = wm0 + tm * 16 + (lane & 15);
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      const int64_t n = nc0 + pr * 32;
      const unsigned off = (m < p.M && n < p.N) ? (unsigned)((m * p.ldr + n) * 2) : 0x80000000u;
      r[pr] = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(rr, off, 0, 0));
    }
  };
  u16x8 rall[TMW][2];
  if (res) {
#pragma unroll
    for (int tm = 0; tm < TMW; ++tm) res_load(tm, rall[tm]);
  }
  __builtin_amdgcn_sched_barrier(0);  // every residual load issued before the first store
#pragma unroll
  for (int tm = 0; tm < TMW; ++tm) {
    const int64_t m = wm0 + tm * 16 + (lane & 15);
    u16x8 rv[2];
    if (res) {  // this tm's two residual chunks (same rows / columns as the stores below)
      rv[0] = rall[tm][0];
      rv[1] = rall[tm][1];
    }
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      float v[8];  // this lane's pre-swap values: tile 2 pr columns 0-3, then tile 2 pr + 1
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float x = acc[tm][2 * pr + h][j] * p.alpha;
          if (MODE != 0) x += bv[2 * pr + h][j];
          v[h * 4 + j] = x;
        }
      if (MODE == 2) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = round_bf(v[j]);
        if (p.act == CULLAVO_ACT_QUICK_GELU) {
          quick_gelu8(v);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = act_apply(p.act, v[j]);
        }
      }
      unsigned p0 = pk_bf2(v[0], v[1]), p1 = pk_bf2(v[2], v[3]);
      unsigned q0 = pk_bf2(v[4], v[5]), q1 = pk_bf2(v[6], v[7]);
      const auto s0 = __builtin_amdgcn_permlane16_swap(p0, q0, false, false);
      const auto s1 = __builtin_amdgcn_permlane16_swap(p1, q1, false, false);
      u32x4e o = u32x4e{s0[0], s1[0], s0[1], s1[1]};
      const int64_t n = nc0 + pr * 32;
      const bool in = m < p.M && n < p.N;
      if (res) {  // store8's round(v) + residual, rounded once more
        u16x8 w = __builtin_bit_cast(u16x8, o);
#pragma unroll
        for (int j = 0; j < 8; ++j) w[j] = f2bf(bf2f(w[j]) + (in ? bf2f(rv[pr][j]) : 0.f));
        o = __builtin_bit_cast(u32x4e, w);
      }
      const unsigned off = in ? (unsigned)((m * p.ldc + n) * 2) : 0x80000000u;
      __builtin_amdgcn_raw_buffer_store_b128(o, rc, off, 0, 0);
    }
  }
}

// ============================================================================================
// 256-row tile, 8 waves, operands streamed by LDS-DMA (buffer_load ... lds)
// ============================================================================================
// Every 1 KiB LDS-DMA wave-instruction writes lane-linearly, so the XOR-swizzled LDS images
// above are produced by permuting each lane's SOURCE address (cdna_hip_programming.md rule
// 21). Out-of-range rows / K tails are zero-filled by the buffer range check: such lanes get
// an offset past num_records.
constexpr unsigned kOOB = 0x7FFFFFF0u;

typedef __attribute__((address_space(3))) void lds_void;

DEV __amdgpu_buffer_rsrc_t make_rsrc(const u16* base, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)bytes, 0x00020000);
}

// fill one [ROWS][64] (layout 0) or [64][ROWS] (layout 1) operand image; NW waves share it
template <int LAYOUT, int ROWS, int NW>
DEV void dma_tile(__amdgpu_buffer_rsrc_t rsrc, int64_t ld, int64_t idx0, int64_t idx_max, int64_t k0, int64_t K,
                  char* lds, int wave, int lane) {
  if (LAYOUT == 0) {
    constexpr int kPieces = ROWS / 8;  // 8 rows of 128 B per 1 KiB piece
#pragma unroll
    for (int i = 0; i < (kPieces + NW - 1) / NW; ++i) {
      const int pc = wave + NW * i;
      if (kPieces % NW != 0 && pc >= kPieces) break;  // 288 rows = 36 pieces over 8 waves (wave-uniform)
      const int row = pc * 8 + (lane >> 3);
      const int chunk = (lane & 7) ^ ((row >> 1) & 7);
      const int64_t gi = idx0 + row, gk = k0 + chunk * 8;
      const unsigned off = (gi < idx_max && gk < K) ? (unsigned)((gi * ld + gk) * 2) : kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)(lds + pc * 1024), 16, off, 0, 0, 0);
    }
  } else {
    constexpr int RB = ROWS * 2;            // bytes per k-row of the image
    constexpr int kPieces = 64 * RB / 1024;
#pragma unroll
    for (int i = 0; i < (kPieces + NW - 1) / NW; ++i) {
      const int pc = wave + NW * i;
      if (kPieces % NW != 0 && pc >= kPieces) break;  // wave-uniform
      const int byte = pc * 1024 + lane * 16;
      const int k = byte / RB, b = byte % RB;
      const int unit = upos<ROWS>(b >> 5, k), half = (b >> 4) & 1;
      const int64_t gk = k0 + k, gi = idx0 + unit * 16 + half * 8;
      const unsigned off = (gk < K && gi < idx_max) ? (unsigned)((gk * ld + gi) * 2) : kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)(lds + pc * 1024), 16, off, 0, 0, 0);
    }
  }
}

// Same pieces with the per-lane source offsets computed once per tile (dma_prep) and the K
// advance passed as the instruction's scalar offset (dma_issue): a K-tile's issue is then one
// m0 write + one buffer_load per piece instead of 64-bit address math and exec-masked range
// selects per piece. Out-of-range rows get kOOBp, which stays past num_records with any K
// advance added. Layout 1 needs no K-range check (rows k >= K lie past the buffer's extent,
// (K-1)*ld + idx_max, as ld >= idx_max); layout 0 needs full K-tiles (gk < K), so the caller
// uses it only when K % 64 == 0 for every layout-0 operand.
constexpr unsigned kOOBp = 0x80000000u;

// pieces per loader wave (ROWS / 8 of them over NW waves; 288 rows over 8 waves: 5 or 4)
template <int ROWS, int NW>
constexpr int dma_per() { return (ROWS / 8 + NW - 1) / NW; }

template <int LAYOUT, int ROWS, int NW>
DEV void dma_prep(int64_t ld, int64_t idx0, int64_t idx_max, int wave, int lane, unsigned (&vo)[dma_per<ROWS, NW>()]) {
#pragma unroll
  for (int i = 0; i < dma_per<ROWS, NW>(); ++i) {
    const int pc = wave + NW * i;
    int64_t gi, rel;
    if (LAYOUT == 0) {
      const int row = pc * 8 + (lane >> 3);
      const int chunk = (lane & 7) ^ ((row >> 1) & 7);
      gi = idx0 + row;
      rel = gi * ld + chunk * 8;
    } else {
      constexpr int RB = ROWS * 2;
      const int byte = pc * 1024 + lane * 16;
      const int k = byte / RB, b = byte % RB;
      const int unit = upos<ROWS>(b >> 5, k), half = (b >> 4) & 1;
      gi = idx0 + unit * 16 + half * 8;
      rel = k * ld + gi;
    }
    vo[i] = gi < idx_max ? (unsigned)(rel * 2) : kOOBp;
  }
}

template <int ROWS, int NW>
DEV void dma_issue(__amdgpu_buffer_rsrc_t rsrc, const unsigned* vo, int soff, char* lds, int wave) {
#pragma unroll
  for (int i = 0; i < dma_per<ROWS, NW>(); ++i) {
    if ((ROWS / 8) % NW != 0 && wave + NW * i >= ROWS / 8) break;  // wave-uniform
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)(lds + (wave + NW * i) * 1024), 16, vo[i], soff, 0, 0);
  }
}

// scalar byte offset of K-tile origin k0 for an operand of layout L
template <int L>
DEV int dma_soff(int64_t k0, int64_t ld) { return (int)(L == 0 ? k0 * 2 : k0 * ld * 2); }

template <int ROWS>
DEV int img1w_off(int k, int unit) { return k * (ROWS * 2) + (upos<ROWS>(unit, k) << 5); }

// Transposed fragment reads issued by inline asm. The ds_read_tr16 builtin carries no
// memory-operand info, so hipcc (ROCm 7.2) assumes it may alias the in-flight LDS-DMA of the
// next stage and waits vmcnt(0) before it, serialising the prefetch (measured: the (0,1)
// and (1,1) kernels lost 25-45 % to it). The asm reads are invisible to the compiler's
// counters: tr_issue() only issues, tr_wait() (ONE s_waitcnt lgkmcnt(0) that ties the
// destination registers) must run before any consumer (cdna_hip_programming.md §5.7 item 1,
// form (ii) + rule 18's sched_barrier). Older compiler-issued LDS reads are also retired by
// that wait, and extra younger asm reads only make the compiler's own counted waits stricter.
DEV unsigned lds_addr(const char* p) {
  return (unsigned)(uintptr_t)(__attribute__((address_space(3))) const char*)p;
}

template <int ROWS>
DEV void tr_issue(const char* lds, int rbase, int ks, int lane, s16x4& lo, s16x4& hi) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int unit = rbase >> 4;
  const int k1 = ks * 32 + 8 * g + q;
  const unsigned a0 = lds_addr(lds + img1w_off<ROWS>(k1, unit) + 8 * p);
  const unsigned a1 = lds_addr(lds + img1w_off<ROWS>(k1 + 4, unit) + 8 * p);
  asm volatile("ds_read_b64_tr_b16 %0, %2\n\tds_read_b64_tr_b16 %1, %3"
               : "=&v"(lo), "=&v"(hi)
               : "v"(a0), "v"(a1)
               : "memory");
}

DEV frag8 tr_join(const s16x4& lo, const s16x4& hi) {
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(frag8, v);
}

// wait for every outstanding LDS read and tie up to 4 fragment pairs (rule 18 fence after)
DEV void tr_wait4(s16x4& a, s16x4& b, s16x4& c, s16x4& d, s16x4& e, s16x4& f, s16x4& g, s16x4& h) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h)
               :: "memory");
}

template <int N>
DEV void tie_all(s16x4 (&lo)[N], s16x4 (&hi)[N]) {
  s16x4 d0 = {}, d1 = {}, d2 = {}, d3 = {}, d4 = {}, d5 = {};
#pragma unroll
  for (int i = 0; i < N; i += 4) {
    if (i + 3 < N) tr_wait4(lo[i], hi[i], lo[i + 1], hi[i + 1], lo[i + 2], hi[i + 2], lo[i + 3], hi[i + 3]);
    else if (i + 1 < N) tr_wait4(lo[i], hi[i], lo[i + 1], hi[i + 1], d0, d1, d2, d3);
    else tr_wait4(lo[i], hi[i], d0, d1, d2, d3, d4, d5);
  }
}

// fragment X[idx = rbase + (lane&15)][k = ks*32 + 8*(lane>>4) + j] from a ROWS-wide image
template <int LAYOUT, int ROWS>
DEV frag8 read_frag_w(const char* lds, int rbase, int ks, int lane) {
  if (LAYOUT == 0) return read_frag<0>(lds, rbase, ks, lane);
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int unit = rbase >> 4;
  const int k1 = ks * 32 + 8 * g + q;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + img1w_off<ROWS>(k1, unit) + 8 * p));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lds + img1w_off<ROWS>(k1 + 4, unit) + 8 * p));
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(frag8, v);
}

// one K-tile of MFMAs from the LDS stage at cur (both 32-wide K halves)
template <int AL, int BL, int BM2, int BN, int TMW, int TN>
DEV void tile_mfma(const char* cur_c, int wm, int wn, int lane, f32x4 (&acc)[TMW][TN]) {
  constexpr int TILE_A = BM2 * BK * 2;
  constexpr int WN_COLS = BN / 4;
  char* cur = const_cast<char*>(cur_c);
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    frag8 fb[TN];
    s16x4 blo[TN], bhi[TN], alo[TMW], ahi[TMW];
    if constexpr (BL == 1) {
#pragma unroll
      for (int t = 0; t < TN; ++t) tr_issue<BN>(cur + TILE_A, wn * WN_COLS + t * 16, ks, lane, blo[t], bhi[t]);
    }
    if constexpr (AL == 1) {
#pragma unroll
      for (int tm = 0; tm < TMW; ++tm) tr_issue<BM2>(cur, wm * (BM2 / 2) + tm * 16, ks, lane, alo[tm], ahi[tm]);
    }
    if constexpr (BL == 1) tie_all<TN>(blo, bhi);
    if constexpr (AL == 1) tie_all<TMW>(alo, ahi);
    if constexpr (AL == 1 || BL == 1) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < TN; ++t)
      fb[t] = BL == 1 ? tr_join(blo[t], bhi[t]) : read_frag<0>(cur + TILE_A, wn * WN_COLS + t * 16, ks, lane);
#pragma unroll
    for (int tm = 0; tm < TMW; ++tm) {
      const frag8 fa = AL == 1 ? tr_join(alo[tm], ahi[tm]) : read_frag<0>(cur, wm * (BM2 / 2) + tm * 16, ks, lane);
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
        acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[tn], fa, acc[tm][tn], 0, 0, 0);
    }
  }
}

// LDR selects which waves stage the next K-tile: 0 = all eight (each wave issues its share of
// LDS-DMA pieces before its MFMAs, so both waves of a SIMD stall on DMA issue together);
// 1 = waves 0-3 only, 2 = waves 4-7 only (one loader per SIMD: its DMA issue runs beside the
// partner wave's MFMAs instead of beside nothing).
// One tile's K-tiles [kb, ke) into acc (zeroed here): LDS-DMA double buffer, one barrier per
// K-tile, the MFMA loop of the 8-wave kernels (shared by the data-parallel and stream-K kernels)
// the fused LoRA's operand tiles (module m = n0 / lora_out): u rows m0.. at column block 64 m and
// lora_B rows n0.., as a 64-deep layout-0 A / B image pair at lds (all eight waves issue)
template <int BM2, int BN>
DEV void lora_stage(const GemmArgs& p, int64_t m0, int64_t n0, char* lds, int wave, int lane) {
  const int64_t mod = n0 / p.lora_out;
  const __amdgpu_buffer_rsrc_t ru = make_rsrc(p.lora_u + mod * 64, ((p.M - 1) * p.ld_lu + 64) * 2);
  const __amdgpu_buffer_rsrc_t rbl = make_rsrc(p.lora_b, ((p.N - 1) * 64 + 64) * 2);
  dma_tile<0, BM2, 8>(ru, p.ld_lu, m0, p.M, 0, 64, lds, wave, lane);
  dma_tile<0, BN, 8>(rbl, 64, n0, p.N, 0, 64, lds + BM2 * BK * 2, wave, lane);
}

// LPF (the fused-LoRA kernels, gemm.hip lora_fuse): the last K-tile's iteration stages the
// adapters' u rows and lora_B rows (a 64-deep layout-0 tile pair) into the stage it frees, so they
// land under the last MFMAs; returns that stage's offset (-1 when not staged)
template <int AL, int BL, int BM2, int BN, int LDR, int TMW, int TN, bool LPF = false>
DEV int tile_k_range(const GemmArgs& p, __amdgpu_buffer_rsrc_t ra, __amdgpu_buffer_rsrc_t rb, int64_t m0,
                     int64_t n0, int kb, int ke, char* smem, int wave, int lane, f32x4 (&acc)[TMW][TN]) {
  constexpr int TILE_A = BM2 * BK * 2;
  constexpr int TILE_B = BN * BK * 2;
  constexpr int STAGE = TILE_A + TILE_B;
  const int wm = wave >> 2, wn = wave & 3;
#pragma unroll
  for (int i = 0; i < TMW; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  dma_tile<AL, BM2, 8>(ra, p.lda, m0, p.M, (int64_t)kb * BK, p.K, smem, wave, lane);
  dma_tile<BL, BN, 8>(rb, p.ldb, n0, p.N, (int64_t)kb * BK, p.K, smem + TILE_A, wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  if (p.dma_pre) {
    constexpr int NWL = LDR == 0 ? 8 : 4;
    const int lw = LDR == 0 ? wave : (wave & 3);
    const bool loader = LDR == 0 || (LDR == 1 ? wave < 4 : wave >= 4);
    unsigned va[dma_per<BM2, NWL>()], vb[dma_per<BN, NWL>()];
    dma_prep<AL, BM2, NWL>(p.lda, m0, p.M, lw, lane, va);
    dma_prep<BL, BN, NWL>(p.ldb, n0, p.N, lw, lane, vb);
    for (int kt = kb; kt < ke; ++kt) {
      char* cur = smem + ((kt - kb) & 1) * STAGE;
      char* nxt = smem + ((kt - kb + 1) & 1) * STAGE;
      const int64_t k1 = (int64_t)(kt + 1) * BK;
      if (kt + 1 < ke && loader) {
        dma_issue<BM2, NWL>(ra, va, dma_soff<AL>(k1, p.lda), nxt, lw);
        dma_issue<BN, NWL>(rb, vb, dma_soff<BL>(k1, p.ldb), nxt + TILE_A, lw);
      }
      if constexpr (LPF) {
        if (kt + 1 == ke) lora_stage<BM2, BN>(p, m0, n0, nxt, wave, lane);
      }
      tile_mfma<AL, BL, BM2, BN, TMW, TN>(cur, wm, wn, lane, acc);
      // every DMA of tile kt+1 landed (raw s_barrier: the compiler emits no extra wait)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return LPF ? (int)(((ke - kb) & 1) * STAGE) : -1;
  }

  for (int kt = kb; kt < ke; ++kt) {
    char* cur = smem + ((kt - kb) & 1) * STAGE;
    const bool more = kt + 1 < ke;
    char* nxt = smem + ((kt - kb + 1) & 1) * STAGE;
    const int64_t k1 = (int64_t)(kt + 1) * BK;
    // next K-tile's LDS-DMA pieces, all issued before this tile's MFMAs (issuing them one by
    // one between MFMA groups measured 5-15 % slower, profiles/r01/gemm_8phase.md)
    if (more) {
      if constexpr (LDR == 0) {
        dma_tile<AL, BM2, 8>(ra, p.lda, m0, p.M, k1, p.K, nxt, wave, lane);
        dma_tile<BL, BN, 8>(rb, p.ldb, n0, p.N, k1, p.K, nxt + TILE_A, wave, lane);
      } else {
        const bool loader = LDR == 1 ? wave < 4 : wave >= 4;
        if (loader) {
          const int lw = wave & 3;
          dma_tile<AL, BM2, 4>(ra, p.lda, m0, p.M, k1, p.K, nxt, lw, lane);
          dma_tile<BL, BN, 4>(rb, p.ldb, n0, p.N, k1, p.K, nxt + TILE_A, lw, lane);
        }
      }
    }
    tile_mfma<AL, BL, BM2, BN, TMW, TN>(cur, wm, wn, lane, acc);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  return -1;
}

// grouped, XCD-friendly tile order: virtual tile index -> (m0, n0)
template <int BM2, int BN>
DEV void tile_origin(const GemmArgs& p, int lid, int64_t& m0, int64_t& n0) {
  if (p.group_m < 0) {
    const int gn = -p.group_m;
    const int per_group = gn * p.tiles_m;
    const int group = lid / per_group;
    const int first_n = group * gn;
    const int gsize = min(p.tiles_n - first_n, gn);
    n0 = (int64_t)(first_n + (lid % per_group) % gsize) * BN;
    m0 = (int64_t)((lid % per_group) / gsize) * BM2;
    return;
  }
  const int gm = p.group_m;
  const int per_group = gm * p.tiles_n;
  const int group = lid / per_group;
  const int first_m = group * gm;
  const int gsize = min(p.tiles_m - first_m, gm);
  m0 = (int64_t)(first_m + (lid % per_group) % gsize) * BM2;
  n0 = (int64_t)((lid % per_group) / gsize) * BN;
}

}  // namespace cvgemm
