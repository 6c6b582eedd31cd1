// Shared device helpers for the CuLLaVO gfx950 kernels: bf16 conversion, vector types,
// wave (64-lane) reductions and the C-ABI error plumbing.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include <algorithm>

#include "../../include/cullavo_capi.h"

typedef unsigned short u16;
typedef __attribute__((ext_vector_type(8))) unsigned short u16x8;  // 8 bf16 = 16 B
typedef __attribute__((ext_vector_type(4))) unsigned short u16x4;  // 4 bf16 = 8 B
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;

#define DEV __device__ __forceinline__

DEV float bf2f(u16 v) { return __uint_as_float(((unsigned)v) << 16); }
// round-to-nearest-even through the native type (v_cvt_pk_bf16_f32 on gfx950; NaN stays NaN)
DEV u16 f2bf(float f) { return __builtin_bit_cast(u16, (__bf16)f); }
DEV float round_bf(float f) { return bf2f(f2bf(f)); }

// ---- LoRA dropout mask ------------------------------------------------------------------------
// Counter-based, so the forward (operand staging), dA (operand staging) and dX (GEMM epilogue)
// regenerate the same mask from (seed, token, feature) without storing it. One 32-bit hash per
// (token, feature pair) gives both features a 16-bit uniform (low half: even feature, high half:
// odd); an element is kept iff its 16 bits >= thr16 = round(p * 2^16) (p = 0.05 -> 0.0500031);
// kept values are scaled by 1/(1-p) (nn.Dropout). The per-token part is hashed once per row.
// (Round 1 hashed every element: ~12 ms of the LoRA step went to it, tools/lora_drop_bench.py.)
// tests/test_lora.py restates the hash in numpy (oracle lora_keep_mask) and checks the masks
// bit-exactly.
DEV uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}
DEV uint32_t drop_row(uint64_t seed, int64_t token) {
  return fmix32((uint32_t)seed ^ fmix32((uint32_t)token * 0x9E3779B1u + (uint32_t)(seed >> 32)));
}
DEV uint32_t drop_pair(uint32_t row, int64_t feat) {
  return fmix32(row ^ ((uint32_t)(feat >> 1) * 0x27D4EB2Fu + 0x165667B1u));
}
DEV bool drop_keep(uint64_t seed, uint32_t thr16, int64_t token, int64_t feat) {
  const uint32_t h = drop_pair(drop_row(seed, token), feat);
  return ((feat & 1) ? (h >> 16) : (h & 0xFFFFu)) >= thr16;
}
// kept-element multipliers (scale or 0) of the N consecutive features f0 .. f0+N-1 of one token,
// f0 and N even: one row hash, N/2 pair hashes
template <int N>
DEV void drop_scales(uint64_t seed, uint32_t thr16, float scale, int64_t token, int64_t f0, float (&m)[N]) {
  const uint32_t row = drop_row(seed, token);
#pragma unroll
  for (int j = 0; j < N; j += 2) {
    const uint32_t h = drop_pair(row, f0 + j);
    m[j] = (h & 0xFFFFu) >= thr16 ? scale : 0.f;
    m[j + 1] = (h >> 16) >= thr16 ? scale : 0.f;
  }
}

template <typename T> struct Elt;
template <> struct Elt<u16> {
  static DEV float ld(const u16* p, int64_t i) { return bf2f(p[i]); }
  static DEV void st(u16* p, int64_t i, float v) { p[i] = f2bf(v); }
  static DEV float rnd(float v) { return round_bf(v); }
};
template <> struct Elt<float> {
  static DEV float ld(const float* p, int64_t i) { return p[i]; }
  static DEV void st(float* p, int64_t i, float v) { p[i] = v; }
  static DEV float rnd(float v) { return v; }
};

// load/store 8 consecutive elements as f32
DEV void load8(const u16* p, float* v) {
  u16x8 x = *reinterpret_cast<const u16x8*>(p);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = bf2f(x[j]);
}
DEV void load8(const float* p, float* v) {
  f32x4 a = *reinterpret_cast<const f32x4*>(p);
  f32x4 b = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) { v[j] = a[j]; v[4 + j] = b[j]; }
}
DEV void store8(u16* p, const float* v) {
  u16x8 x;
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = f2bf(v[j]);
  *reinterpret_cast<u16x8*>(p) = x;
}
DEV void store8(float* p, const float* v) {
  f32x4 a, b;
#pragma unroll
  for (int j = 0; j < 4; ++j) { a[j] = v[j]; b[j] = v[4 + j]; }
  *reinterpret_cast<f32x4*>(p) = a;
  *reinterpret_cast<f32x4*>(p + 4) = b;
}

DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
DEV double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ---- host-side error plumbing ------------------------------------------------------------
void cullavo_set_error(const std::string& msg);
int cullavo_check_launch(const char* what);

#define CV_REQUIRE(cond, code, msg)                  \
  do {                                               \
    if (!(cond)) {                                   \
      cullavo_set_error(std::string(__func__) + ": " + (msg)); \
      return (code);                                 \
    }                                                \
  } while (0)

#define CV_STREAM(s) (reinterpret_cast<hipStream_t>(s))

// gemm_f32.hip: cullavo_gemm_ex with f32_operands = 1
int cullavo_gemm_f32_impl(const cullavo_gemm_desc& d, hipStream_t s);

// attn_generic.hip: f32 storage / head dims 16-32 (dispatched from attention.hip)
int cullavo_attn_generic_fwd(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                             void* o, int64_t ldo, float* lse, int B, int H, int Lq, int Lk, int D, float scale,
                             int causal, const int32_t* ks, int dtype, hipStream_t s);
int cullavo_attn_generic_bwd(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                             const void* o, int64_t ldo, const void* dout, int64_t lddo, const float* lse,
                             float* delta, void* dq, int64_t lddq, void* dk, int64_t lddk, void* dv, int64_t lddv,
                             int B, int H, int Lq, int Lk, int D, float scale, int causal, const int32_t* ks,
                             int dtype, hipStream_t s);

__host__ __device__ inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }
