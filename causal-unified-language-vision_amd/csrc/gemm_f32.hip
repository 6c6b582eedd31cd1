// f32-operand GEMM: the parity mode of cullavo_gemm_ex (desc.f32_operands = 1). Every operand
// (A, B, bias, residual, addend, preact, C) is f32 and no intermediate is rounded, so a model
// built on f32 arenas computes the reference's fp32 module chain (tf:llama/modeling_llama.py,
// tf:clip/modeling_clip.py, tf:llava/modeling_llava.py in fp32) with one f32 rounding per
// product: v_mfma_f32_16x16x4_f32 is an exact k-ordered f32 fma chain
// (cdna_hip_programming.md "FP32-input MFMA").
//
// 128x128 tile, 4 waves (2x2, 64x64 each = 4x4 MFMA tiles), BK = 16, operands staged through
// registers into k-major LDS images (both layouts; layout 0 is transposed on the LDS write),
// double-buffered with one barrier per K step. Same epilogue order as the bf16 kernels
// (alpha, output dropout, bias, addend, preact, act, residual, beta). Operand dropout (LoRA)
// is applied while staging, from the same counter hash.
#include "common.h"

namespace {

constexpr int FB = 128, FK = 16, FLD = FB + 4;

struct F32Args {
  const float* A;
  const float* B;
  float* C;
  const float* bias;
  float* preact;
  const float* residual;
  const float* addend;
  int64_t M, N, K, lda, ldb, ldc, ldr, ld_add;
  float alpha, beta;
  int act;
  int drop_mode;
  uint32_t drop_thr;
  float drop_scale;
  uint64_t drop_seed;
};

DEV float act_f32(int act, float x) {
  if (act == CULLAVO_ACT_GELU) return 0.5f * x * (1.f + erff(x * 0.70710678118654752f));
  if (act == CULLAVO_ACT_QUICK_GELU) return x / (1.f + __expf(-1.702f * x));
  return x;
}

// global -> registers for one 128 x 16 operand tile (2 x float4 per thread). Element (i, k)
// of the operand (i = row of C for A / column of C for B). LAYOUT 0: X[i][k]; 1: X[k][i].
template <int LAYOUT>
DEV void f32_load(const float* __restrict__ X, int64_t ld, int64_t i0, int64_t imax, int64_t k0, int64_t K,
                  f32x4 (&r)[2]) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int q = threadIdx.x + 256 * u;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (LAYOUT == 0) {
      const int row = q >> 2, k4 = (q & 3) * 4;
      const int64_t gi = i0 + row;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (gi < imax && k0 + k4 + j < K) v[j] = X[gi * ld + k0 + k4 + j];
    } else {
      const int k = q >> 5, i4 = (q & 31) * 4;
      const int64_t gk = k0 + k;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (gk < K && i0 + i4 + j < imax) v[j] = X[gk * ld + i0 + i4 + j];
    }
    r[u] = v;
  }
}

// LoRA dropout while staging: the operand is x[token][feature]; for A (layout 0) element
// (i, k) = (token i, feature k), for B (layout 1) element (k, i) = (token k, feature i)
template <int LAYOUT>
DEV void f32_drop(const F32Args& p, int64_t i0, int64_t k0, f32x4 (&r)[2]) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int q = threadIdx.x + 256 * u;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int64_t tok, feat;
      if (LAYOUT == 0) { tok = i0 + (q >> 2); feat = k0 + (q & 3) * 4 + j; }
      else { tok = k0 + (q >> 5); feat = i0 + (q & 31) * 4 + j; }
      r[u][j] = drop_keep(p.drop_seed, p.drop_thr, tok, feat) ? r[u][j] * p.drop_scale : 0.f;
    }
  }
}

// registers -> k-major LDS image [FK][FLD]
template <int LAYOUT>
DEV void f32_store(float* img, const f32x4 (&r)[2]) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int q = threadIdx.x + 256 * u;
    if (LAYOUT == 0) {
      const int row = q >> 2, k4 = (q & 3) * 4;
#pragma unroll
      for (int j = 0; j < 4; ++j) img[(k4 + j) * FLD + row] = r[u][j];
    } else {
      const int k = q >> 5, i4 = (q & 31) * 4;
      *reinterpret_cast<f32x4*>(img + k * FLD + i4) = r[u];
    }
  }
}

DEV void f32_epilogue(const F32Args& p, const f32x4& acc, int64_t m, int64_t n) {
  if (m >= p.M) return;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t nn = n + j;
    if (nn >= p.N) return;
    float v = acc[j] * p.alpha;
    if (p.drop_mode == 3) v = drop_keep(p.drop_seed, p.drop_thr, m, nn) ? v * p.drop_scale : 0.f;
    if (p.bias) v += p.bias[nn];
    if (p.addend) v += p.addend[m * p.ld_add + nn];
    if (p.preact) p.preact[m * p.ldc + nn] = v;
    v = act_f32(p.act, v);
    if (p.residual) v += p.residual[m * p.ldr + nn];
    float* cp = p.C + m * p.ldc + nn;
    if (p.beta != 0.f) v += p.beta * *cp;
    *cp = v;
  }
}

template <int AL, int BL, int DROP>
__global__ __launch_bounds__(256) void gemm_f32_k(F32Args p, int tiles_m, int tiles_n) {
  __shared__ __attribute__((aligned(16))) float sA[2][FK * FLD];
  __shared__ __attribute__((aligned(16))) float sB[2][FK * FLD];
  // grouped tile order (8 M-tiles sweep N) for L2 reuse
  const int lid = blockIdx.x;
  const int per_group = 8 * tiles_n;
  const int first_m = (lid / per_group) * 8;
  const int gsize = min(tiles_m - first_m, 8);
  const int64_t m0 = (int64_t)(first_m + (lid % per_group) % gsize) * FB;
  const int64_t n0 = (int64_t)((lid % per_group) / gsize) * FB;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (int)cdiv(p.K, FK);
  f32x4 ra[2], rb[2];
  f32_load<AL>(p.A, p.lda, m0, p.M, 0, p.K, ra);
  f32_load<BL>(p.B, p.ldb, n0, p.N, 0, p.K, rb);
  if (DROP == 1) f32_drop<AL>(p, m0, 0, ra);
  if (DROP == 2) f32_drop<BL>(p, n0, 0, rb);
  f32_store<AL>(sA[0], ra);
  f32_store<BL>(sB[0], rb);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    const int64_t k1 = (int64_t)(kt + 1) * FK;
    if (more) {
      f32_load<AL>(p.A, p.lda, m0, p.M, k1, p.K, ra);
      f32_load<BL>(p.B, p.ldb, n0, p.N, k1, p.K, rb);
    }
    const float* a_img = sA[cur];
    const float* b_img = sB[cur];
#pragma unroll
    for (int ks = 0; ks < FK / 4; ++ks) {
      const int k = ks * 4 + (lane >> 4);
      float fa[4], fb[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        fa[t] = a_img[k * FLD + wm * 64 + t * 16 + (lane & 15)];
        fb[t] = b_img[k * FLD + wn * 64 + t * 16 + (lane & 15)];
      }
      // swapped operands: lane ends with C[m = lane&15 row][n = 4*(lane>>4) + reg]
#pragma unroll
      for (int tm = 0; tm < 4; ++tm)
#pragma unroll
        for (int tn = 0; tn < 4; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x4f32(fb[tn], fa[tm], acc[tm][tn], 0, 0, 0);
    }
    if (more) {
      if (DROP == 1) f32_drop<AL>(p, m0, k1, ra);
      if (DROP == 2) f32_drop<BL>(p, n0, k1, rb);
      f32_store<AL>(sA[cur ^ 1], ra);
      f32_store<BL>(sB[cur ^ 1], rb);
    }
    __syncthreads();
  }
#pragma unroll
  for (int tm = 0; tm < 4; ++tm) {
    const int64_t m = m0 + wm * 64 + tm * 16 + (lane & 15);
#pragma unroll
    for (int tn = 0; tn < 4; ++tn) f32_epilogue(p, acc[tm][tn], m, n0 + wn * 64 + tn * 16 + (lane >> 4) * 4);
  }
}

template <int AL, int BL, int DROP>
int launch_f32(const F32Args& p, hipStream_t s) {
  const int tm = (int)cdiv(p.M, FB), tn = (int)cdiv(p.N, FB);
  gemm_f32_k<AL, BL, DROP><<<tm * tn, 256, 0, s>>>(p, tm, tn);
  return cullavo_check_launch("gemm (f32 operands)");
}

template <int DROP>
int dispatch_f32(const F32Args& p, int al, int bl, hipStream_t s) {
  if (al == 0 && bl == 0) return launch_f32<0, 0, DROP>(p, s);
  if (al == 0 && bl == 1) return launch_f32<0, 1, DROP>(p, s);
  if (al == 1 && bl == 0) return launch_f32<1, 0, DROP>(p, s);
  return launch_f32<1, 1, DROP>(p, s);
}

}  // namespace

// called by gemm_impl (gemm.hip) after the shared argument checks
int cullavo_gemm_f32_impl(const cullavo_gemm_desc& d, hipStream_t s) {
  CV_REQUIRE(d.c_dtype == CULLAVO_DT_F32, CULLAVO_EINVAL, "f32_operands needs c_dtype f32");
  CV_REQUIRE(d.drop_operand != 1 || d.a_layout == 0, CULLAVO_EUNSUPPORTED, "dropout on A needs a_layout 0");
  CV_REQUIRE(d.drop_operand != 2 || d.b_layout == 1, CULLAVO_EUNSUPPORTED, "dropout on B needs b_layout 1");
  if (d.M == 0 || d.N == 0) return CULLAVO_OK;
  CV_REQUIRE(cdiv(d.M, FB) * cdiv(d.N, FB) < (1ll << 31), CULLAVO_EINVAL, "too many tiles");
  F32Args p;
  p.A = (const float*)d.A; p.B = (const float*)d.B; p.C = (float*)d.C;
  p.bias = (const float*)d.bias; p.preact = (float*)d.preact; p.residual = (const float*)d.residual;
  p.addend = (const float*)d.addend;
  p.M = d.M; p.N = d.N; p.K = d.K; p.lda = d.lda; p.ldb = d.ldb; p.ldc = d.ldc; p.ldr = d.ldr;
  p.ld_add = d.ld_addend;
  p.alpha = d.alpha; p.beta = d.beta; p.act = d.act;
  const bool dropping = d.drop_operand != 0 && d.drop_p > 0.f;
  p.drop_mode = dropping ? d.drop_operand : 0;
  p.drop_thr = (uint32_t)(d.drop_p * 65536.0f + 0.5f);
  p.drop_scale = dropping ? 1.f / (1.f - d.drop_p) : 1.f;
  p.drop_seed = d.drop_seed;
  if (p.drop_mode == 1) return dispatch_f32<1>(p, d.a_layout, d.b_layout, s);
  if (p.drop_mode == 2) return dispatch_f32<2>(p, d.a_layout, d.b_layout, s);
  return dispatch_f32<0>(p, d.a_layout, d.b_layout, s);
}
