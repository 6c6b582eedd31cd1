// Flash attention for the shapes the MFMA kernels of attention.hip do not take: f32 storage
// (the f32 parity mode, SURVEY.md §7 "Hard parts: parity tolerance") and head dims 16 / 32
// (BASELINE config 1: ViT 64/4, LM 128/4). Same contract as cullavo_attn_fwd / _bwd
// (tf:llama/modeling_llama.py:191-214 eager attention with an f32 softmax,
// tf:clip/modeling_clip.py:280-336): lse in natural log, fully masked rows -> zero output and
// lse = +inf, kv_start masks left padding.
//
// Arithmetic is f32 on the VALU with operands staged in LDS (64 keys per block): these shapes
// are test / tiny-model sizes, where the exact f32 chain matters and the FLOPs do not. The
// backward recomputes P from lse (no stored probabilities): delta = rowsum(dO*O), one kernel
// for dK/dV (a workgroup per 64-key block, query blocks of 32 streamed) and one for dQ.
#include "common.h"

namespace {

constexpr int KB = 64;   // keys per block
constexpr int QF = 64;   // query rows per forward / dQ workgroup
constexpr int QB = 32;   // query rows per dK/dV inner block

template <typename T>
DEV void stage_rows(float* dst, int ld_dst, const T* src, int64_t ld_src, int64_t row0, int nrows_valid, int nrows,
                    int D) {
  for (int idx = threadIdx.x; idx < nrows * D; idx += 256) {
    const int r = idx / D, c = idx - r * D;
    dst[r * ld_dst + c] = r < nrows_valid ? Elt<T>::ld(src, (row0 + r) * ld_src + c) : 0.f;
  }
}

DEV bool visible(int64_t qg, int64_t jg, int Lk, int ks, bool causal) {
  return jg < Lk && jg >= ks && (!causal || jg <= qg);
}

// ---- forward -----------------------------------------------------------------------------------
// thread t: query row r = t >> 2, keys j = part + 4 i (i < 16), output columns part + 4 c
template <typename T, int D>
__global__ __launch_bounds__(256) void attn_gen_fwd_k(const T* __restrict__ Q, int64_t ldq, const T* __restrict__ K,
                                                      int64_t ldk, const T* __restrict__ V, int64_t ldv,
                                                      T* __restrict__ O, int64_t ldo, float* __restrict__ LSE, int H,
                                                      int Lq, int Lk, float scale, int causal,
                                                      const int32_t* __restrict__ kv_start) {
  constexpr int LD = D + 1;
  extern __shared__ float sm[];
  float* sQ = sm;
  float* sK = sQ + QF * LD;
  float* sV = sK + KB * LD;
  float* sP = sV + KB * LD;  // [QF][KB + 1]
  const int nqb = (int)cdiv(Lq, QF);
  const int qb = blockIdx.x % nqb, h = (blockIdx.x / nqb) % H, b = blockIdx.x / (nqb * H);
  const int q0 = qb * QF;
  const int t = threadIdx.x, r = t >> 2, part = t & 3;
  const int ks = kv_start ? kv_start[b] : 0;
  const int64_t qg = q0 + r;
  stage_rows<T>(sQ, LD, Q + h * D, ldq, (int64_t)b * Lq + q0, min(QF, Lq - q0), QF, D);
  float m = -INFINITY, l = 0.f;
  float o[D / 4];
#pragma unroll
  for (int c = 0; c < D / 4; ++c) o[c] = 0.f;
  const int kend = causal ? min(Lk, q0 + QF) : Lk;
  for (int k0 = 0; k0 < kend; k0 += KB) {
    __syncthreads();
    stage_rows<T>(sK, LD, K + h * D, ldk, (int64_t)b * Lk + k0, min(KB, Lk - k0), KB, D);
    stage_rows<T>(sV, LD, V + h * D, ldv, (int64_t)b * Lk + k0, min(KB, Lk - k0), KB, D);
    __syncthreads();
    float s[KB / 4];
    float bmax = -INFINITY;
#pragma unroll
    for (int i = 0; i < KB / 4; ++i) {
      const int j = part + 4 * i;
      float acc = 0.f;
      for (int d = 0; d < D; ++d) acc = fmaf(sQ[r * LD + d], sK[j * LD + d], acc);
      s[i] = visible(qg, k0 + j, Lk, ks, causal) && qg < Lq ? acc * scale : -INFINITY;
      bmax = fmaxf(bmax, s[i]);
    }
    bmax = fmaxf(bmax, __shfl_xor(bmax, 1, 64));
    bmax = fmaxf(bmax, __shfl_xor(bmax, 2, 64));
    const float mnew = fmaxf(m, bmax);
    const float alpha = mnew == -INFINITY ? 1.f : __expf(m - mnew);
    float psum = 0.f;
#pragma unroll
    for (int i = 0; i < KB / 4; ++i) {
      const float p = s[i] == -INFINITY ? 0.f : __expf(s[i] - mnew);
      sP[r * (KB + 1) + part + 4 * i] = p;
      psum += p;
    }
    psum += __shfl_xor(psum, 1, 64);
    psum += __shfl_xor(psum, 2, 64);
    l = l * alpha + psum;
    m = mnew;
    __syncthreads();
#pragma unroll
    for (int c = 0; c < D / 4; ++c) o[c] *= alpha;
    for (int j = 0; j < KB; ++j) {
      const float p = sP[r * (KB + 1) + j];
#pragma unroll
      for (int c = 0; c < D / 4; ++c) o[c] = fmaf(p, sV[j * LD + part + 4 * c], o[c]);
    }
  }
  if (qg < Lq) {
    const float inv = l > 0.f ? 1.f / l : 0.f;
    T* op = O + ((int64_t)b * Lq + qg) * ldo + h * D;
#pragma unroll
    for (int c = 0; c < D / 4; ++c) Elt<T>::st(op, part + 4 * c, o[c] * inv);
    if (part == 0) LSE[((int64_t)b * H + h) * Lq + qg] = l > 0.f ? m + __logf(l) : INFINITY;
  }
}

// ---- backward -----------------------------------------------------------------------------------
// delta[b,h,q] = sum_d dO*O (one wave per row)
template <typename T>
__global__ __launch_bounds__(256) void attn_gen_delta_k(const T* __restrict__ O, int64_t ldo, const T* __restrict__ dO,
                                                        int64_t lddo, float* __restrict__ delta, int H, int Lq,
                                                        int D, int64_t rows) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int lane = threadIdx.x & 63;
  const int q = (int)(row % Lq), h = (int)((row / Lq) % H), b = (int)(row / ((int64_t)Lq * H));
  const int64_t tok = (int64_t)b * Lq + q;
  float acc = 0.f;
  for (int d = lane; d < D; d += 64)
    acc += Elt<T>::ld(dO, tok * lddo + h * D + d) * Elt<T>::ld(O, tok * ldo + h * D + d);
  acc = wave_sum(acc);
  if (lane == 0) delta[row] = acc;
}

// dK, dV of one 64-key block; query blocks of QB rows streamed. Phase 1: thread (query row
// rq = t >> 3, keys j = part + 8 i) computes P and dS into LDS; phase 2: thread (key row
// kr = t >> 2, columns part + 4 c) accumulates dV += P^T dO, dK += dS^T Q.
template <typename T, int D>
__global__ __launch_bounds__(256) void attn_gen_bwd_kv_k(const T* __restrict__ Q, int64_t ldq, const T* __restrict__ K,
                                                         int64_t ldk, const T* __restrict__ V, int64_t ldv,
                                                         const T* __restrict__ dO, int64_t lddo,
                                                         const float* __restrict__ LSE,
                                                         const float* __restrict__ DELTA, T* __restrict__ dK,
                                                         int64_t lddk, T* __restrict__ dV, int64_t lddv, int H, int Lq,
                                                         int Lk, float scale, int causal,
                                                         const int32_t* __restrict__ kv_start) {
  constexpr int LD = D + 1;
  extern __shared__ float sm[];
  float* sK = sm;
  float* sV = sK + KB * LD;
  float* sQ = sV + KB * LD;
  float* sdO = sQ + QB * LD;
  float* sP = sdO + QB * LD;       // [QB][KB + 1]
  float* sdS = sP + QB * (KB + 1);  // [QB][KB + 1]
  float* sL = sdS + QB * (KB + 1);  // lse [QB]
  float* sD = sL + QB;              // delta [QB]
  const int nkb = (int)cdiv(Lk, KB);
  const int kb = blockIdx.x % nkb, h = (blockIdx.x / nkb) % H, b = blockIdx.x / (nkb * H);
  const int k0 = kb * KB;
  const int t = threadIdx.x;
  const int ks = kv_start ? kv_start[b] : 0;
  stage_rows<T>(sK, LD, K + h * D, ldk, (int64_t)b * Lk + k0, min(KB, Lk - k0), KB, D);
  stage_rows<T>(sV, LD, V + h * D, ldv, (int64_t)b * Lk + k0, min(KB, Lk - k0), KB, D);
  const int kr = t >> 2, part4 = t & 3;
  float dk[D / 4], dv[D / 4];
#pragma unroll
  for (int c = 0; c < D / 4; ++c) dk[c] = dv[c] = 0.f;
  const int rq = t >> 3, part8 = t & 7;
  const int qstart = causal ? (k0 / QB) * QB : 0;
  for (int q0 = qstart; q0 < Lq; q0 += QB) {
    __syncthreads();
    stage_rows<T>(sQ, LD, Q + h * D, ldq, (int64_t)b * Lq + q0, min(QB, Lq - q0), QB, D);
    stage_rows<T>(sdO, LD, dO + h * D, lddo, (int64_t)b * Lq + q0, min(QB, Lq - q0), QB, D);
    if (t < QB) {
      const int q = q0 + t;
      sL[t] = q < Lq ? LSE[((int64_t)b * H + h) * Lq + q] : INFINITY;
      sD[t] = q < Lq ? DELTA[((int64_t)b * H + h) * Lq + q] : 0.f;
    }
    __syncthreads();
    const int64_t qg = q0 + rq;
#pragma unroll
    for (int i = 0; i < KB / 8; ++i) {
      const int j = part8 + 8 * i;
      float sacc = 0.f, dpacc = 0.f;
      for (int d = 0; d < D; ++d) {
        sacc = fmaf(sQ[rq * LD + d], sK[j * LD + d], sacc);
        dpacc = fmaf(sdO[rq * LD + d], sV[j * LD + d], dpacc);
      }
      const bool ok = qg < Lq && visible(qg, k0 + j, Lk, ks, causal) && sL[rq] != INFINITY;
      const float p = ok ? __expf(sacc * scale - sL[rq]) : 0.f;
      sP[rq * (KB + 1) + j] = p;
      sdS[rq * (KB + 1) + j] = p * (dpacc - sD[rq]);
    }
    __syncthreads();
    for (int r = 0; r < QB; ++r) {
      const float p = sP[r * (KB + 1) + kr], ds = sdS[r * (KB + 1) + kr];
#pragma unroll
      for (int c = 0; c < D / 4; ++c) {
        dv[c] = fmaf(p, sdO[r * LD + part4 + 4 * c], dv[c]);
        dk[c] = fmaf(ds, sQ[r * LD + part4 + 4 * c], dk[c]);
      }
    }
  }
  const int64_t kg = k0 + kr;
  if (kg < Lk) {
    T* dkp = dK + ((int64_t)b * Lk + kg) * lddk + h * D;
    T* dvp = dV + ((int64_t)b * Lk + kg) * lddv + h * D;
#pragma unroll
    for (int c = 0; c < D / 4; ++c) {
      Elt<T>::st(dkp, part4 + 4 * c, dk[c] * scale);
      Elt<T>::st(dvp, part4 + 4 * c, dv[c]);
    }
  }
}

// dQ of one 64-row query block, key blocks streamed; thread (row r = t >> 2, keys
// part + 4 i) forms dS, then (row r, columns part + 4 c) accumulates dQ += dS K.
template <typename T, int D>
__global__ __launch_bounds__(256) void attn_gen_bwd_q_k(const T* __restrict__ Q, int64_t ldq, const T* __restrict__ K,
                                                        int64_t ldk, const T* __restrict__ V, int64_t ldv,
                                                        const T* __restrict__ dO, int64_t lddo,
                                                        const float* __restrict__ LSE, const float* __restrict__ DELTA,
                                                        T* __restrict__ dQ, int64_t lddq, int H, int Lq, int Lk,
                                                        float scale, int causal, const int32_t* __restrict__ kv_start) {
  constexpr int LD = D + 1;
  extern __shared__ float sm[];
  float* sQ = sm;
  float* sdO = sQ + QF * LD;
  float* sK = sdO + QF * LD;
  float* sV = sK + KB * LD;
  float* sdS = sV + KB * LD;  // [QF][KB + 1]
  const int nqb = (int)cdiv(Lq, QF);
  const int qb = blockIdx.x % nqb, h = (blockIdx.x / nqb) % H, b = blockIdx.x / (nqb * H);
  const int q0 = qb * QF;
  const int t = threadIdx.x, r = t >> 2, part = t & 3;
  const int ks = kv_start ? kv_start[b] : 0;
  const int64_t qg = q0 + r;
  stage_rows<T>(sQ, LD, Q + h * D, ldq, (int64_t)b * Lq + q0, min(QF, Lq - q0), QF, D);
  stage_rows<T>(sdO, LD, dO + h * D, lddo, (int64_t)b * Lq + q0, min(QF, Lq - q0), QF, D);
  const float lse = qg < Lq ? LSE[((int64_t)b * H + h) * Lq + qg] : INFINITY;
  const float del = qg < Lq ? DELTA[((int64_t)b * H + h) * Lq + qg] : 0.f;
  float dq[D / 4];
#pragma unroll
  for (int c = 0; c < D / 4; ++c) dq[c] = 0.f;
  const int kend = causal ? min(Lk, q0 + QF) : Lk;
  for (int k0 = 0; k0 < kend; k0 += KB) {
    __syncthreads();
    stage_rows<T>(sK, LD, K + h * D, ldk, (int64_t)b * Lk + k0, min(KB, Lk - k0), KB, D);
    stage_rows<T>(sV, LD, V + h * D, ldv, (int64_t)b * Lk + k0, min(KB, Lk - k0), KB, D);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < KB / 4; ++i) {
      const int j = part + 4 * i;
      float sacc = 0.f, dpacc = 0.f;
      for (int d = 0; d < D; ++d) {
        sacc = fmaf(sQ[r * LD + d], sK[j * LD + d], sacc);
        dpacc = fmaf(sdO[r * LD + d], sV[j * LD + d], dpacc);
      }
      const bool ok = qg < Lq && visible(qg, k0 + j, Lk, ks, causal) && lse != INFINITY;
      const float p = ok ? __expf(sacc * scale - lse) : 0.f;
      sdS[r * (KB + 1) + j] = p * (dpacc - del);
    }
    __syncthreads();
    for (int j = 0; j < KB; ++j) {
      const float ds = sdS[r * (KB + 1) + j];
#pragma unroll
      for (int c = 0; c < D / 4; ++c) dq[c] = fmaf(ds, sK[j * LD + part + 4 * c], dq[c]);
    }
  }
  if (qg < Lq) {
    T* qp = dQ + ((int64_t)b * Lq + qg) * lddq + h * D;
#pragma unroll
    for (int c = 0; c < D / 4; ++c) Elt<T>::st(qp, part + 4 * c, dq[c] * scale);
  }
}

template <typename T, int D>
int gen_fwd(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv, void* o, int64_t ldo,
            float* lse, int B, int H, int Lq, int Lk, float scale, int causal, const int32_t* ks, hipStream_t s) {
  constexpr int LD = D + 1;
  const int smem = (QF * LD + 2 * KB * LD + QF * (KB + 1)) * 4;
  static bool once = false;
  if (!once) {
    (void)hipFuncSetAttribute((const void*)attn_gen_fwd_k<T, D>, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    once = true;
  }
  const unsigned grid = (unsigned)(cdiv(Lq, QF) * H * B);
  attn_gen_fwd_k<T, D><<<grid, 256, smem, s>>>((const T*)q, ldq, (const T*)k, ldk, (const T*)v, ldv, (T*)o, ldo, lse,
                                               H, Lq, Lk, scale, causal, ks);
  return cullavo_check_launch("attn_fwd (generic)");
}

template <typename T, int D>
int gen_bwd(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv, const void* o,
            int64_t ldo, const void* dout, int64_t lddo, const float* lse, float* delta, void* dq, int64_t lddq,
            void* dk, int64_t lddk, void* dv, int64_t lddv, int B, int H, int Lq, int Lk, float scale, int causal,
            const int32_t* ks, hipStream_t s) {
  constexpr int LD = D + 1;
  const int smem_kv = (2 * KB * LD + 2 * QB * LD + 2 * QB * (KB + 1) + 2 * QB) * 4;
  const int smem_q = (2 * QF * LD + 2 * KB * LD + QF * (KB + 1)) * 4;
  static bool once = false;
  if (!once) {
    (void)hipFuncSetAttribute((const void*)attn_gen_bwd_kv_k<T, D>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              smem_kv);
    (void)hipFuncSetAttribute((const void*)attn_gen_bwd_q_k<T, D>, hipFuncAttributeMaxDynamicSharedMemorySize, smem_q);
    once = true;
  }
  const int64_t rows = (int64_t)B * H * Lq;
  attn_gen_delta_k<T><<<(unsigned)cdiv(rows, 4), 256, 0, s>>>((const T*)o, ldo, (const T*)dout, lddo, delta, H, Lq, D,
                                                               rows);
  attn_gen_bwd_kv_k<T, D><<<(unsigned)(cdiv(Lk, KB) * H * B), 256, smem_kv, s>>>(
      (const T*)q, ldq, (const T*)k, ldk, (const T*)v, ldv, (const T*)dout, lddo, lse, delta, (T*)dk, lddk, (T*)dv,
      lddv, H, Lq, Lk, scale, causal, ks);
  attn_gen_bwd_q_k<T, D><<<(unsigned)(cdiv(Lq, QF) * H * B), 256, smem_q, s>>>(
      (const T*)q, ldq, (const T*)k, ldk, (const T*)v, ldv, (const T*)dout, lddo, lse, delta, (T*)dq, lddq, H, Lq, Lk,
      scale, causal, ks);
  return cullavo_check_launch("attn_bwd (generic)");
}

}  // namespace

// Dispatch used by cullavo_attn_fwd / _bwd (attention.hip) for f32 storage or D in {16, 32}.
int cullavo_attn_generic_fwd(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                             void* o, int64_t ldo, float* lse, int B, int H, int Lq, int Lk, int D, float scale,
                             int causal, const int32_t* ks, int dtype, hipStream_t s) {
#define GF(T_, D_) return gen_fwd<T_, D_>(q, ldq, k, ldk, v, ldv, o, ldo, lse, B, H, Lq, Lk, scale, causal, ks, s)
#define GFD(T_)                  \
  switch (D) {                   \
    case 16: GF(T_, 16);         \
    case 32: GF(T_, 32);         \
    case 64: GF(T_, 64);         \
    case 128: GF(T_, 128);       \
    default: break;              \
  }
  if (dtype == CULLAVO_DT_F32) { GFD(float) }
  else { GFD(u16) }
#undef GFD
#undef GF
  cullavo_set_error("attention: head_dim must be 16, 32, 64 or 128");
  return CULLAVO_EUNSUPPORTED;
}

int cullavo_attn_generic_bwd(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                             const void* o, int64_t ldo, const void* dout, int64_t lddo, const float* lse,
                             float* delta, void* dq, int64_t lddq, void* dk, int64_t lddk, void* dv, int64_t lddv,
                             int B, int H, int Lq, int Lk, int D, float scale, int causal, const int32_t* ks,
                             int dtype, hipStream_t s) {
#define GB(T_, D_)                                                                                                 \
  return gen_bwd<T_, D_>(q, ldq, k, ldk, v, ldv, o, ldo, dout, lddo, lse, delta, dq, lddq, dk, lddk, dv, lddv, B, H, \
                         Lq, Lk, scale, causal, ks, s)
#define GBD(T_)                  \
  switch (D) {                   \
    case 16: GB(T_, 16);         \
    case 32: GB(T_, 32);         \
    case 64: GB(T_, 64);         \
    case 128: GB(T_, 128);       \
    default: break;              \
  }
  if (dtype == CULLAVO_DT_F32) { GBD(float) }
  else { GBD(u16) }
#undef GBD
#undef GB
  cullavo_set_error("attention: head_dim must be 16, 32, 64 or 128");
  return CULLAVO_EUNSUPPORTED;
}
