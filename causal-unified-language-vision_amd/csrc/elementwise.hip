// Element-wise and small-reduction kernels of the CuLLaVO step: SwiGLU, activation backward,
// bias-gradient column sums, Llama RoPE, and the optimiser pieces (sum of squares, clip
// coefficient, fused AdamW). All HBM-bound: 16 B per lane per access, grid-stride loops.
#include "common.h"

namespace {

DEV float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }
DEV float siluf_(float x) { return x / (1.f + __expf(-x)); }
// swiglu_bwd_k's sigmoid: the expression of gemm_common.h sigmoid_rcp (the SwiGLU backward fused into
// the down-projection dX GEMM's epilogue), so the two paths are bitwise equal
DEV float sigmoid_rcp_(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }

// one 16-B vector per thread (the loops stay grid-stride): against a 2048-block cap the SwiGLU
// kernels run 10 % faster (tools/stream_bench.py: 5.1 -> 5.7 TB/s), more loads in flight per CU
int ew_grid(int64_t nvec) { return (int)std::min<int64_t>(std::max<int64_t>(1, cdiv(nvec, 256)), 1 << 30); }

// ---- SwiGLU (tf:llama/modeling_llama.py:163-176: down(act(gate(x)) * up(x))) --------------
// gu: fused gate|up projection output [rows, 2F]; one 8-wide column group per thread
template <typename T>
__global__ __launch_bounds__(256) void swiglu_fwd_k(const T* __restrict__ gu, int64_t rows, int64_t F,
                                                    T* __restrict__ o) {
  const int64_t fv = F / 8, nvec = rows * fv;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / fv, c = (i % fv) * 8;
    float gv[8], uv[8], ov[8];
    load8(gu + r * 2 * F + c, gv);
    load8(gu + r * 2 * F + F + c, uv);
#pragma unroll
    for (int j = 0; j < 8; ++j) ov[j] = Elt<T>::rnd(siluf_(gv[j])) * uv[j];
    store8(o + r * F + c, ov);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void swiglu_bwd_k(const T* __restrict__ d, const T* __restrict__ gu,
                                                    int64_t rows, int64_t F, T* __restrict__ dgu) {
  const int64_t fv = F / 8, nvec = rows * fv;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / fv, c = (i % fv) * 8;
    float dv[8], gv[8], uv[8], a[8], b[8];
    load8(d + r * F + c, dv);
    load8(gu + r * 2 * F + c, gv);
    load8(gu + r * 2 * F + F + c, uv);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float s = sigmoid_rcp_(gv[j]);
      const float silu = gv[j] * s;
      b[j] = dv[j] * Elt<T>::rnd(silu);
      a[j] = dv[j] * uv[j] * s * (1.f + gv[j] * (1.f - s));
    }
    store8(dgu + r * 2 * F + c, a);
    store8(dgu + r * 2 * F + F + c, b);
  }
}

// ---- 16-bit matrix transpose (K-major weight copies for the dX GEMMs) ------------------------
// 64x64 tiles through LDS: 16-B coalesced loads of source rows, 16-B coalesced stores of
// destination rows (8 source rows of one column gathered from LDS per thread). HBM-bound:
// 4 B per element moved.
__global__ __launch_bounds__(256) void transpose16_k(const u16* __restrict__ src, int64_t lds_, u16* __restrict__ dst,
                                                     int64_t ldd, int64_t rows, int64_t cols, int64_t tiles_c) {
  __shared__ u16 tile[64][64 + 8];
  const int64_t tr = blockIdx.x / tiles_c, tc = blockIdx.x % tiles_c;
  const int64_t r0 = tr * 64, c0 = tc * 64;
  const int t = threadIdx.x;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int id = t + k * 256, r = id >> 3, c8 = (id & 7) * 8;
    u16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (r0 + r < rows && c0 + c8 < cols) v = *(const u16x8*)(src + (r0 + r) * lds_ + c0 + c8);
    *(u16x8*)&tile[r][c8] = v;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int id = t + k * 256, c = id >> 3, r8 = (id & 7) * 8;
    u16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = tile[r8 + j][c];
    if (c0 + c < cols && r0 + r8 < rows) *(u16x8*)(dst + (c0 + c) * ldd + r0 + r8) = v;
  }
}

// ---- activation backward (projector GELU, CLIP quick_gelu) ---------------------------------
template <typename T, int ACT>
__global__ __launch_bounds__(256) void act_bwd_k(const T* __restrict__ dy, const T* __restrict__ x,
                                                 T* __restrict__ dx, int64_t nvec) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * 256) {
    float dv[8], xv[8], o[8];
    load8(dy + i * 8, dv);
    load8(x + i * 8, xv);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = xv[j];
      float dg;
      if (ACT == CULLAVO_ACT_GELU) {
        const float cdf = 0.5f * (1.f + erff(v * 0.70710678118654752f));
        const float pdf = 0.39894228040143268f * __expf(-0.5f * v * v);
        dg = cdf + v * pdf;
      } else {
        const float s = sigmoidf_(1.702f * v);
        dg = s + 1.702f * v * s * (1.f - s);
      }
      o[j] = dv[j] * dg;
    }
    store8(dx + i * 8, o);
  }
}

// ---- column sums (bias gradients) ----------------------------------------------------------
// block: 32 column groups of 8 columns x 8 row lanes; grid.y splits the rows.
constexpr int kColsumSplit = 32;
template <typename T>
__global__ __launch_bounds__(256) void colsum_k(const T* __restrict__ x, int64_t rows, int64_t cols,
                                                float* __restrict__ part) {
  __shared__ float red[8][256 + 8];
  const int cg = threadIdx.x & 31, rl = threadIdx.x >> 5;
  const int64_t c0 = (int64_t)blockIdx.x * 256 + cg * 8;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (c0 < cols) {
    for (int64_t r = rl + 8 * blockIdx.y; r < rows; r += 8 * gridDim.y) {
      float v[8];
      load8(x + r * cols + c0, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += v[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[rl][cg * 8 + j] = acc[j];
  __syncthreads();
  const int c = threadIdx.x;  // 256 columns of this block
  const int64_t col = (int64_t)blockIdx.x * 256 + c;
  if (col < cols) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += red[k][c];
    part[(int64_t)blockIdx.y * cols + col] = s;
  }
}

template <typename TO>
__global__ __launch_bounds__(256) void colsum_final_k(const float* __restrict__ part, int nsplit,
                                                      int64_t cols, TO* __restrict__ out, float beta) {
  const int64_t col = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (col >= cols) return;
  float s = 0.f;
  for (int p = 0; p < nsplit; ++p) s += part[(int64_t)p * cols + col];
  if (beta != 0.f) s += beta * Elt<TO>::ld(out, col);
  Elt<TO>::st(out, col, s);
}

// ---- RoPE (tf:llama/modeling_llama.py:73-160) ----------------------------------------------
// one block per token; thread = (head slot, group of 4 frequency indices). cos/sin are
// computed in f32 from pos * inv_freq and rounded to the activation dtype (reference :121-125);
// out = rnd(rnd(x*cos) + rnd(rotate_half(x)*sin)), rotate_half(x) = cat(-x2, x1).
template <typename T>
DEV void rope_heads(T* base, int64_t ld, int nh, int half, int i4, int hslot, int nslot,
                    const float* c, const float* s, int inverse) {
  for (int h = hslot; h < nh; h += nslot) {
    T* p1 = base + (int64_t)h * 2 * half + i4 * 4;
    T* p2 = p1 + half;
    float x1[4], x2[4], o1[4], o2[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      x1[j] = Elt<T>::ld(p1, j);
      x2[j] = Elt<T>::ld(p2, j);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (!inverse) {
        o1[j] = Elt<T>::rnd(Elt<T>::rnd(x1[j] * c[j]) + Elt<T>::rnd(-x2[j] * s[j]));
        o2[j] = Elt<T>::rnd(Elt<T>::rnd(x2[j] * c[j]) + Elt<T>::rnd(x1[j] * s[j]));
      } else {  // transpose rotation: the gradient of the forward map
        o1[j] = x1[j] * c[j] + x2[j] * s[j];
        o2[j] = x2[j] * c[j] - x1[j] * s[j];
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      Elt<T>::st(p1, j, o1[j]);
      Elt<T>::st(p2, j, o2[j]);
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void rope_k(T* __restrict__ q, int64_t ldq, T* __restrict__ k,
                                              int64_t ldk, const int64_t* __restrict__ pos, int hq,
                                              int hk, int D, float theta, int inverse) {
  const int64_t t = blockIdx.x;
  const int half = D / 2;
  const int ng = half / 4;  // groups of 4 frequencies per head
  const int i4 = threadIdx.x % ng;
  const int hslot = threadIdx.x / ng;
  const int nslot = 256 / ng;
  const float p = (float)pos[t];
  float c[4], s[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int i = i4 * 4 + j;
    const float inv_freq = 1.0f / powf(theta, (float)(2 * i) / (float)D);
    const float ang = p * inv_freq;
    c[j] = Elt<T>::rnd(cosf(ang));
    s[j] = Elt<T>::rnd(sinf(ang));
  }
  if (hslot >= nslot) return;
  rope_heads<T>(q + t * ldq, ldq, hq, half, i4, hslot, nslot, c, s, inverse);
  if (k != nullptr) rope_heads<T>(k + t * ldk, ldk, hk, half, i4, hslot, nslot, c, s, inverse);
}

// 16-B variant: the block computes the token's half-D (cos, sin) pairs once into LDS (same f32
// formula and rounding as rope_k, which evaluated them 16x redundantly per thread), then each
// item = (head, group of 8 frequencies) moves x1[8] and x2[8] with one 16-B load/store each.
// Needs D % 16 == 0 and 16-B aligned rows.
template <typename T>
__global__ __launch_bounds__(256) void rope8_k(T* __restrict__ q, int64_t ldq, T* __restrict__ k,
                                               int64_t ldk, const int64_t* __restrict__ pos, int hq,
                                               int hk, int D, float theta, int inverse) {
  __shared__ float cs[256], sn[256];
  const int64_t t = blockIdx.x;
  const int half = D / 2, ng = half / 8;
  if (threadIdx.x < half) {
    const int i = threadIdx.x;
    const float inv_freq = 1.0f / powf(theta, (float)(2 * i) / (float)D);
    const float ang = (float)pos[t] * inv_freq;
    cs[i] = Elt<T>::rnd(cosf(ang));
    sn[i] = Elt<T>::rnd(sinf(ang));
  }
  __syncthreads();
  const int nq = hq * ng, nall = (hq + (k != nullptr ? hk : 0)) * ng;
  for (int it = threadIdx.x; it < nall; it += 256) {
    const bool isq = it < nq;
    const int w = isq ? it : it - nq, h = w / ng, g8 = (w % ng) * 8;
    T* p1 = (isq ? q + t * ldq : k + t * ldk) + (int64_t)h * D + g8;
    T* p2 = p1 + half;
    float x1[8], x2[8], o1[8], o2[8];
    load8(p1, x1);
    load8(p2, x2);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float c = cs[g8 + j], sv = sn[g8 + j];
      if (!inverse) {
        o1[j] = Elt<T>::rnd(Elt<T>::rnd(x1[j] * c) + Elt<T>::rnd(-x2[j] * sv));
        o2[j] = Elt<T>::rnd(Elt<T>::rnd(x2[j] * c) + Elt<T>::rnd(x1[j] * sv));
      } else {
        o1[j] = x1[j] * c + x2[j] * sv;
        o2[j] = x2[j] * c - x1[j] * sv;
      }
    }
    store8(p1, o1);
    store8(p2, o2);
  }
}

// RoPE of the decode step's new rows fused with the KV-cache append (cullavo_rope_kv_append):
// rope8_k's arithmetic on q (in place) and k, the rotated k written straight to its cache row
// (b, start[b] + t % Lnew) instead of back into the projection output, and v copied beside it --
// one launch and one pass over k instead of rope8_k + kv_append_k (decode.hip).
__global__ __launch_bounds__(256) void rope_append8_k(u16* __restrict__ q, int64_t ldq, const u16* __restrict__ k,
                                                      int64_t ldk, const u16* __restrict__ v, int64_t ldv,
                                                      const int64_t* __restrict__ pos, int hq, int hk, int D,
                                                      float theta, u16* __restrict__ kc, u16* __restrict__ vc,
                                                      int64_t ld_tok, int64_t ld_b, const int32_t* __restrict__ start,
                                                      int Lnew) {
  __shared__ float cs[256], sn[256];
  const int64_t t = blockIdx.x;
  const int half = D / 2, ng = half / 8;
  if (threadIdx.x < half) {
    const int i = threadIdx.x;
    const float inv_freq = 1.0f / powf(theta, (float)(2 * i) / (float)D);
    const float ang = (float)pos[t] * inv_freq;
    cs[i] = Elt<u16>::rnd(cosf(ang));
    sn[i] = Elt<u16>::rnd(sinf(ang));
  }
  __syncthreads();
  const int b = (int)(t / Lnew), tt = (int)(t % Lnew);
  const int64_t crow = (int64_t)b * ld_b + (int64_t)(start[b] + tt) * ld_tok;
  const int nq = hq * ng, nall = (hq + hk) * ng;
  for (int it = threadIdx.x; it < nall; it += 256) {
    const bool isq = it < nq;
    const int w = isq ? it : it - nq, h = w / ng, g8 = (w % ng) * 8;
    const int64_t col = (int64_t)h * D + g8;
    const u16* s1 = isq ? q + t * ldq + col : k + t * ldk + col;
    u16* d1 = isq ? q + t * ldq + col : kc + crow + col;
    float x1[8], x2[8], o1[8], o2[8];
    load8(s1, x1);
    load8(s1 + half, x2);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float c = cs[g8 + j], sv = sn[g8 + j];
      o1[j] = Elt<u16>::rnd(Elt<u16>::rnd(x1[j] * c) + Elt<u16>::rnd(-x2[j] * sv));
      o2[j] = Elt<u16>::rnd(Elt<u16>::rnd(x2[j] * c) + Elt<u16>::rnd(x1[j] * sv));
    }
    store8(d1, o1);
    store8(d1 + half, o2);
  }
  for (int c8 = threadIdx.x * 8; c8 < hk * D; c8 += 256 * 8)
    *reinterpret_cast<u16x8*>(vc + crow + c8) = *reinterpret_cast<const u16x8*>(v + t * ldv + c8);
}

// ---- optimiser ------------------------------------------------------------------------------
// block b sums a fixed grid-stride subset in a fixed order (lane accumulation, then the wave
// tree, then waves 0..3) into partials[b]; sumsq_final_k adds the partials to out[0] in a
// fixed tree order. Same inputs -> same bits, whatever the scheduling.
template <typename T>
__global__ __launch_bounds__(256) void sumsq_k(const T* __restrict__ x, int64_t n, float* __restrict__ partials) {
  __shared__ float red[4];
  float acc = 0.f;
  const int64_t nvec = n / 8;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * 256) {
    float v[8];
    load8(x + i * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += v[j] * v[j];
  }
  if (blockIdx.x == 0) {  // tail
    for (int64_t i = nvec * 8 + threadIdx.x; i < n; i += 256) {
      const float v = Elt<T>::ld(x, i);
      acc += v * v;
    }
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) partials[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(256) void sumsq_final_k(const float* __restrict__ partials, int np,
                                                     float* __restrict__ out) {
  __shared__ float red[4];
  float acc = 0.f;
  for (int i = threadIdx.x; i < np; i += 256) acc += partials[i];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) out[0] += (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ void clip_coef_k(const float* sumsq, float max_norm, float* coef, float* norm_out) {
  const float norm = sqrtf(sumsq[0]);
  if (norm_out) norm_out[0] = norm;
  coef[0] = fminf(1.f, max_norm / (norm + 1e-6f));
}

template <typename T>
__global__ __launch_bounds__(256) void scale_k(T* __restrict__ x, int64_t n, const float* __restrict__ sc) {
  const float s = sc[0];
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    Elt<T>::st(x, i, Elt<T>::ld(x, i) * s);
}

// torch.optim.AdamW (single-tensor math): p *= 1-lr*wd; m = lerp(m, g, 1-b1);
// v = b2*v + (1-b2) g^2; p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps)
// (one element, with the stored dtypes' roundings)
template <typename T, typename S>
DEV void adamw_elem(float gv, float& pv, float& mv, float& vv, float lr, float b1, float b2, float eps, float wd,
                    float bc2_sqrt, float step_size) {
#pragma clang fp contract(off)  // no FMA fusion: the 8-wide and element-wise paths round alike
  pv = Elt<T>::rnd(pv * (1.f - lr * wd));
  mv = Elt<S>::rnd(mv + (gv - mv) * (1.f - b1));
  vv = Elt<S>::rnd(vv * b2 + (1.f - b2) * gv * gv);
  const float denom = sqrtf(vv) / bc2_sqrt + eps;
  pv = pv - step_size * mv / denom;
}

// 8 elements per lane per access (16 B of bf16 params / grads, 16 or 32 B of state), so the
// 14-22 B/param stream is issued as full-width loads; the scalar loop takes the tail (and every
// element when a buffer is not 16-B aligned: vec = false).
template <typename T, typename S>
__global__ __launch_bounds__(256) void adamw_k(T* __restrict__ p, const T* __restrict__ g,
                                               S* __restrict__ m, S* __restrict__ v, int64_t n,
                                               float lr, float b1, float b2, float eps, float wd,
                                               float bc1, float bc2_sqrt,
                                               const float* __restrict__ gscale, bool vec) {
  const float gs = gscale ? gscale[0] : 1.f;
  const float step_size = lr / bc1;
  const int64_t nvec = vec ? n / 8 : 0;
  // two grid-stride steps per trip: eight 16-B loads in flight per lane instead of four
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i0 = blockIdx.x * 256 + threadIdx.x; i0 < nvec; i0 += 2 * stride) {
    float gv[2][8], pv[2][8], mv[2][8], vv[2][8];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int64_t i = i0 + u * stride;
      if (i < nvec) {
        load8(g + i * 8, gv[u]);
        load8(p + i * 8, pv[u]);
        load8(m + i * 8, mv[u]);
        load8(v + i * 8, vv[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int64_t i = i0 + u * stride;
      if (i < nvec) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          adamw_elem<T, S>(gv[u][j] * gs, pv[u][j], mv[u][j], vv[u][j], lr, b1, b2, eps, wd, bc2_sqrt, step_size);
        store8(p + i * 8, pv[u]);
        store8(m + i * 8, mv[u]);
        store8(v + i * 8, vv[u]);
      }
    }
  }
  for (int64_t i = nvec * 8 + blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    float pv = Elt<T>::ld(p, i), mv = Elt<S>::ld(m, i), vv = Elt<S>::ld(v, i);
    adamw_elem<T, S>(Elt<T>::ld(g, i) * gs, pv, mv, vv, lr, b1, b2, eps, wd, bc2_sqrt, step_size);
    Elt<T>::st(p, i, pv);
    Elt<S>::st(m, i, mv);
    Elt<S>::st(v, i, vv);
  }
}

}  // namespace

extern "C" int cullavo_swiglu_fwd(const void* gu, int64_t rows, int64_t F, void* out, int dtype,
                                  void* stream) {
  CV_REQUIRE(F % 8 == 0, CULLAVO_EINVAL, "F must be a multiple of 8");
  if (rows == 0 || F == 0) return CULLAVO_OK;
  hipStream_t s = CV_STREAM(stream);
  const int g = ew_grid(rows * F / 8);
  if (dtype == CULLAVO_DT_BF16) swiglu_fwd_k<u16><<<g, 256, 0, s>>>((const u16*)gu, rows, F, (u16*)out);
  else if (dtype == CULLAVO_DT_F32) swiglu_fwd_k<float><<<g, 256, 0, s>>>((const float*)gu, rows, F, (float*)out);
  else CV_REQUIRE(false, CULLAVO_EUNSUPPORTED, "dtype");
  return cullavo_check_launch("swiglu_fwd");
}

extern "C" int cullavo_swiglu_bwd(const void* dout, const void* gu, int64_t rows, int64_t F, void* dgu,
                                  int dtype, void* stream) {
  CV_REQUIRE(F % 8 == 0, CULLAVO_EINVAL, "F must be a multiple of 8");
  if (rows == 0 || F == 0) return CULLAVO_OK;
  hipStream_t s = CV_STREAM(stream);
  const int g = ew_grid(rows * F / 8);
  if (dtype == CULLAVO_DT_BF16) swiglu_bwd_k<u16><<<g, 256, 0, s>>>((const u16*)dout, (const u16*)gu, rows, F, (u16*)dgu);
  else if (dtype == CULLAVO_DT_F32) swiglu_bwd_k<float><<<g, 256, 0, s>>>((const float*)dout, (const float*)gu, rows, F, (float*)dgu);
  else CV_REQUIRE(false, CULLAVO_EUNSUPPORTED, "dtype");
  return cullavo_check_launch("swiglu_bwd");
}

extern "C" int cullavo_act_bwd(int act, const void* dy, const void* preact, void* dx, int64_t n,
                               int dtype, void* stream) {
  CV_REQUIRE(n % 8 == 0, CULLAVO_EINVAL, "n must be a multiple of 8");
  CV_REQUIRE(act == CULLAVO_ACT_GELU || act == CULLAVO_ACT_QUICK_GELU, CULLAVO_EINVAL, "act");
  if (n == 0) return CULLAVO_OK;
  hipStream_t s = CV_STREAM(stream);
  const int64_t nv = n / 8;
  const int g = ew_grid(nv);
  if (dtype == CULLAVO_DT_BF16) {
    if (act == CULLAVO_ACT_GELU) act_bwd_k<u16, CULLAVO_ACT_GELU><<<g, 256, 0, s>>>((const u16*)dy, (const u16*)preact, (u16*)dx, nv);
    else act_bwd_k<u16, CULLAVO_ACT_QUICK_GELU><<<g, 256, 0, s>>>((const u16*)dy, (const u16*)preact, (u16*)dx, nv);
  } else if (dtype == CULLAVO_DT_F32) {
    if (act == CULLAVO_ACT_GELU) act_bwd_k<float, CULLAVO_ACT_GELU><<<g, 256, 0, s>>>((const float*)dy, (const float*)preact, (float*)dx, nv);
    else act_bwd_k<float, CULLAVO_ACT_QUICK_GELU><<<g, 256, 0, s>>>((const float*)dy, (const float*)preact, (float*)dx, nv);
  } else {
    CV_REQUIRE(false, CULLAVO_EUNSUPPORTED, "dtype");
  }
  return cullavo_check_launch("act_bwd");
}

extern "C" size_t cullavo_colsum_workspace(int64_t rows, int64_t cols) {
  (void)rows;
  return (size_t)kColsumSplit * cols * sizeof(float);
}

extern "C" int cullavo_colsum(const void* x, int64_t rows, int64_t cols, void* out, int out_dtype,
                              float beta, float* ws, int dtype, void* stream) {
  CV_REQUIRE(cols % 8 == 0, CULLAVO_EINVAL, "cols must be a multiple of 8");
  CV_REQUIRE(ws != nullptr, CULLAVO_EINVAL, "workspace required");
  if (cols == 0) return CULLAVO_OK;
  hipStream_t s = CV_STREAM(stream);
  dim3 grid((unsigned)cdiv(cols, 256), kColsumSplit);
  if (dtype == CULLAVO_DT_BF16) colsum_k<u16><<<grid, 256, 0, s>>>((const u16*)x, rows, cols, ws);
  else if (dtype == CULLAVO_DT_F32) colsum_k<float><<<grid, 256, 0, s>>>((const float*)x, rows, cols, ws);
  else CV_REQUIRE(false, CULLAVO_EUNSUPPORTED, "dtype");
  if (out_dtype == CULLAVO_DT_BF16) colsum_final_k<u16><<<cdiv(cols, 256), 256, 0, s>>>(ws, kColsumSplit, cols, (u16*)out, beta);
  else colsum_final_k<float><<<cdiv(cols, 256), 256, 0, s>>>(ws, kColsumSplit, cols, (float*)out, beta);
  return cullavo_check_launch("colsum");
}

extern "C" int cullavo_rope(void* q, int64_t ldq, void* k, int64_t ldk, const int64_t* position_ids,
                            int64_t tokens, int hq, int hk, int head_dim, float theta, int inverse,
                            int dtype, void* stream) {
  CV_REQUIRE(head_dim % 8 == 0 && head_dim >= 8 && head_dim / 8 <= 256, CULLAVO_EINVAL, "head_dim");
  if (tokens == 0) return CULLAVO_OK;
  hipStream_t s = CV_STREAM(stream);
  const uintptr_t al = (uintptr_t)q | (uintptr_t)k;
  const bool vec = head_dim % 16 == 0 && head_dim <= 512 && ldq % 8 == 0 && (k == nullptr || ldk % 8 == 0) &&
                   (al & 15) == 0;
  if (vec) {
    if (dtype == CULLAVO_DT_BF16) rope8_k<u16><<<(unsigned)tokens, 256, 0, s>>>((u16*)q, ldq, (u16*)k, ldk, position_ids, hq, hk, head_dim, theta, inverse);
    else if (dtype == CULLAVO_DT_F32) rope8_k<float><<<(unsigned)tokens, 256, 0, s>>>((float*)q, ldq, (float*)k, ldk, position_ids, hq, hk, head_dim, theta, inverse);
    else CV_REQUIRE(false, CULLAVO_EUNSUPPORTED, "dtype");
    return cullavo_check_launch("rope");
  }
  if (dtype == CULLAVO_DT_BF16) rope_k<u16><<<(unsigned)tokens, 256, 0, s>>>((u16*)q, ldq, (u16*)k, ldk, position_ids, hq, hk, head_dim, theta, inverse);
  else if (dtype == CULLAVO_DT_F32) rope_k<float><<<(unsigned)tokens, 256, 0, s>>>((float*)q, ldq, (float*)k, ldk, position_ids, hq, hk, head_dim, theta, inverse);
  else CV_REQUIRE(false, CULLAVO_EUNSUPPORTED, "dtype");
  return cullavo_check_launch("rope");
}

extern "C" int cullavo_rope_kv_append(void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                                      const int64_t* position_ids, int64_t tokens, int hq, int hk, int head_dim,
                                      float theta, void* k_cache, void* v_cache, int64_t ld_tok, int64_t ld_b,
                                      const int32_t* start, int Lnew, int dtype, void* stream) {
  CV_REQUIRE(dtype == CULLAVO_DT_BF16, CULLAVO_EUNSUPPORTED, "rope_kv_append: bf16");
  CV_REQUIRE(head_dim % 16 == 0 && head_dim <= 512 && Lnew >= 1 && tokens % Lnew == 0, CULLAVO_EINVAL,
             "rope_kv_append: head_dim a multiple of 16 up to 512, tokens = B * Lnew");
  CV_REQUIRE(ldq % 8 == 0 && ldk % 8 == 0 && ldv % 8 == 0 && ld_tok % 8 == 0 && ld_b % 8 == 0 &&
                 (((uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)k_cache | (uintptr_t)v_cache) & 15) == 0,
             CULLAVO_EINVAL, "rope_kv_append: 16-byte aligned rows");
  if (tokens == 0) return CULLAVO_OK;
  hipStream_t s = CV_STREAM(stream);
  rope_append8_k<<<(unsigned)tokens, 256, 0, s>>>((u16*)q, ldq, (const u16*)k, ldk, (const u16*)v, ldv, position_ids, hq,
                                                  hk, head_dim, theta, (u16*)k_cache, (u16*)v_cache, ld_tok, ld_b,
                                                  start, Lnew);
  return cullavo_check_launch("rope_kv_append");
}

extern "C" int cullavo_sumsq(const void* x, int64_t n, float* out, float* partials, int dtype, void* stream) {
  if (n == 0) return CULLAVO_OK;
  CV_REQUIRE(partials != nullptr, CULLAVO_EINVAL, "partials workspace (CULLAVO_SUMSQ_PARTIALS floats)");
  CV_REQUIRE(dtype != CULLAVO_DT_BF16 || ((uintptr_t)x & 15) == 0, CULLAVO_EINVAL, "x must be 16-B aligned");
  CV_REQUIRE(dtype != CULLAVO_DT_F32 || ((uintptr_t)x & 15) == 0, CULLAVO_EINVAL, "x must be 16-B aligned");
  hipStream_t s = CV_STREAM(stream);
  const int g = (int)std::min<int64_t>(CULLAVO_SUMSQ_PARTIALS, std::max<int64_t>(1, cdiv(n / 8, 256)));
  if (dtype == CULLAVO_DT_BF16) sumsq_k<u16><<<g, 256, 0, s>>>((const u16*)x, n, partials);
  else if (dtype == CULLAVO_DT_F32) sumsq_k<float><<<g, 256, 0, s>>>((const float*)x, n, partials);
  else CV_REQUIRE(false, CULLAVO_EUNSUPPORTED, "dtype");
  sumsq_final_k<<<1, 256, 0, s>>>(partials, g, out);
  return cullavo_check_launch("sumsq");
}

extern "C" int cullavo_clip_coef(const float* sumsq, float max_norm, float* coef, float* norm_out,
                                 void* stream) {
  clip_coef_k<<<1, 1, 0, CV_STREAM(stream)>>>(sumsq, max_norm, coef, norm_out);
  return cullavo_check_launch("clip_coef");
}

extern "C" int cullavo_scale_inplace(void* x, int64_t n, const float* scale, int dtype, void* stream) {
  if (n == 0) return CULLAVO_OK;
  hipStream_t s = CV_STREAM(stream);
  if (dtype == CULLAVO_DT_BF16) scale_k<u16><<<ew_grid(n), 256, 0, s>>>((u16*)x, n, scale);
  else if (dtype == CULLAVO_DT_F32) scale_k<float><<<ew_grid(n), 256, 0, s>>>((float*)x, n, scale);
  else CV_REQUIRE(false, CULLAVO_EUNSUPPORTED, "dtype");
  return cullavo_check_launch("scale_inplace");
}

extern "C" int cullavo_adamw(void* param, const void* grad, void* exp_avg, void* exp_avg_sq, int64_t n,
                             float lr, float beta1, float beta2, float eps, float weight_decay,
                             int64_t step, const float* grad_scale, int dtype, int state_dtype,
                             void* stream) {
  CV_REQUIRE(step >= 1, CULLAVO_EINVAL, "step must be >= 1");
  if (n == 0) return CULLAVO_OK;
  hipStream_t s = CV_STREAM(stream);
  const float bc1 = 1.f - (float)std::pow((double)beta1, (double)step);
  const float bc2s = (float)std::sqrt(1.0 - std::pow((double)beta2, (double)step));
  const bool vec = (((uintptr_t)param | (uintptr_t)grad | (uintptr_t)exp_avg | (uintptr_t)exp_avg_sq) & 15) == 0;
  // ~4 vectors per thread instead of the 2048-block grid-stride cap: more loads in flight per
  // CU (tools/adamw_bench.py, 1.6 G elements: 4.13 -> 3.78 ms, 5.5 -> 6.0 TB/s); non-temporal
  // accesses measured no different
  const int64_t nv = vec ? n / 8 : n;
  const int g = (int)std::min<int64_t>(std::max<int64_t>(1, cdiv(nv, 256 * 4)), 1 << 30);
#define ADAM(T, S) adamw_k<T, S><<<g, 256, 0, s>>>((T*)param, (const T*)grad, (S*)exp_avg, (S*)exp_avg_sq, n, lr, beta1, beta2, eps, weight_decay, bc1, bc2s, grad_scale, vec)
  if (dtype == CULLAVO_DT_BF16 && state_dtype == CULLAVO_DT_BF16) ADAM(u16, u16);
  else if (dtype == CULLAVO_DT_BF16 && state_dtype == CULLAVO_DT_F32) ADAM(u16, float);
  else if (dtype == CULLAVO_DT_F32 && state_dtype == CULLAVO_DT_F32) ADAM(float, float);
  else CV_REQUIRE(false, CULLAVO_EUNSUPPORTED, "dtype combination");
#undef ADAM
  return cullavo_check_launch("adamw");
}

extern "C" int cullavo_transpose16(const void* src, int64_t ld_src, void* dst, int64_t ld_dst, int64_t rows,
                                   int64_t cols, void* stream) {
  CV_REQUIRE(rows % 8 == 0 && cols % 8 == 0 && ld_src % 8 == 0 && ld_dst % 8 == 0, CULLAVO_EINVAL,
             "rows, cols and leading dims must be multiples of 8");
  CV_REQUIRE(ld_src >= cols && ld_dst >= rows, CULLAVO_EINVAL, "leading dims");
  CV_REQUIRE(((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 15) == 0, CULLAVO_EINVAL, "16-B alignment");
  if (rows == 0 || cols == 0) return CULLAVO_OK;
  const int64_t tiles_c = cdiv(cols, 64), tiles = cdiv(rows, 64) * tiles_c;
  CV_REQUIRE(tiles < (1ll << 31), CULLAVO_EINVAL, "matrix too large");
  transpose16_k<<<(unsigned)tiles, 256, 0, CV_STREAM(stream)>>>((const u16*)src, ld_src, (u16*)dst, ld_dst, rows,
                                                                cols, tiles_c);
  return cullavo_check_launch("transpose16");
}
