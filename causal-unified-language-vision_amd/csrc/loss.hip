// Shifted, attention-masked cross entropy of CuLLaVOModel.forward
// (reference cullavo/arch_cullavo.py:651-665): targets = labels[..., 1:] kept where
// attention_mask[..., 1:] != 0, nn.CrossEntropyLoss(ignore_index=-100, reduction='mean') over
// the f32-upcast logits (transformers 4.37 LlamaForCausalLM upcasts logits to f32).
// One block per logits row; f32 online max / sum-exp over the bf16 row (HBM-bound).
#include "common.h"

namespace {

__global__ void shift_targets_k(const int64_t* __restrict__ labels, const int64_t* __restrict__ mask, int B,
                                int L, int64_t ignore, int64_t* __restrict__ tgt) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= (int64_t)B * L) return;
  const int t = (int)(r % L);
  int64_t v = ignore;
  if (t + 1 < L && (mask == nullptr || mask[r + 1] != 0)) v = labels[r + 1];
  tgt[r] = v;
}

template <typename T>
__global__ __launch_bounds__(256) void ce_fwd_k(const T* __restrict__ logits, int64_t ldl,
                                                const int64_t* __restrict__ tgt, int64_t V,
                                                int64_t ignore, float* __restrict__ row_loss,
                                                float* __restrict__ row_lse) {
  __shared__ float sm[4], ss[4];
  const int64_t r = blockIdx.x;
  const int64_t t = tgt[r];
  const T* x = logits + r * ldl;
  float m = -INFINITY, s = 0.f;
  const int64_t nv = V / 8;
  for (int64_t i = threadIdx.x; i < nv; i += 256) {
    float v[8];
    load8(x + i * 8, v);
    float bm = v[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) bm = fmaxf(bm, v[j]);
    const float nm = fmaxf(m, bm);
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += __expf(v[j] - nm);
    s = s * __expf(m - nm) + acc;
    m = nm;
  }
  for (int64_t i = nv * 8 + threadIdx.x; i < V; i += 256) {  // tail
    const float v = Elt<T>::ld(x, i);
    const float nm = fmaxf(m, v);
    s = s * __expf(m - nm) + __expf(v - nm);
    m = nm;
  }
  // wave then block combine of (m, s)
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const float om = __shfl_xor(m, o, 64), os = __shfl_xor(s, o, 64);
    const float nm = fmaxf(m, om);
    s = (nm == -INFINITY) ? 0.f : s * __expf(m - nm) + os * __expf(om - nm);
    m = nm;
  }
  if ((threadIdx.x & 63) == 0) { sm[threadIdx.x >> 6] = m; ss[threadIdx.x >> 6] = s; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = sm[0], Ssum = ss[0];
    for (int w = 1; w < 4; ++w) {
      const float nm = fmaxf(M, sm[w]);
      Ssum = Ssum * __expf(M - nm) + ss[w] * __expf(sm[w] - nm);
      M = nm;
    }
    const float lse = M + logf(Ssum);
    row_lse[r] = lse;
    row_loss[r] = (t == ignore || t < 0 || t >= V) ? 0.f : lse - Elt<T>::ld(x, t);
  }
}

// single block: deterministic fixed-order sum of the per-row losses and the valid count
__global__ __launch_bounds__(1024) void ce_reduce_k(const float* __restrict__ row_loss,
                                                    const int64_t* __restrict__ tgt, int64_t rows,
                                                    int64_t ignore, float* __restrict__ out) {
  __shared__ double red[16];
  __shared__ double redc[16];
  double s = 0.0, c = 0.0;
  for (int64_t r = threadIdx.x; r < rows; r += 1024) {
    if (tgt[r] != ignore) { s += row_loss[r]; c += 1.0; }
  }
  s = wave_sum_d(s);
  c = wave_sum_d(c);
  if ((threadIdx.x & 63) == 0) { red[threadIdx.x >> 6] = s; redc[threadIdx.x >> 6] = c; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double S = 0.0, C = 0.0;
    for (int w = 0; w < 16; ++w) { S += red[w]; C += redc[w]; }
    out[0] = (float)(S / C);  // 0/0 -> NaN like nn.CrossEntropyLoss on an empty selection
    out[1] = (float)C;
    out[2] = (float)(1.0 / C);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void ce_bwd_k(const T* __restrict__ logits, int64_t ldl,
                                                const int64_t* __restrict__ tgt,
                                                const float* __restrict__ lse,
                                                const float* __restrict__ loss_out,
                                                const float* __restrict__ gl, int64_t V, int64_t ignore,
                                                T* __restrict__ d, int64_t ldd) {
  const int64_t r = blockIdx.x;
  const int64_t t = tgt[r];
  const bool valid = !(t == ignore || t < 0 || t >= V);
  const float scale = valid ? (gl ? gl[0] : 1.f) * loss_out[2] : 0.f;
  const float l = lse[r];
  const T* x = logits + r * ldl;
  T* dr = d + r * ldd;
  const int64_t nv = V / 8;
  for (int64_t i = threadIdx.x; i < nv; i += 256) {
    float v[8], o[8];
    load8(x + i * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int64_t col = i * 8 + j;
      o[j] = (__expf(v[j] - l) - (col == t ? 1.f : 0.f)) * scale;
    }
    store8(dr + i * 8, o);
  }
  for (int64_t i = nv * 8 + threadIdx.x; i < V; i += 256) {
    const float v = Elt<T>::ld(x, i);
    Elt<T>::st(dr, i, (__expf(v - l) - (i == t ? 1.f : 0.f)) * scale);
  }
}

}  // namespace

extern "C" int cullavo_shift_targets(const int64_t* labels, const int64_t* mask, int B, int L,
                                     int64_t ignore_index, int64_t* targets, void* stream) {
  const int64_t n = (int64_t)B * L;
  if (n == 0) return CULLAVO_OK;
  shift_targets_k<<<(unsigned)cdiv(n, 256), 256, 0, CV_STREAM(stream)>>>(labels, mask, B, L, ignore_index, targets);
  return cullavo_check_launch("shift_targets");
}

extern "C" int cullavo_ce_fwd(const void* logits, int64_t ldl, const int64_t* targets, int64_t rows,
                              int64_t V, int64_t ignore_index, float* row_loss, float* row_lse, int dtype,
                              void* stream) {
  CV_REQUIRE(ldl % 8 == 0 && ldl >= V, CULLAVO_EINVAL, "ldl must be a multiple of 8 and >= V");
  if (rows == 0) return CULLAVO_OK;
  hipStream_t s = CV_STREAM(stream);
  if (dtype == CULLAVO_DT_BF16) ce_fwd_k<u16><<<(unsigned)rows, 256, 0, s>>>((const u16*)logits, ldl, targets, V, ignore_index, row_loss, row_lse);
  else if (dtype == CULLAVO_DT_F32) ce_fwd_k<float><<<(unsigned)rows, 256, 0, s>>>((const float*)logits, ldl, targets, V, ignore_index, row_loss, row_lse);
  else CV_REQUIRE(false, CULLAVO_EUNSUPPORTED, "dtype");
  return cullavo_check_launch("ce_fwd");
}

extern "C" int cullavo_ce_reduce(const float* row_loss, const int64_t* targets, int64_t rows,
                                 int64_t ignore_index, float* loss_out, void* stream) {
  ce_reduce_k<<<1, 1024, 0, CV_STREAM(stream)>>>(row_loss, targets, rows, ignore_index, loss_out);
  return cullavo_check_launch("ce_reduce");
}

extern "C" int cullavo_ce_bwd(const void* logits, int64_t ldl, const int64_t* targets, const float* row_lse,
                              const float* loss_out, const float* grad_loss, int64_t rows, int64_t V,
                              int64_t ignore_index, void* dlogits, int64_t ldd, int dtype, void* stream) {
  CV_REQUIRE(ldl % 8 == 0 && ldd % 8 == 0, CULLAVO_EINVAL, "row strides must be multiples of 8");
  if (rows == 0) return CULLAVO_OK;
  hipStream_t s = CV_STREAM(stream);
  if (dtype == CULLAVO_DT_BF16) ce_bwd_k<u16><<<(unsigned)rows, 256, 0, s>>>((const u16*)logits, ldl, targets, row_lse, loss_out, grad_loss, V, ignore_index, (u16*)dlogits, ldd);
  else if (dtype == CULLAVO_DT_F32) ce_bwd_k<float><<<(unsigned)rows, 256, 0, s>>>((const float*)logits, ldl, targets, row_lse, loss_out, grad_loss, V, ignore_index, (float*)dlogits, ldd);
  else CV_REQUIRE(false, CULLAVO_EUNSUPPORTED, "dtype");
  return cullavo_check_launch("ce_bwd");
}
